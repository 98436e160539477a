#!/bin/bash
# GPU box (round 5): k_extend with a 32-column LDS ring (17.7 KB per wave: 8 waves per CU instead of 6; wider windows
# overflow to the retry pass) -- lone-launch C3 (2 rounds) and C4 (1) against the in-tree build, with checksums.
tag=${1:-extr32}
mkdir -p gpurun_out/$tag
bash tools/ab_libs.sh $tag c3 1 2 tools/bin/libbsq_r32.so && bash tools/ab_libs.sh $tag c4 1 1 tools/bin/libbsq_r32.so
for v in base r32; do
  if [ $v = base ]; then unset BSQ_LIB; else export BSQ_LIB=$PWD/tools/bin/libbsq_r32.so; fi
  timeout -k 10 300 python -u bench.py --timed-only --checksums > gpurun_out/$tag/ck_$v.json 2>> gpurun_out/$tag/ck.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$tag/ck_$v.json')); print('c3 $v', d['value'], d['ms_per_step'], d['checksums'], d.get('retried_reads'))"
done
