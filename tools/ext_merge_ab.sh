#!/bin/bash
# GPU box (round 5): one loop over a seed's left and right extensions (one ksw_extend2 call site; experiment build
# tools/bin/libbsq_merge.so) -- alignment tests on it, lone-launch C3 (2 rounds) and C4 (1) against the in-tree build,
# then the C3 step with full-batch checksums for both.
tag=${1:-extmerge}
mkdir -p gpurun_out/$tag
BSQ_LIB=$PWD/tools/bin/libbsq_merge.so timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_configs.py tests/test_gpu_long_reads.py tests/test_gpu_c4.py > gpurun_out/$tag/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$tag/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh $tag c3 1 2 tools/bin/libbsq_merge.so && bash tools/ab_libs.sh $tag c4 1 1 tools/bin/libbsq_merge.so || exit 1
for v in base merge; do
  if [ $v = base ]; then unset BSQ_LIB; else export BSQ_LIB=$PWD/tools/bin/libbsq_merge.so; fi
  timeout -k 10 300 python -u bench.py --timed-only --checksums > gpurun_out/$tag/ck_$v.json 2>> gpurun_out/$tag/ck.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$tag/ck_$v.json')); print('c3 $v', d['value'], d['ms_per_step'], d['checksums'], d.get('retried_reads'))"
done
