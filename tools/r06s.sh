#!/bin/bash
# GPU box (round 6): C4 k-mer table depth 15 (46 GB of 32-B entries) against the default 13, with the 64-bit-row
# kernels preloading 13 levels (in-tree) or all 15 (exp/libbsq_km15.so) -- C4 seeding parity at depth 15 with the
# 15-level build, then the C4 step with checksums, alternating.
tag=${1:-r06s}; out=gpurun_out/$tag; mkdir -p $out
BSQ_LIB=exp/libbsq_km15.so BSQ_KMER_K=15 timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_c4.py -k "seeding or all_columns" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
run() {   # name lib K
  local name=$1 lib=$2 k=$3
  if [ -n "$lib" ]; then export BSQ_LIB=$lib; else unset BSQ_LIB; fi
  if [ -n "$k" ]; then export BSQ_KMER_K=$k; else unset BSQ_KMER_K; fi
  timeout -k 10 500 python bench.py --config c4 --timed-only --checksums > $out/$name.json 2> $out/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', d['value'], d['ms_per_step'], d['checksums'], {k: round(v, 2) for k, v in d['stages_ms'].items()})"
}
for rep in 1 2; do
  run k13_$rep "" ""
  run k15_$rep "" 15
  run k15pre_$rep exp/libbsq_km15.so 15
done
