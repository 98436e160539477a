#!/bin/bash
# GPU box (round 6; experiment profiles/r06/ss_pair/ss_pair.patch, reverted): the seed-strategy pass two calls at a time (BSQ_SS_PAIR=1: the next call started where the
# current one usually returns, kept only if it did) -- seeding parity with it on, then A/B against the previous build
# (exp/libbsq_head.so): lone C2 seeding (head / pair / the new build without the pair), the C3 and C4 steps.
tag=${1:-r06x}; out=gpurun_out/$tag; mkdir -p $out
BSQ_SS_PAIR=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_c4.py -k "parity or seeding or option or c3_100mbp_all or c4_3gbp_all" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
run() {   # name cfg lib pair extra...
  local name=$1 cfg=$2 lib=$3 pr=$4; shift 4
  if [ -n "$lib" ]; then export BSQ_LIB=$lib; else unset BSQ_LIB; fi
  BSQ_SS_PAIR=$pr timeout -k 10 500 python bench.py --config $cfg --timed-only --checksums "$@" > $out/$name.json 2> $out/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', d['value'], d['ms_per_step'], d['checksums'], {k: round(v, 3) for k, v in d['stages_ms'].items()})"
}
for rep in 1 2; do
  run c2_head_$rep c2 exp/libbsq_head.so 0 --streams 1
  run c2_pair_$rep c2 "" 1 --streams 1
  run c2_nopair_$rep c2 "" 0 --streams 1
done
for rep in 1 2; do
  run c3_head_$rep c3 exp/libbsq_head.so 0
  run c3_pair_$rep c3 "" 1
done
for rep in 1 2; do
  run c4_head_$rep c4 exp/libbsq_head.so 0
  run c4_pair_$rep c4 "" 1
done
