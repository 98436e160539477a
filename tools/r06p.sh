#!/bin/bash
# GPU box (round 6; experiment profiles/r06/ss_walk/ss_unique_walk.patch, reverted): the seed-strategy pass walks a
# unique interval along the text (smem.hip seed_strategy1_x) --
# seeding / alignment parity on the in-tree build, then A/B against the previous build (exp/libbsq_base.so): lone C2
# seeding, the C3 and C4 steps with checksums, alternating.
tag=${1:-r06p}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_c4.py -k "parity or seeding or option or all_columns" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_lib.sh $tag/c2 exp/libbsq_base.so c2 2 || exit 1
run() {   # name cfg lib
  local name=$1 cfg=$2 lib=$3
  if [ -n "$lib" ]; then export BSQ_LIB=$lib; else unset BSQ_LIB; fi
  timeout -k 10 500 python bench.py --config $cfg --timed-only --checksums > $out/$name.json 2> $out/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', d['value'], d['ms_per_step'], d['checksums'], {k: round(v, 2) for k, v in d['stages_ms'].items()})"
}
for rep in 1 2; do
  run c3_new_$rep c3
  run c3_old_$rep c3 exp/libbsq_base.so
done
for rep in 1 2; do
  run c4_new_$rep c4
  run c4_old_$rep c4 exp/libbsq_base.so
done
