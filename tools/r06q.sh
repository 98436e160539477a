#!/bin/bash
# GPU box (round 6; experiment profiles/r06/sort_path/onesweep.patch, reverted): the lane-balance sorts through rocprim's Onesweep path instead of its block + merge-sort path
# (bsq_api.cpp sort_keys; BSQ_SORT_MERGE=1 = the previous path) -- parity, then A/B: the C3 step with checksums and
# lone C3 launches, alternating.
tag=${1:-r06q}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py -k "parity or all_columns or option or lrand48" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
run() {   # name merge cfg extra...
  local name=$1 m=$2 cfg=$3; shift 3
  BSQ_SORT_MERGE=$m timeout -k 10 500 python bench.py --config $cfg --timed-only --checksums "$@" > $out/$name.json 2> $out/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', d['value'], d['ms_per_step'], d['checksums'], {k: round(v, 3) for k, v in d['stages_ms'].items()})"
}
for rep in 1 2 3; do
  run c3_onesweep_$rep 0 c3
  run c3_merge_$rep 1 c3
done
for rep in 1 2; do
  run c3lone_onesweep_$rep 0 c3 --streams 1
  run c3lone_merge_$rep 1 c3 --streams 1
done
