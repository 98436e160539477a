#!/bin/bash
# GPU box (round 6; experiment profiles/r06/ss_split/ss_split.patch, reverted): the seed-strategy pass (and the sort) in a kernel of its own after the SMEM passes
# (BSQ_SS_SPLIT=1: k_seed_ss, 82 / 94 VGPRs, no LDS) -- seeding parity with it on, then A/B in one build: lone C2
# seeding, the C3 and C4 steps with checksums, alternating.
tag=${1:-r06y}; out=gpurun_out/$tag; mkdir -p $out
BSQ_SS_SPLIT=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_c4.py -k "parity or seeding or option or c3_100mbp_all or c4_3gbp_all" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
run() {   # name cfg split extra...
  local name=$1 cfg=$2 sp=$3; shift 3
  BSQ_SS_SPLIT=$sp timeout -k 10 500 python bench.py --config $cfg --timed-only "$@" > $out/$name.json 2> $out/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', d['value'], d['ms_per_step'], d.get('checksums'), {k: round(v, 3) for k, v in d['stages_ms'].items() if v})"
}
for rep in 1 2; do
  run c2_base_$rep c2 0 --streams 1
  run c2_split_$rep c2 1 --streams 1
done
for rep in 1 2; do
  run c3_base_$rep c3 0 --checksums
  run c3_split_$rep c3 1 --checksums
done
for rep in 1 2; do
  run c4_base_$rep c4 0 --checksums
  run c4_split_$rep c4 1 --checksums
done
