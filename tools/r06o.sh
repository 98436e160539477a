#!/bin/bash
# GPU box (round 6; the experiment is profiles/r06/quad/quad.patch, reverted): backward list entries extended four per trip (BSQ_SMEM_QUAD=1: up to eight rank blocks in flight,
# 160 / 200 VGPRs -> 12 / 8 waves per CU for u32 / 64-bit rows) -- seeding parity with it on, then the C3 and C4 step
# A/B (timed, checksums), alternating; BSQ_TEST_LCAP sizes the LDS list share to the lower occupancy.
tag=${1:-r06o}; out=gpurun_out/$tag; mkdir -p $out
BSQ_SMEM_QUAD=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_c4.py -k "parity or seeding or golden or wide or kmer or spill" > $out/tests_quad.log 2>&1
rc=$?; tail -3 $out/tests_quad.log; [ $rc -eq 0 ] || exit $rc
run() {   # name cfg env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 500 python bench.py --config $cfg --timed-only --checksums > $out/$name.json 2> $out/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', d['value'], d['ms_per_step'], d['checksums'], {k: round(v, 2) for k, v in d['stages_ms'].items()})"
}
for rep in 1 2; do
  run c3_p2_$rep c3 BSQ_SMEM_QUAD=0
  run c3_p4_$rep c3 BSQ_SMEM_QUAD=1
  run c3_p4l21_$rep c3 BSQ_SMEM_QUAD=1 BSQ_TEST_LCAP=21
done
for rep in 1 2; do
  run c4_p2_$rep c4 BSQ_SMEM_QUAD=0
  run c4_p4l22_$rep c4 BSQ_SMEM_QUAD=1 BSQ_TEST_LCAP=22
done
