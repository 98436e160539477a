#!/bin/bash
# GPU box (round 6): 64-bit-row seeding with backward entries one per trip at 16 waves per CU (BSQ_WIDE_SINGLE=1) --
# the wide-row and C4 parity tests with it on, then the C4 step A/B (timed, checksums), alternating.
tag=${1:-r06n}; out=gpurun_out/$tag; mkdir -p $out
BSQ_WIDE_SINGLE=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_c4.py -k "wide or c4 or kmer" > $out/tests_single.log 2>&1
rc=$?; tail -3 $out/tests_single.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 0 1; do
    BSQ_WIDE_SINGLE=$v timeout -k 10 500 python bench.py --config c4 --timed-only --checksums > $out/c4_single${v}_$rep.json 2> $out/c4_single${v}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$out/c4_single${v}_$rep.json')); print('single=$v', d['value'], d['ms_per_step'], d['checksums'], {k: round(v, 2) for k, v in d['stages_ms'].items()})"
  done
done
