#!/bin/bash
# GPU box (round 6): the 15-level k-mer table for 64-bit rows as the default -- the k-mer-depth and C4 parity tests
# (incl. the C4 replicated group: two index copies on one GPU), then the full C4 bench line.
set -o pipefail
tag=${1:-r06t}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_c4.py > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config c4 > $out/bench_c4.json 2> $out/bench_c4.err || exit 1
python3 -c "import json; d=json.load(open('$out/bench_c4.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('value_sql_call'), d.get('parity_sample'))"
