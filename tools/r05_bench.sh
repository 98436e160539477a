#!/bin/bash
# GPU box: the default bench line (C3) plus the given extra test files; outputs under gpurun_out/<tag>.
#   bash tools/r05_bench.sh <tag> [test files...]
tag=${1:-r05}; shift
mkdir -p gpurun_out/$tag
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/$tag/tests.log 2>&1
  rc=$?; tail -15 gpurun_out/$tag/tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python -u bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
rc=$?; tail -3 gpurun_out/$tag/bench.err; exit $rc
