#!/bin/bash
# GPU box (round 6): the whole -m gpu suite, then the default bench line (C3) -- the round's checkpoint.
#   bash tools/r06_check.sh <tag> [bench args...]
tag=${1:-r06a}; shift
mkdir -p gpurun_out/$tag
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/$tag/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$tag/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
rc=$?; cat gpurun_out/$tag/bench.json | head -c 1500; exit $rc
