#!/bin/bash
# GPU box: run the given GPU test files (all of tests/ when none), one pytest process, 300 s per test.
#   bash tools/gpu_tests.sh <tag> [test files...]
tag=${1:-tests}; shift
mkdir -p gpurun_out/$tag
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${@:-tests} > gpurun_out/$tag/tests.log 2>&1
rc=$?
tail -40 gpurun_out/$tag/tests.log
exit $rc
