#!/bin/bash
# GPU box (round 5): extension sort key (sides and left extent) -- the whole -m gpu suite,
# then the final-tree profiling (tools/r05_final.sh).
tag=${1:-r05x}
mkdir -p gpurun_out/$tag
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/$tag/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$tag/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/r05_final.sh $tag
