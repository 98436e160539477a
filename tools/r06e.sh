#!/bin/bash
# GPU box (round 6): the whole GPU suite on the compact k-mer table, then its A/B (tools/kc_ab.sh).
tag=${1:-r06e}
mkdir -p gpurun_out/$tag
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/$tag/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$tag/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/kc_ab.sh $tag > gpurun_out/$tag/kc_ab.txt 2>&1; cat gpurun_out/$tag/kc_ab.txt
