#!/bin/bash
# GPU box (round 6): the GPU suite with the query base carried in the extension ring's words, then lone C3 launches
# against the previous library (exp/libbsq_base.so) and the C3 step, alternating.
tag=${1:-r06g}
mkdir -p gpurun_out/$tag
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/$tag/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$tag/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_lib.sh $tag/lone exp/libbsq_base.so c3 3 > gpurun_out/$tag/lone_ab.txt 2>&1 || exit 1
cat gpurun_out/$tag/lone_ab.txt
for rep in 1 2; do
  for v in base exp; do
    if [ $v = exp ]; then export BSQ_LIB=exp/libbsq_base.so; else unset BSQ_LIB; fi
    timeout -k 10 300 python bench.py --timed-only --checksums > gpurun_out/$tag/step_${v}_$rep.json 2> gpurun_out/$tag/step_${v}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/$tag/step_${v}_$rep.json')); print('$v', d['value'], d['ms_per_step'], d['checksums'])"
  done
done
