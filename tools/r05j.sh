#!/bin/bash
# GPU box (round 5): C4 with the depth-13 k-mer table by default -- the C4 GPU tests, then the C4 line and its lone
# rocprof stats.
tag=${1:-r05j}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_c4.py > gpurun_out/$tag/tests_c4.log 2>&1
rc=$?; tail -3 gpurun_out/$tag/tests_c4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python3 -u bench.py --config c4 > gpurun_out/$tag/c4.json 2> gpurun_out/$tag/c4.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/$tag/c4.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d.get('parity_sample'), d['sql_cursor']['reads_per_s_with_columns'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/trace1 -o kt -- python3 bench.py --config c4 --timed-only --streams 1 --steps 1 --warmup 1 > gpurun_out/$tag/trace1.json 2> gpurun_out/$tag/trace1.log
echo done
