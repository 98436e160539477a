#!/bin/bash
# GPU box: parity tests, then the default bench (no CPU baseline unless $FULL is set).
set -e
tag=${1:-chk}
mkdir -p gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$tag/gputests.log 2>&1 || { tail -30 gpurun_out/$tag/gputests.log; exit 1; }
tail -2 gpurun_out/$tag/gputests.log
if [ -n "$FULL" ]; then extra=""; else extra="--no-cpu-baseline"; fi
timeout -k 10 300 python bench.py $extra > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
python -c "import json; d=json.load(open('gpurun_out/$tag/bench.json')); print(d['value'], d['stages_ms'], d.get('parity_sample'))"
