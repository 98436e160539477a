#!/bin/bash
set -e
mkdir -p gpurun_out/lc2
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/lc2/parity.log 2>&1
for c in 20 16 15; do BSQ_LCAP=$c timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/lc2/l$c.json 2>/dev/null; done
