#!/bin/bash
set -e
mkdir -p gpurun_out/lc
for c in 28 24 20 18 16 14; do BSQ_LCAP=$c timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/lc/l$c.json 2>/dev/null; done
