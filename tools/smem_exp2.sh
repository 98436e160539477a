#!/bin/bash
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/sx2
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/sx2/parity.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/sx2/flat.json
BSQ_SMEM=lds timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/sx2/lds.json
timeout -k 10 300 rocprofv3 -i tools/pmc_sq.txt --kernel-trace --output-format csv -d gpurun_out/sx2/flatpmc -o pmc -- python3 bench.py --no-cpu-baseline --reads 200000 --steps 1 --warmup 0 > gpurun_out/sx2/flatpmc.log 2>&1
