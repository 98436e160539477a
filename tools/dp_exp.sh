#!/bin/bash
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/dx
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/dx/bench.json
timeout -k 10 400 rocprofv3 -i tools/pmc_dp.txt --kernel-trace --output-format csv -d gpurun_out/dx/pmc -o pmc -- python3 bench.py --no-cpu-baseline --reads 200000 --steps 1 --warmup 0 > gpurun_out/dx/pmc.log 2>&1
