#!/bin/bash
# smem experiments: grid sweep for the flat kernel + SQ counters for both kernels (GPU box, repo root)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/sx
for b in 256 512 1024 4000; do BSQ_SMEM_BLOCKS=$b timeout -k 10 200 python bench.py --no-cpu-baseline --reads 400000 --steps 2 --warmup 1 > gpurun_out/sx/blocks_$b.json; done
timeout -k 10 300 rocprofv3 -i tools/pmc_sq.txt --kernel-trace --output-format csv -d gpurun_out/sx/flat -o pmc -- python3 bench.py --no-cpu-baseline --reads 200000 --steps 1 --warmup 0 > gpurun_out/sx/flat.log 2>&1
BSQ_SMEM=lds timeout -k 10 300 rocprofv3 -i tools/pmc_sq.txt --kernel-trace --output-format csv -d gpurun_out/sx/lds -o pmc -- python3 bench.py --no-cpu-baseline --reads 200000 --steps 1 --warmup 0 > gpurun_out/sx/lds.log 2>&1
