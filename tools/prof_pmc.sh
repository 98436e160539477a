#!/bin/bash
# Usage (GPU box, repo root): bash tools/prof_pmc.sh <tag> <counter file> [bench args...]
# Lists the available counters, then collects the PMC passes of <counter file> (kernel-trace only).
set -e
tag=$1; shift; cf=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/$tag
rocprofv3 -L > gpurun_out/$tag/counters_list.txt 2>&1 || true
timeout -k 10 600 rocprofv3 -i $cf --kernel-trace --output-format csv -d gpurun_out/$tag -o pmc -- python3 bench.py --no-cpu-baseline "$@" > gpurun_out/$tag/run.log 2>&1
