#!/bin/bash
# GPU box: kernel + memory-copy timeline of the pipelined cursor (bench.py --cursor-only), for the drop-in loop.
#   bash tools/cursor_probe.sh <tag>
set -e
export TMPDIR=/tmp
tag=$1; out=gpurun_out/$tag; mkdir -p $out
BSQ_PIPE_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $out/cur -o cur -- python3 bench.py --cursor-only --steps 1 --warmup 1 > $out/cur.json 2> $out/cur.err
echo done
