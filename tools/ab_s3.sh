#!/bin/bash
# GPU box: reg2aln diagonal pass A/B under rocprof (lone 1M-read launches) and the column-stream priority A/B
# of the pipelined cursor.   bash tools/ab_s3.sh <tag>
set -e
export TMPDIR=/tmp
tag=$1; out=gpurun_out/$tag; mkdir -p $out
for d in 1 0; do
  BSQ_R2A_DIAG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/diag$d -o kt -- python3 bench.py --timed-only --streams 1 --steps 2 --warmup 1 > $out/diag$d.json 2> $out/diag$d.log
done
for p in 1 0; do
  BSQ_COLS_PRIORITY=$p timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-codec > $out/prio$p.json 2> $out/prio$p.err
done
timeout -k 10 500 python3 bench.py --config c4 --timed-only --streams 1 --steps 2 --warmup 1 > $out/c4.json 2> $out/c4.err
echo done
