#!/bin/bash
# GPU box (round 6): the C3 step's concurrency on the final kernels -- concurrent batches (--streams) x HIP hardware
# queues (BSQ_HW_QUEUES), two alternating rounds, checksums.
tag=${1:-r06h}; out=gpurun_out/$tag; mkdir -p $out
for rep in 1 2; do
  for cfg in "4 8" "3 8" "5 8" "6 8" "4 4" "4 16" "6 16"; do
    set -- $cfg
    BSQ_HW_QUEUES=$2 timeout -k 10 300 python bench.py --timed-only --checksums --streams $1 > $out/s$1_q$2_$rep.json 2> $out/s$1_q$2_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$out/s$1_q$2_$rep.json')); print('streams $1 queues $2', d['value'], d['ms_per_step'], d['checksums'])"
  done
done
