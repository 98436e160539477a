#!/bin/bash
# GPU box: the drop-in cursor loop (bench.py --cursor-only) over pipeline depth (fetches in flight), concurrent
# alignments (BSQ_PIPE_RUN) and HIP hardware queues (BSQ_HW_QUEUES -> GPU_MAX_HW_QUEUES), two rounds.
tag=${1:-cursw}
mkdir -p gpurun_out/$tag
if [ -n "$CURSOR_SWEEP" ]; then IFS=, read -ra CFGS <<< "$CURSOR_SWEEP"; else CFGS=("8 4 8" "16 6 8"); fi
for rep in 1 2; do for v in "${CFGS[@]}"; do set -- $v
  f=gpurun_out/$tag/d$1r$2q$3_$rep
  BSQ_HW_QUEUES=$3 BSQ_PIPE_RUN=$2 timeout -k 10 300 python -u bench.py --cursor-only --cursor-depth $1 > $f.json 2> $f.err || exit 1
  python3 -c "import json; d=json.load(open('$f.json')); s=d['sql_cursor']; print('depth $1 run $2 queues $3', s['reads_per_s_with_columns'], s['reads_per_s_records_only'], s['copy_staging_reads_per_s_with_columns'])"
done; done
