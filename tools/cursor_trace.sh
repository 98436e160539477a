#!/bin/bash
# GPU box: the drop-in cursor loop (bench.py --cursor-only) with the pipeline's per-job trace (BSQ_PIPE_TRACE),
# at the default depth and at deeper pipelines / more concurrent alignments.
tag=${1:-cur}
mkdir -p gpurun_out/$tag
BSQ_PIPE_TRACE=1 timeout -k 10 300 python -u bench.py --cursor-only > gpurun_out/$tag/d8.json 2> gpurun_out/$tag/d8.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/$tag/d8.json')); print('d8', d['sql_cursor'])"
for v in "12 4" "16 4" "8 6" "16 6"; do set -- $v
  BSQ_PIPE_RUN=$2 timeout -k 10 300 python -u bench.py --cursor-only --cursor-depth $1 > gpurun_out/$tag/d$1r$2.json 2> gpurun_out/$tag/d$1r$2.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$tag/d$1r$2.json')); s=d['sql_cursor']; print('depth $1 run $2', s['reads_per_s_with_columns'], s['reads_per_s_records_only'], s['copy_staging_reads_per_s_with_columns'])"
done
