#!/bin/bash
# GPU box: pipeline / drop-in tests, then the cursor loop (traced once, then two plain runs).
tag=${1:-curc}
mkdir -p gpurun_out/$tag
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pipeline.py tests/test_pg_extension.py tests/test_gpu_sql.py tests/test_pg_shim.py tests/test_gpu_render.py > gpurun_out/$tag/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$tag/tests.log; [ $rc -eq 0 ] || exit $rc
BSQ_PIPE_TRACE=1 timeout -k 10 300 python -u bench.py --cursor-only > gpurun_out/$tag/trace.json 2> gpurun_out/$tag/trace.err || exit 1
python3 -c "import json; s=json.load(open('gpurun_out/$tag/trace.json'))['sql_cursor']; print('traced', s['reads_per_s_with_columns'], s['reads_per_s_records_only'], s['copy_staging_reads_per_s_with_columns'])"
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --cursor-only > gpurun_out/$tag/c_$rep.json 2> gpurun_out/$tag/c_$rep.err || exit 1
  python3 -c "import json; s=json.load(open('gpurun_out/$tag/c_$rep.json'))['sql_cursor']; print('cursor', s['reads_per_s_with_columns'], s['reads_per_s_records_only'], s['copy_staging_reads_per_s_with_columns'])"
done
