#!/bin/bash
# GPU box (round 5): pooled pipeline workspaces -- pipeline / drop-in / group tests, the C3 cursor twice, the C4 line.
tag=${1:-r05h}
mkdir -p gpurun_out/$tag
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pipeline.py tests/test_pg_extension.py tests/test_gpu_sql.py tests/test_pg_shim.py tests/test_gpu_render.py tests/test_gpu_group.py tests/test_gpu_group_bench.py tests/test_gpu_configs.py > gpurun_out/$tag/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$tag/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --cursor-only > gpurun_out/$tag/c_$rep.json 2> gpurun_out/$tag/c_$rep.err || exit 1
  python3 -c "import json; s=json.load(open('gpurun_out/$tag/c_$rep.json'))['sql_cursor']; print('cursor', s['reads_per_s_with_columns'], s['reads_per_s_records_only'], s['copy_staging_reads_per_s_with_columns'])"
done
timeout -k 10 700 python3 -u bench.py --config c4 > gpurun_out/$tag/c4.json 2> gpurun_out/$tag/c4.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/$tag/c4.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_sample'), d.get('sa_certificate'), d['sql_cursor'])"
