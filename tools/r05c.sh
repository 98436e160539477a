#!/bin/bash
# GPU box (round 5): pipeline/drop-in tests; the seeding/parity tests with the new seeding variants switched on; the
# full bench line; then the A/B of persistent lanes (BSQ_SMEM_LANES) x the seed-strategy text walk (BSQ_SS_WALK):
# C3 timed steps with the full-batch checksum, and C2 (seeding only).
tag=${1:-r05c}
mkdir -p gpurun_out/$tag
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pipeline.py tests/test_pg_extension.py tests/test_gpu_sql.py tests/test_pg_shim.py > gpurun_out/$tag/tests.log 2>&1
rc=$?; tail -4 gpurun_out/$tag/tests.log; [ $rc -eq 0 ] || exit $rc
BSQ_SMEM_LANES=1 BSQ_SS_WALK=1 BSQ_SMEM_MERGE=1 timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_seeding.py tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_configs.py tests/test_gpu_chain.py > gpurun_out/$tag/tests_lanes.log 2>&1
rc=$?; tail -4 gpurun_out/$tag/tests_lanes.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/$tag/bench.json')); print(d['value'], d['ms_per_step'], d['sql_cursor'])"
for rep in 1 2; do for v in "0 0 0" "0 1 0" "0 0 1" "1 0 0" "1 1 1"; do set -- $v
  export BSQ_SMEM_LANES=$1 BSQ_SS_WALK=$2 BSQ_SMEM_MERGE=$3
  timeout -k 10 200 python -u bench.py --timed-only --checksums > gpurun_out/$tag/l$1w$2m$3_$rep.json 2>> gpurun_out/$tag/ab.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$tag/l$1w$2m$3_$rep.json')); print('c3 lanes=$1 walk=$2 merge=$3', d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['checksums'])"
  timeout -k 10 200 python -u bench.py --config c2 --timed-only > gpurun_out/$tag/c2l$1w$2m$3_$rep.json 2>> gpurun_out/$tag/ab.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$tag/c2l$1w$2m$3_$rep.json')); print('c2 lanes=$1 walk=$2 merge=$3', d['value'], d['ms_per_step'])"
done; done
