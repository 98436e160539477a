#!/bin/bash
# GPU box: parity tests of the seeding paths, then A/B of the state-machine seeding kernel (BSQ_SMEM_SM=1) against
# k_smem_lds (0) on the timed steps of C2 and C3 (C3 with the full-batch checksums).  bash tools/sm_check.sh <tag> [tests]
tag=${1:-sm}; shift
mkdir -p gpurun_out/$tag
tests=${@:-tests/test_gpu_seeding.py tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_chain.py tests/test_gpu_configs.py::test_c2_100mbp_seeding tests/test_gpu_configs.py::test_c3_100mbp_all_columns}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $tests > gpurun_out/$tag/tests.log 2>&1
rc=$?; tail -25 gpurun_out/$tag/tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in c2 c3; do for sm in 1 0 1; do
  BSQ_SMEM_SM=$sm timeout -k 10 300 python -u bench.py --config $cfg --timed-only --checksums > gpurun_out/$tag/${cfg}_sm$sm.json 2>> gpurun_out/$tag/bench.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/$tag/${cfg}_sm$sm.json')); print('$cfg sm=$sm', d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d.get('checksums'))"
done; done
