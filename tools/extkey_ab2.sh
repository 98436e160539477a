#!/bin/bash
# GPU box (round 5): extension sort key: kind + longer extent (new) vs sides + left extent (tools/bin/libbsq_k1.so) -- alignment tests on the new
# library, then C3 / C2 (full-batch checksums) alternating with the previous build (BSQ_LIB=tools/bin/libbsq_k1.so),
# two rounds, and C4 once each.
tag=${1:-extkey}
mkdir -p gpurun_out/$tag
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_configs.py tests/test_gpu_pipeline.py > gpurun_out/$tag/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$tag/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in k1 new; do
  if [ $v = k1 ]; then export BSQ_LIB=$PWD/tools/bin/libbsq_k1.so; else unset BSQ_LIB; fi
  timeout -k 10 300 python -u bench.py --timed-only --checksums > gpurun_out/$tag/c3_${v}_$rep.json 2>> gpurun_out/$tag/ab.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$tag/c3_${v}_$rep.json')); print('c3 $v', d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['checksums'])"
done; done
for v in k1 new; do
  if [ $v = k1 ]; then export BSQ_LIB=$PWD/tools/bin/libbsq_k1.so; else unset BSQ_LIB; fi
  timeout -k 10 600 python -u bench.py --config c4 --timed-only --checksums > gpurun_out/$tag/c4_${v}.json 2>> gpurun_out/$tag/ab.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$tag/c4_${v}.json')); print('c4 $v', d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['checksums'])"
done
