#!/bin/bash
# GPU box (round 5): 13 preloaded k-mer levels for 64-bit rows -- C4 and wide-row tests, then C4 timed steps (full-batch
# checksum) alternating with the previous build (BSQ_LIB=tools/bin/libbsq_base.so), two rounds.
tag=${1:-km}
mkdir -p gpurun_out/$tag
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_c4.py tests/test_gpu_parity.py -k "c4 or wide or kmer" > gpurun_out/$tag/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$tag/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in base new; do
  if [ $v = base ]; then export BSQ_LIB=$PWD/tools/bin/libbsq_base.so; else unset BSQ_LIB; fi
  timeout -k 10 600 python -u bench.py --config c4 --timed-only --checksums > gpurun_out/$tag/c4_${v}_$rep.json 2>> gpurun_out/$tag/ab.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$tag/c4_${v}_$rep.json')); print('c4 $v', d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['checksums'])"
done; done
