#!/bin/bash
# GPU box (round 5): k-mer table depth (BSQ_KMER_K) -- seeding/parity tests at K = 13, then C2 seeding and C3 timed
# steps (full-batch checksum) at K = 11..14, two rounds.
tag=${1:-kmer}
mkdir -p gpurun_out/$tag
BSQ_KMER_K=13 timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_seeding.py tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_configs.py > gpurun_out/$tag/tests_k13.log 2>&1
rc=$?; tail -3 gpurun_out/$tag/tests_k13.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for k in 11 12 13 14; do
  BSQ_KMER_K=$k timeout -k 10 300 python -u bench.py --config c2 --timed-only > gpurun_out/$tag/c2k${k}_$rep.json 2>> gpurun_out/$tag/ab.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$tag/c2k${k}_$rep.json')); print('c2 K=$k', d['value'], d['ms_per_step'], d['index_build_s'])"
  BSQ_KMER_K=$k timeout -k 10 300 python -u bench.py --timed-only --checksums > gpurun_out/$tag/c3k${k}_$rep.json 2>> gpurun_out/$tag/ab.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$tag/c3k${k}_$rep.json')); print('c3 K=$k', d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['checksums'])"
done; done
