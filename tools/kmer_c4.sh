#!/bin/bash
# GPU box (round 5): k-mer table depth at C4 (timed steps with the full-batch checksum), K = 11, 12, 13, 11.
tag=${1:-kmer4}
mkdir -p gpurun_out/$tag
for k in 11 12 13; do
  BSQ_KMER_K=$k timeout -k 10 600 python -u bench.py --config c4 --timed-only --checksums > gpurun_out/$tag/c4k$k.json 2>> gpurun_out/$tag/ab.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$tag/c4k$k.json')); print('c4 K=$k', d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['checksums'])"
done
