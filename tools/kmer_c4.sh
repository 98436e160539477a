#!/bin/bash
# GPU box (round 5): k-mer table depth at C4 (timed steps with the full-batch checksum) for K in $KLIST.
tag=${1:-kmer4}
mkdir -p gpurun_out/$tag
i=0
for k in ${KLIST:-11 12 13}; do
  i=$((i+1)); f=gpurun_out/$tag/c4k${k}_$i.json
  BSQ_KMER_K=$k timeout -k 10 600 python -u bench.py --config c4 --timed-only --checksums > $f 2>> gpurun_out/$tag/ab.err || exit 1
  python3 -c "import json; d=json.load(open('$f')); print('c4 K=$k', d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['checksums'], d['index_build_s'])"
done
