#!/bin/bash
# GPU box (round 5): k-mer table depth below the default at C2 / C3 (is the Infinity Cache the limit?), two rounds.
tag=${1:-kmer2}
mkdir -p gpurun_out/$tag
for rep in 1 2; do for k in 9 10 11; do
  BSQ_KMER_K=$k timeout -k 10 300 python -u bench.py --config c2 --timed-only > gpurun_out/$tag/c2k${k}_$rep.json 2>> gpurun_out/$tag/ab.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$tag/c2k${k}_$rep.json')); print('c2 K=$k', d['value'], d['ms_per_step'])"
  BSQ_KMER_K=$k timeout -k 10 300 python -u bench.py --timed-only > gpurun_out/$tag/c3k${k}_$rep.json 2>> gpurun_out/$tag/ab.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$tag/c3k${k}_$rep.json')); print('c3 K=$k', d['value'], d['ms_per_step'])"
done; done
