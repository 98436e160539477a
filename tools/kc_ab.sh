#!/bin/bash
# GPU box (round 6): the compact k-mer table A/B -- the C3 step (4 batches, 20 steps, checksums) and C2 seeding, two
# alternating rounds over: 16-B entries at depth 10 (the round-5 default), compact at depth 10, 11 (default), 12.
#   bash tools/kc_ab.sh <tag>
tag=$1; out=gpurun_out/$tag; mkdir -p $out
run() {   # name, env...
  local nm=$1; shift
  for cfg in c3 c2; do
    env "$@" timeout -k 10 300 python bench.py --config $cfg --timed-only --checksums > $out/${nm}_${cfg}_$rep.json 2> $out/${nm}_${cfg}_$rep.err || return 1
    python3 -c "import json; d=json.load(open('$out/${nm}_${cfg}_$rep.json')); print('$nm', '$cfg', d['value'], d['ms_per_step'], d.get('checksums'), {k: round(v, 3) for k, v in d['stages_ms'].items()})"
  done
}
for rep in 1 2; do
  run full10 BSQ_KMER_COMPACT=0 || exit 1
  run kc11 BSQ_KMER_K=11 || exit 1
  run kc12 BSQ_KMER_K=12 || exit 1
  run kc10 BSQ_KMER_K=10 || exit 1
done
