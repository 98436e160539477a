#!/bin/bash
# GPU box: step-level A/B of seeding occupancy settings (co-residency with the DP stages of the other batches):
# env settings given as arguments, each run twice in alternation, C3 timed steps only.
#   bash tools/ab_cores.sh <tag> "ENV=.. ENV2=.." "..." ...
tag=$1; shift
mkdir -p gpurun_out/$tag
for rep in 1 2; do
  k=0
  for setting in "$@"; do
    env $setting timeout -k 10 200 python -u bench.py --timed-only > gpurun_out/$tag/v${k}_$rep.json 2>> gpurun_out/$tag/err.log || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/$tag/v${k}_$rep.json')); print('$setting', 'rep $rep', d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()})"
    k=$((k+1))
  done
done
