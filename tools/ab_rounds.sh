#!/bin/bash
# GPU box: C3 timed step, one stream of batch runs (default) vs a barrier after every step (--lockstep), alternated.
#   bash tools/ab_rounds.sh <tag> [steps]
set -e
tag=$1; k=${2:-20}; out=gpurun_out/$tag; mkdir -p $out
for rep in 1 2; do
  for m in rounds lockstep; do
    f=""; [ $m = lockstep ] && f="--lockstep"
    timeout -k 10 300 python3 bench.py --timed-only --steps $k --warmup 2 $f > $out/$m$rep.json 2> $out/$m$rep.err
    python3 -c "import json; d=json.loads(open('$out/$m$rep.json').read().strip().splitlines()[-1]); print('$m', d['value'], d['ms_per_step'], d['stages_ms'])"
  done
done
