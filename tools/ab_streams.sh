#!/bin/bash
# GPU box: C3 timed steps (stream of batch runs) at several batch counts, alternated twice.
#   bash tools/ab_streams.sh <tag> "<counts>" [steps]
set -e
tag=$1; counts=${2:-"3 4 6"}; k=${3:-20}; out=gpurun_out/$tag; mkdir -p $out
for rep in 1 2; do
  for s in $counts; do
    timeout -k 10 300 python3 bench.py --timed-only --steps $k --warmup 2 --streams $s > $out/s$s.$rep.json 2> $out/s$s.$rep.err
    python3 -c "import json; d=json.loads(open('$out/s$s.$rep.json').read().strip().splitlines()[-1]); print('streams $s', d['value'], d['ms_per_step'])"
  done
done
