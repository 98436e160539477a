#!/bin/bash
# GPU box: the step at several batch counts, alternating (C3, timed steps only).  bash tools/ab_streams2.sh <tag> <reps> <S>...
tag=$1; reps=$2; shift 2; out=gpurun_out/$tag; mkdir -p $out
for rep in $(seq 1 $reps); do
  for s in "$@"; do
    timeout -k 10 300 python bench.py --timed-only --streams $s --steps 20 --warmup 3 > $out/s${s}_$rep.json 2> $out/s${s}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$out/s${s}_$rep.json')); print('S=$s', d['value'], d['ms_per_step'])"
  done
done
