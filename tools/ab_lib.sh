#!/bin/bash
# GPU box: A/B of an experiment build of libbsq (BSQ_LIB) against the in-tree one, lone launches (--streams 1),
# alternating, stage times from the bench line.   bash tools/ab_lib.sh <tag> <exp lib> [config] [reps] [extra args]
tag=$1; lib=$2; cfg=${3:-c3}; reps=${4:-2}; shift 4; extra="$@"; out=gpurun_out/$tag; mkdir -p $out
T=300; [ "$cfg" = c4 ] && T=600
for rep in $(seq 1 $reps); do
  for v in base exp; do
    if [ $v = exp ]; then export BSQ_LIB=$lib; else unset BSQ_LIB; fi
    timeout -k 10 $T python bench.py --config $cfg --timed-only --streams 1 --steps 2 --warmup 1 $extra > $out/ab_${v}_$rep.json 2> $out/ab_${v}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$out/ab_${v}_$rep.json')); print('$v', d['value'], d['ms_per_step'], d['stages_ms'])"
  done
done
