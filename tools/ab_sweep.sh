#!/bin/bash
# GPU box: sweep an environment knob over several values (two passes), stage times from the bench line.
#   bash tools/ab_sweep.sh <tag> <VAR> "<v1> <v2> ..." [config] [streams]
tag=$1; var=$2; vals=$3; cfg=${4:-c3}; ns=${5:-1}; out=gpurun_out/$tag; mkdir -p $out
for rep in 1 2; do
  for v in $vals; do
    env $var=$v timeout -k 10 300 python bench.py --config $cfg --timed-only --streams $ns --steps ${STEPS:-3} --warmup 1 > $out/ab_${v}_$rep.json 2> $out/ab_${v}_$rep.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$out/ab_${v}_$rep.json')); print('$var=$v', d['value'], d['ms_per_step'], d['stages_ms'])"
  done
done
