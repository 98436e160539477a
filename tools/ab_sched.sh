#!/bin/bash
# GPU box: A/B of the extension / whole-wave CIGAR work counters against their fixed-stride schedules (env knobs),
# alternating, C3 bench lines.   bash tools/ab_sched.sh <tag> <streams> <reps>
tag=$1; ns=${2:-1}; reps=${3:-2}; out=gpurun_out/$tag; mkdir -p $out
for rep in $(seq 1 $reps); do
  for v in static dynamic; do
    if [ $v = static ]; then export BSQ_EXT_STATIC=1 BSQ_R2A_STATIC=1; else unset BSQ_EXT_STATIC BSQ_R2A_STATIC; fi
    timeout -k 10 300 python bench.py --timed-only --streams $ns --steps 20 --warmup 3 > $out/${v}_s${ns}_$rep.json 2> $out/${v}_s${ns}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$out/${v}_s${ns}_$rep.json')); print('$v s$ns', d['value'], d['ms_per_step'], d['stages_ms'])"
  done
done
