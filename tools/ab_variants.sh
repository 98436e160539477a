#!/bin/bash
# GPU box: A/B of (library, environment) variants, alternating, stage times from the bench line.
#   bash tools/ab_variants.sh <tag> <config> <streams> <reps> "<name>:<lib or base>:<VAR=v,VAR=v or ->" ...
tag=$1; cfg=$2; ns=$3; reps=$4; shift 4; out=gpurun_out/$tag; mkdir -p $out
T=300; [ "$cfg" = c4 ] && T=600
for rep in $(seq 1 $reps); do
  for spec in "$@"; do
    IFS=: read -r n lib envs <<< "$spec"
    args=()
    [ "$lib" != base ] && args+=("BSQ_LIB=$lib")
    [ "$envs" != - ] && IFS=, read -ra ev <<< "$envs" && args+=("${ev[@]}")
    env "${args[@]}" timeout -k 10 $T python bench.py --config $cfg --timed-only --streams $ns --steps ${STEPS:-3} --warmup 1 > $out/${n}_$rep.json 2> $out/${n}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$out/${n}_$rep.json')); print('$n', d['value'], d['ms_per_step'], d['stages_ms'])"
  done
done
