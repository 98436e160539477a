#!/bin/bash
# GPU box: A/B/C of experiment builds of libbsq (BSQ_LIB) against the in-tree one, alternating, bench lines per run.
#   bash tools/ab_libs.sh <tag> <config> <streams> <reps> <lib>...      (streams 1: lone launches; 4: the timed step)
tag=$1; cfg=$2; ns=$3; reps=$4; shift 4; libs="base $@"; out=gpurun_out/$tag; mkdir -p $out
T=300; [ "$cfg" = c4 ] && T=600
for rep in $(seq 1 $reps); do
  for v in $libs; do
    if [ $v = base ]; then unset BSQ_LIB; n=base; else export BSQ_LIB=$v; n=$(basename $v .so); fi
    timeout -k 10 $T python bench.py --config $cfg --timed-only --streams $ns --steps 10 --warmup 2 > $out/${n}_${cfg}_s${ns}_$rep.json 2> $out/${n}_${cfg}_s${ns}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$out/${n}_${cfg}_s${ns}_$rep.json')); print('$n', '$cfg s$ns', d['value'], d['ms_per_step'], d['stages_ms'])"
  done
done
