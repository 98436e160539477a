#!/bin/bash
# SQ counters of one lone launch per stage (GPU box, repo root): two rocprofv3 --pmc passes, kernel-trace only, over
# `bench.py --timed-only --streams 1 --steps 1 --warmup 0` (every stage kernel dispatch belongs to that launch).
#   bash tools/sq_round.sh <tag> [config]      -> gpurun_out/<tag>/sq_<config>.json (bench.py reads profiles/sq_<config>.json)
set -e
export TMPDIR=/tmp
tag=$1; cfg=${2:-c3}; out=gpurun_out/$tag; mkdir -p $out
T=300; [ "$cfg" = c4 ] && T=700
passes=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH"
 "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS"
)
i=0
for p in "${passes[@]}"; do
  timeout -s KILL $T rocprofv3 --pmc $p --kernel-trace --output-format csv -d $out/sq_${cfg}_p$i -o pmc -- python3 bench.py --config $cfg --timed-only --streams 1 --steps 1 --warmup 0 > $out/sq_${cfg}_p$i.json 2> $out/sq_${cfg}_p$i.log
  i=$((i+1))
done
python3 tools/sq_from_pmc.py $out $cfg $tag > $out/sq_$cfg.json
echo done
