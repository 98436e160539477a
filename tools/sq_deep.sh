#!/bin/bash
# SQ counters that split a stage's wave cycles (round 6): issue by instruction class (VALU / LDS / VMEM /
# scalar), waits, in-flight levels (average LDS and VMEM latency), LDS bank conflicts -- three rocprofv3 --pmc passes,
# kernel-trace only, over one lone launch (bench.py --timed-only --streams 1 --steps 1 --warmup 0).
#   bash tools/sq_deep.sh <tag> [config]   -> gpurun_out/<tag>/sqd_<config>.json
set -e
export TMPDIR=/tmp
tag=$1; cfg=${2:-c3}; out=gpurun_out/$tag; mkdir -p $out
T=300; [ "$cfg" = c4 ] && T=700
passes=(
 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
 "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SMEM"
 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR"
)
i=0
for p in "${passes[@]}"; do
  timeout -s KILL $T rocprofv3 --pmc $p --kernel-trace --output-format csv -d $out/sqd_${cfg}_p$i -o pmc -- python3 bench.py --config $cfg --timed-only --streams 1 --steps 1 --warmup 0 > $out/sqd_${cfg}_p$i.json 2> $out/sqd_${cfg}_p$i.log
  i=$((i+1))
done
python3 tools/sq_deep_from_pmc.py $out $cfg $tag > $out/sqd_$cfg.json
echo done
