#!/bin/bash
# GPU box: SQ counter passes (kernel-trace only, one rocprofv3 run per pass) of a lone C3 launch for each value
# of an environment knob.   bash tools/pmc_ab.sh <tag> <VAR> <values...>
set -e
export TMPDIR=/tmp
tag=$1; var=$2; shift 2; out=gpurun_out/$tag; mkdir -p $out
passes=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR"
 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
)
for v in "$@"; do
  i=0
  for p in "${passes[@]}"; do
    env $var=$v timeout -s KILL 300 rocprofv3 --pmc $p --kernel-trace --output-format csv -d $out/${v}_p$i -o pmc -- python3 bench.py --timed-only --streams 1 --steps 1 --warmup 0 > $out/${v}_p$i.log 2>&1
    i=$((i+1))
  done
done
for v in "$@"; do
  mkdir -p $out/sum_$v; cp -r $out/${v}_p* $out/sum_$v/ 2>/dev/null || true
  python3 tools/pmc_summary.py $out/sum_$v > $out/summary_$v.txt
done
echo done
