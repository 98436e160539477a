#!/bin/bash
# SQ/TCC counter passes (one rocprofv3 run per pass, kernel-trace only) of lone C3 launches and of C4 seeding.
#   bash tools/prof_sq.sh <tag>     (GPU box, repo root)
set -e
export TMPDIR=/tmp
tag=$1; out=gpurun_out/$tag; mkdir -p $out
passes=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM"
 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
 "FETCH_SIZE TCC_HIT_sum"
)
i=0
for p in "${passes[@]}"; do
  timeout -s KILL 300 rocprofv3 --pmc $p --kernel-trace --output-format csv -d $out/c3_p$i -o pmc -- python3 bench.py --timed-only --streams 1 --steps 1 --warmup 0 > $out/c3_p$i.log 2>&1
  if [ -n "$C4" ]; then
    EXP_READS=1000000 timeout -s KILL 300 rocprofv3 --pmc $p --kernel-trace --output-format csv -d $out/c4_p$i -o pmc -- python3 exp/c4_seed.py > $out/c4_p$i.log 2>&1
  fi
  i=$((i+1))
done
python3 tools/pmc_summary.py $out > $out/summary.txt
echo done
