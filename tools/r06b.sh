#!/bin/bash
# GPU box (round 6): checkpoint (GPU suite + bench line), the PMC counter list, then the CU-split A/B at C3.
tag=${1:-r06b}
bash tools/r06_check.sh $tag || exit 1
timeout -k 10 60 rocprofv3 -L > gpurun_out/$tag/counters.txt 2>&1
bash tools/cu_split_ab.sh $tag c3 0 4 5 6 3 4:blk 5:blk 6:blk
