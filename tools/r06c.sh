#!/bin/bash
# GPU box (round 6): checkpoint (GPU suite + bench line) on the tree with the deferred-store extension cell loop,
# the PMC counter list, the extension A/B against the previous library (lone C3 launches), the CU-split A/B at C3.
tag=${1:-r06c}
bash tools/r06_check.sh $tag || exit 1
timeout -k 10 60 rocprofv3 -L > gpurun_out/$tag/counters.txt 2>&1
bash tools/ab_lib.sh $tag/ext exp/libbsq_base.so c3 2 > gpurun_out/$tag/ext_ab.txt 2>&1 || exit 1
bash tools/cu_split_ab.sh $tag c3 0 4 5 6 3 4:blk 6:blk > gpurun_out/$tag/split_ab.txt 2>&1
