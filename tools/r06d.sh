#!/bin/bash
# GPU box (round 6): the SQ split of every kernel of a lone C3 launch (tools/sq_deep.sh), then the C4 bench line.
tag=${1:-r06d}
mkdir -p gpurun_out/$tag
bash tools/sq_deep.sh $tag c3 || exit 1
timeout -k 10 1000 python -u bench.py --config c4 > gpurun_out/$tag/bench_c4.json 2> gpurun_out/$tag/bench_c4.err
