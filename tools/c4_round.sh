#!/bin/bash
# GPU box: the C4 line (bench with CPU baseline and oracle parity sample) and the lone-launch rocprof stats,
# or (second argument "pmc") the FETCH_SIZE / WRITE_SIZE passes of one lone launch.
#   bash tools/c4_round.sh <tag> [pmc]
set -e
export TMPDIR=/tmp
tag=$1; out=gpurun_out/$tag; mkdir -p $out
if [ "$2" = pmc ]; then
  timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o pmc -- python3 bench.py --config c4 --timed-only --streams 1 --steps 1 --warmup 0 > $out/fetch.json 2> $out/fetch.log
  timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o pmc -- python3 bench.py --config c4 --timed-only --streams 1 --steps 1 --warmup 0 > $out/write.json 2> $out/write.log
else
  timeout -k 10 700 python3 bench.py --config c4 > $out/bench.json 2> $out/bench.err
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace1 -o kt -- python3 bench.py --config c4 --timed-only --streams 1 --steps 1 --warmup 1 > $out/trace1.json 2> $out/trace1.log
fi
echo done
