#!/bin/bash
# GPU box: rocprofv3 kernel-trace stats of lone launches (--streams 1) for one environment variant, plus
# separate FETCH_SIZE / WRITE_SIZE passes.   bash tools/prof_variant.sh <tag> <config> [VAR=value ...]
set -e
export TMPDIR=/tmp
tag=$1; cfg=$2; shift 2; out=gpurun_out/$tag; mkdir -p $out
for kv in "$@"; do export "$kv"; done
T=300; [ "$cfg" = c4 ] && T=900
timeout -k 10 $T rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace1 -o kt -- python3 bench.py --config $cfg --timed-only --streams 1 --steps 3 --warmup 1 > $out/trace1.json 2> $out/trace1.log
timeout -k 10 $T rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o pmc -- python3 bench.py --config $cfg --timed-only --streams 1 --steps 1 --warmup 0 > $out/fetch.json 2> $out/fetch.log
timeout -k 10 $T rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o pmc -- python3 bench.py --config $cfg --timed-only --streams 1 --steps 1 --warmup 0 > $out/write.json 2> $out/write.log
echo done
