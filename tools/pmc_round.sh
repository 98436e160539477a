#!/bin/bash
# GPU box: FETCH_SIZE and WRITE_SIZE passes (kernel-trace only) of one lone launch, and the FETCH_SIZE calibration.
#   bash tools/pmc_round.sh <tag> [config]      -> gpurun_out/<tag>/{fetch,write,calib}; tools/traffic_from_pmc.py reads them
set -e
export TMPDIR=/tmp
tag=$1; cfg=${2:-c3}; out=gpurun_out/$tag; mkdir -p $out
T=400; [ "$cfg" = c4 ] && T=700
hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -Wno-unused-result -o $out/calib_fetch tools/calib_fetch.hip
timeout -k 10 $T rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o pmc -- python3 bench.py --config $cfg --timed-only --streams 1 --steps 1 --warmup 0 > $out/fetch.json 2> $out/fetch.log
timeout -k 10 $T rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o pmc -- python3 bench.py --config $cfg --timed-only --streams 1 --steps 1 --warmup 0 > $out/write.json 2> $out/write.log
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/calib -o pmc -- $out/calib_fetch > $out/calib.log 2>&1
echo done
