#!/bin/bash
# Round profile (GPU box, repo root): bash tools/profile_round.sh <tag> [config]   (config: c3 (default), c4, c2)
#   the bench line (with CPU baseline), rocprofv3 kernel-trace stats of the timed steps (concurrent batches) and
#   of lone launches (--streams 1: the line's `roofline` figure), separate FETCH_SIZE and WRITE_SIZE passes over
#   one lone launch (kernel-trace only), and the FETCH_SIZE calibration program.
set -e
export TMPDIR=/tmp
tag=$1; cfg=${2:-c3}; out=gpurun_out/$tag; mkdir -p $out
T=600; [ "$cfg" = c4 ] && T=1100
hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -Wno-unused-result -o $out/calib_fetch tools/calib_fetch.hip
timeout -k 10 120 $out/calib_fetch > $out/ceiling.log 2>&1
timeout -k 10 $T python bench.py --config $cfg > $out/bench.json 2> $out/bench.err
timeout -k 10 $T rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o kt -- python3 bench.py --config $cfg --timed-only > $out/trace.json 2> $out/trace.log
timeout -k 10 $T rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace1 -o kt -- python3 bench.py --config $cfg --timed-only --streams 1 > $out/trace1.json 2> $out/trace1.log
timeout -k 10 $T rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o pmc -- python3 bench.py --config $cfg --timed-only --streams 1 --steps 1 --warmup 0 > $out/fetch.json 2> $out/fetch.log
timeout -k 10 $T rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o pmc -- python3 bench.py --config $cfg --timed-only --streams 1 --steps 1 --warmup 0 > $out/write.json 2> $out/write.log
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/calib -o pmc -- $out/calib_fetch > $out/calib.log 2>&1
echo done
