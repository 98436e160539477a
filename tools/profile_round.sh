#!/bin/bash
# Round profile (GPU box, repo root): bash tools/profile_round.sh <tag>
#   bench (with CPU baseline), rocprofv3 kernel-trace stats of the same command, separate FETCH_SIZE and
#   WRITE_SIZE passes (kernel-trace only), and the FETCH_SIZE calibration program.
set -e
export TMPDIR=/tmp
tag=$1; out=gpurun_out/$tag; mkdir -p $out
hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -Wno-unused-result -o $out/calib_fetch tools/calib_fetch.hip
timeout -k 10 120 $out/calib_fetch > $out/ceiling.log 2>&1
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o kt -- python3 bench.py --timed-only > $out/trace.json 2> $out/trace.log
# lone launches: one batch of all reads per step (the bench line's roofline.isolated figure)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace1 -o kt -- python3 bench.py --timed-only --streams 1 > $out/trace1.json 2> $out/trace1.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o pmc -- python3 bench.py --timed-only --steps 1 --warmup 0 > $out/fetch.json 2> $out/fetch.log
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o pmc -- python3 bench.py --timed-only --steps 1 --warmup 0 > $out/write.json 2> $out/write.log
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/calib -o pmc -- $out/calib_fetch > $out/calib.log 2>&1
echo done
