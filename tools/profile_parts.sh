#!/bin/bash
# GPU box: tools/profile_round.sh in shorter calls.   bash tools/profile_parts.sh <tag> <part> [config]
#   part trace: rocprofv3 stats of the timed steps and of lone launches (--streams 1)
#   part pmc:   FETCH_SIZE and WRITE_SIZE passes over one lone launch, and the FETCH_SIZE calibration program
set -e
export TMPDIR=/tmp
tag=$1; part=$2; cfg=${3:-c3}; out=gpurun_out/$tag; mkdir -p $out
if [ "$part" = trace ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o kt -- python3 bench.py --config $cfg --timed-only > $out/trace.json 2> $out/trace.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace1 -o kt -- python3 bench.py --config $cfg --timed-only --streams 1 --steps 3 --warmup 1 > $out/trace1.json 2> $out/trace1.log
else
  hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -Wno-unused-result -o $out/calib_fetch tools/calib_fetch.hip
  timeout -k 10 120 $out/calib_fetch > $out/ceiling.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o pmc -- python3 bench.py --config $cfg --timed-only --streams 1 --steps 1 --warmup 0 > $out/fetch.json 2> $out/fetch.log
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o pmc -- python3 bench.py --config $cfg --timed-only --streams 1 --steps 1 --warmup 0 > $out/write.json 2> $out/write.log
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/calib -o pmc -- $out/calib_fetch > $out/calib.log 2>&1
fi
echo done
