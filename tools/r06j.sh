#!/bin/bash
# GPU box (round 6, final tree): C4 PMC traffic of one lone launch (FETCH/WRITE passes + the calibration program) and
# its SQ passes, then the C1 and C2 bench lines.
set -e
export TMPDIR=/tmp
tag=${1:-r06j}; out=gpurun_out/$tag; mkdir -p $out
hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -Wno-unused-result -o $out/calib_fetch tools/calib_fetch.hip
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o pmc -- python3 bench.py --config c4 --timed-only --streams 1 --steps 1 --warmup 0 > $out/fetch.json 2> $out/fetch.log
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o pmc -- python3 bench.py --config c4 --timed-only --streams 1 --steps 1 --warmup 0 > $out/write.json 2> $out/write.log
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/calib -o pmc -- $out/calib_fetch > $out/calib.log 2>&1
python3 tools/traffic_from_pmc.py $out $out/traffic_c4.json $tag > /dev/null
bash tools/sq_round.sh $tag c4
timeout -k 10 300 python -u bench.py --config c2 > $out/bench_c2.json 2> $out/bench_c2.err
timeout -k 10 300 python -u bench.py --config c1 > $out/bench_c1.json 2> $out/bench_c1.err
echo done
