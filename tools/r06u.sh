#!/bin/bash
# GPU box (round 6, final tree after the depth-15 table): the whole GPU suite (with the RCCL rehearsal test), then the C4 PMC traffic passes of
# one lone launch with the calibration program.
tag=${1:-r06u}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -Wno-unused-result -o $out/calib_fetch tools/calib_fetch.hip || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o pmc -- python3 bench.py --config c4 --timed-only --streams 1 --steps 1 --warmup 0 > $out/fetch.json 2> $out/fetch.log || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o pmc -- python3 bench.py --config c4 --timed-only --streams 1 --steps 1 --warmup 0 > $out/write.json 2> $out/write.log || exit 1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/calib -o pmc -- $out/calib_fetch > $out/calib.log 2>&1 || exit 1
python3 tools/traffic_from_pmc.py $out $out/traffic_c4.json $tag > /dev/null
echo done
