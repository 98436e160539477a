#!/bin/bash
# GPU box (round 6, final tree): the default (C3) bench line with CPU baseline, rocprofv3 kernel-trace stats of the
# timed steps and of lone launches, the FETCH/WRITE PMC passes of one lone launch with the FETCH_SIZE calibration
# program (C3 traffic), then the C4 lone-launch kernel stats.   bash tools/r06v.sh <tag>
set -e
export TMPDIR=/tmp
tag=${1:-r06v}; out=gpurun_out/$tag; mkdir -p $out
hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -Wno-unused-result -o $out/calib_fetch tools/calib_fetch.hip
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('sql_cursor') or {}).get('reads_per_s_with_columns'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o kt -- python3 bench.py --timed-only > $out/trace.json 2> $out/trace.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace1 -o kt -- python3 bench.py --timed-only --streams 1 > $out/trace1.json 2> $out/trace1.log
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o pmc -- python3 bench.py --timed-only --streams 1 --steps 1 --warmup 0 > $out/fetch.json 2> $out/fetch.log
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o pmc -- python3 bench.py --timed-only --streams 1 --steps 1 --warmup 0 > $out/write.json 2> $out/write.log
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/calib -o pmc -- $out/calib_fetch > $out/calib.log 2>&1
python3 tools/traffic_from_pmc.py $out $out/traffic_c3.json $tag > /dev/null
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace1_c4 -o kt -- python3 bench.py --config c4 --timed-only --streams 1 > $out/trace1_c4.json 2> $out/trace1_c4.log
echo done
