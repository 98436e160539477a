#!/bin/bash
# GPU box (round 6): the default bench line with CPU baseline, rocprofv3 kernel-trace stats of the timed steps and of
# lone launches, the FETCH/WRITE PMC passes of one lone launch with the FETCH_SIZE calibration program, the SQ passes
# (tools/sq_round.sh) and the deeper SQ split (tools/sq_deep.sh), all under gpurun_out/<tag>.
#   bash tools/r06_final.sh <tag> [config]
set -e
export TMPDIR=/tmp
tag=${1:-r06f}; cfg=${2:-c3}; out=gpurun_out/$tag; mkdir -p $out
T=600; [ "$cfg" = c4 ] && T=1100
hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -Wno-unused-result -o $out/calib_fetch tools/calib_fetch.hip
timeout -k 10 $T python -u bench.py --config $cfg > $out/bench.json 2> $out/bench.err
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('sql_cursor') or {}).get('reads_per_s_with_columns'))"
timeout -k 10 $T rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o kt -- python3 bench.py --config $cfg --timed-only > $out/trace.json 2> $out/trace.log
timeout -k 10 $T rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace1 -o kt -- python3 bench.py --config $cfg --timed-only --streams 1 > $out/trace1.json 2> $out/trace1.log
timeout -k 10 $T rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o pmc -- python3 bench.py --config $cfg --timed-only --streams 1 --steps 1 --warmup 0 > $out/fetch.json 2> $out/fetch.log
timeout -k 10 $T rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o pmc -- python3 bench.py --config $cfg --timed-only --streams 1 --steps 1 --warmup 0 > $out/write.json 2> $out/write.log
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/calib -o pmc -- $out/calib_fetch > $out/calib.log 2>&1
python3 tools/traffic_from_pmc.py $out $out/traffic_$cfg.json $tag > /dev/null
bash tools/sq_round.sh $tag $cfg
[ "$cfg" = c3 ] && bash tools/sq_deep.sh $tag $cfg
echo done
