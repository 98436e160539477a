#!/bin/bash
# GPU box (round 6, final tree): the C4 bench line and its rocprofv3 kernel-trace stats (timed steps, lone launches).
set -e
export TMPDIR=/tmp
tag=${1:-r06i}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u bench.py --config c4 > $out/bench_c4.json 2> $out/bench_c4.err
python3 -c "import json; d=json.load(open('$out/bench_c4.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('value_sql_call'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o kt -- python3 bench.py --config c4 --timed-only > $out/trace.json 2> $out/trace.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace1 -o kt -- python3 bench.py --config c4 --timed-only --streams 1 > $out/trace1.json 2> $out/trace1.log
echo done
