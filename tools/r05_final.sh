#!/bin/bash
# GPU box (round 5, final tree): the default bench line with CPU baseline, rocprofv3 kernel-trace stats of the timed
# steps and of lone launches, the FETCH/WRITE PMC passes and the SQ passes of one lone launch, all under gpurun_out/<tag>.
#   bash tools/r05_final.sh <tag>
set -e
export TMPDIR=/tmp
tag=${1:-r05f}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['sql_cursor']['reads_per_s_with_columns'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o kt -- python3 bench.py --timed-only > $out/trace.json 2> $out/trace.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace1 -o kt -- python3 bench.py --timed-only --streams 1 > $out/trace1.json 2> $out/trace1.log
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o pmc -- python3 bench.py --timed-only --streams 1 --steps 1 --warmup 0 > $out/fetch.json 2> $out/fetch.log
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o pmc -- python3 bench.py --timed-only --streams 1 --steps 1 --warmup 0 > $out/write.json 2> $out/write.log
bash tools/sq_round.sh $tag c3
echo done
