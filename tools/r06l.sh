#!/bin/bash
# GPU box (round 6): the C1 and C2 bench lines, then the native-RCCL rehearsal (tools/rehearse_rccl.sh).
tag=${1:-r06l}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 300 python -u bench.py --config c2 > $out/bench_c2.json 2> $out/bench_c2.err || exit 1
timeout -k 10 300 python -u bench.py --config c1 > $out/bench_c1.json 2> $out/bench_c1.err || exit 1
for c in c1 c2; do python3 -c "import json; d=json.load(open('$out/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('parity_sample') or {}).get('checksum_match'))"; done
bash tools/rehearse_rccl.sh $tag/rccl
