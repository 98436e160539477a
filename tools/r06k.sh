#!/bin/bash
# GPU box (round 6): libbsq's load-time hardware-queue default -- the C3 step with GPU_MAX_HW_QUEUES unset and left to
# the library (must match 8, not HIP's 4), explicit 4 and 8; then the drop-in cursor at 4 and at the library default.
tag=${1:-r06k}; out=gpurun_out/$tag; mkdir -p $out
for rep in 1 2; do
  env -u GPU_MAX_HW_QUEUES BSQ_HW_QUEUES=lib timeout -k 10 300 python bench.py --timed-only --checksums > $out/lib_$rep.json 2> $out/lib_$rep.err || exit 1
  BSQ_HW_QUEUES=4 timeout -k 10 300 python bench.py --timed-only --checksums > $out/q4_$rep.json 2> $out/q4_$rep.err || exit 1
  BSQ_HW_QUEUES=8 timeout -k 10 300 python bench.py --timed-only --checksums > $out/q8_$rep.json 2> $out/q8_$rep.err || exit 1
  for v in lib q4 q8; do python3 -c "import json; d=json.load(open('$out/${v}_$rep.json')); print('$v', d['value'], d['ms_per_step'], d['checksums'])"; done
done
env -u GPU_MAX_HW_QUEUES BSQ_HW_QUEUES=lib timeout -k 10 300 python bench.py --cursor-only > $out/cursor_lib.json 2> $out/cursor_lib.err || exit 1
BSQ_HW_QUEUES=4 timeout -k 10 300 python bench.py --cursor-only > $out/cursor_q4.json 2> $out/cursor_q4.err || exit 1
for v in lib q4; do python3 -c "import json; d=json.load(open('$out/cursor_$v.json'))['sql_cursor']; print('cursor $v', d['reads_per_s_with_columns'], d['reads_per_s_records_only'], d['steady_state'])"; done
