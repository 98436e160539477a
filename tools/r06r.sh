#!/bin/bash
# (The band-class sort was then removed from the library: BSQ_R2A_NOSORT no longer exists; profiles/r06/r2a_order/.)
# GPU box (round 6): the CIGAR stage's diagonal pass over reads in batch order instead of the band-class order
# (BSQ_R2A_NOSORT=1: no k_r2a_key + sort; the pass still routes each read to the kernel of its class) -- parity with
# it on, A/B of the C3 step (checksums) and lone launches, then FETCH_SIZE / WRITE_SIZE passes of one lone launch each.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r06r}; out=gpurun_out/$tag; mkdir -p $out
BSQ_R2A_NOSORT=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_long_reads.py -k "parity or all_columns or option or lrand48 or long" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
run() {   # name nosort cfg extra...
  local name=$1 m=$2 cfg=$3; shift 3
  BSQ_R2A_NOSORT=$m timeout -k 10 500 python bench.py --config $cfg --timed-only --checksums "$@" > $out/$name.json 2> $out/$name.err || exit 1
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', d['value'], d['ms_per_step'], d['checksums'], {k: round(v, 3) for k, v in d['stages_ms'].items()})"
}
for rep in 1 2 3; do
  run c3_nosort_$rep 1 c3
  run c3_sort_$rep 0 c3
done
for rep in 1 2; do
  run c3lone_nosort_$rep 1 c3 --streams 1
  run c3lone_sort_$rep 0 c3 --streams 1
done
for m in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    BSQ_R2A_NOSORT=$m timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $out/pmc_${m}_$c -o pmc -- python3 bench.py --config c3 --timed-only --streams 1 --steps 1 --warmup 0 > $out/pmc_${m}_$c.json 2> $out/pmc_${m}_$c.log || exit 1
    python3 tools/pmc_summary.py $out/pmc_${m}_$c reg2aln > $out/pmc_${m}_$c.txt; python3 tools/pmc_summary.py $out/pmc_${m}_$c r2a_key >> $out/pmc_${m}_$c.txt
  done
done
echo done
