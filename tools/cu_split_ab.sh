#!/bin/bash
# GPU box (round 6): seeding and the DP stages of the 4-batch step on disjoint CU sets
# (BSQ_CU_SPLIT=s[:blk], bsq_api.cpp) against the shared default; the timed step (C3 or C4) with checksums, two
# alternating rounds.   bash tools/cu_split_ab.sh <tag> [config] [splits...]
# The split was removed from the library; apply profiles/r06/cu_split/cu_split.patch (git apply) to rerun it.
tag=$1; cfg=${2:-c3}; shift 2; splits=${@:-"0 4 5 6 3 4:blk 5:blk 6:blk"}
out=gpurun_out/$tag; mkdir -p $out
T=300; [ "$cfg" = c4 ] && T=700
for rep in 1 2; do
  for sp in $splits; do
    f=$out/split_${sp/:/_}_$rep.json
    if [ "$sp" = 0 ]; then
      timeout -k 10 $T python bench.py --config $cfg --timed-only --checksums > $f 2> $f.err || exit 1
    else
      BSQ_CU_SPLIT=$sp timeout -k 10 $T python bench.py --config $cfg --timed-only --checksums > $f 2> $f.err || exit 1
    fi
    python3 -c "import json; d=json.load(open('$f')); print('split=$sp', d['value'], d['ms_per_step'], d['checksums'], {k: round(v, 2) for k, v in d['stages_ms'].items()})"
  done
done
