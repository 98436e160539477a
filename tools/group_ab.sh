#!/bin/bash
# GPU box: the one-device group line against the N = 1 line at full size, and the exchange routes.
#   bash tools/group_ab.sh <tag> [config]      (config: c3 default, c4)
set -e
tag=$1; cfg=${2:-c3}; out=gpurun_out/$tag; mkdir -p $out
T=400; [ "$cfg" = c4 ] && T=900
timeout -k 10 $T python bench.py --config $cfg --no-cpu-baseline --timed-only > $out/n1_$cfg.json 2> $out/n1_$cfg.err
timeout -k 10 $T python bench.py --config $cfg --gpus 1 --group-devices 0 --no-cpu-baseline --no-isolated > $out/g1_$cfg.json 2> $out/g1_$cfg.err
timeout -k 10 $T python bench.py --config $cfg --no-cpu-baseline --timed-only > $out/n1b_$cfg.json 2> $out/n1b_$cfg.err
timeout -k 10 $T python bench.py --config $cfg --gpus 1 --group-devices 0 --no-cpu-baseline --no-isolated > $out/g1b_$cfg.json 2> $out/g1b_$cfg.err
MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 timeout -k 10 $T python bench.py --config $cfg --exchange-world1 --no-cpu-baseline --timed-only > $out/x1_$cfg.json 2> $out/x1_$cfg.err
if [ "$cfg" = c3 ]; then
  for x in links via-first; do
    timeout -k 10 $T python bench.py --gpus 2 --group-devices 0,0 --reads 500000 --exchange $x --no-cpu-baseline --no-isolated > $out/g2_$x.json 2> $out/g2_$x.err
  done
fi
python - $out $cfg <<'PY'
import json, sys
out, cfg = sys.argv[1], sys.argv[2]
import glob, os
for f in sorted(glob.glob(f"{out}/*.json")):
    d = json.load(open(f))
    print(os.path.basename(f), d["value"], d["ms_per_step"], (d.get("exchange") or {}).get("mode"), d["config"].get("step_schedule"))
PY
