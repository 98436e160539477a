#!/bin/bash
# Timing experiments (GPU box): stage times with parts of the DP switched off (BSQ_EXP bits, see
# bsq_device.h DOpts::exp_flags).  Results differ from the oracle under these flags; timing only.
set -e
mkdir -p gpurun_out/exp
for f in 0 1 2 4; do
  BSQ_EXP=$f timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/exp/f$f.json 2> gpurun_out/exp/f$f.err || true
  python -c "import json,sys; d=json.load(open('gpurun_out/exp/f$f.json')); print('flag $f', d['value'], d['stages_ms'])"
done
