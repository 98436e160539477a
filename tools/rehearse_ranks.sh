#!/bin/bash
# GPU box: the driver's multi-GPU bench command shape, rehearsed with ranks sharing the one GPU over gloo (RCCL
# refuses two ranks on one device: tools/probe_rccl_dup.py), at 2 and 4 ranks.  The native RCCL exchange path is
# only runnable at world 1 here (--exchange-world1, tests/test_gpu_group_bench.py).
tag=${1:-rehearse}
mkdir -p gpurun_out/$tag
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) \
    bench.py --gpus $n --steps 3 --warmup 1 --dist-backend gloo --no-cpu-baseline --no-codec > gpurun_out/$tag/n$n.json 2> gpurun_out/$tag/n$n.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/$tag/n$n.json').read().strip().splitlines()[-1]); print('ranks $n', d['n_gpus'], d['value'], d['ms_per_step'], d['scaling'], d.get('exchange'))"
done
