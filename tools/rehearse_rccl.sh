#!/bin/bash
# GPU box (round 6): the driver's torchrun bench with the NATIVE RCCL exchange between processes, ranks sharing the one
# GPU (BSQ_REHEARSE_SHARED_GPU=1: a host id per rank, RCCL over loopback sockets).  First the RCCL probe, then
# bench.py --gpus 2 and 4 with --checksums (rank 0's copy of every rank's records must equal a one-GPU run of that
# rank's reads: --seed-offset r), then those one-GPU runs.  Rates are meaningless here (one shared GPU).
tag=${1:-rccl}; out=gpurun_out/$tag; mkdir -p $out
export NCCL_DEBUG=WARN
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
  tools/probe_rccl_hostid.py > $out/probe.log 2>&1
rc=$?; grep -E "^rank" $out/probe.log; [ $rc -eq 0 ] || { tail -20 $out/probe.log; exit $rc; }
for n in 2 4; do
  BSQ_REHEARSE_SHARED_GPU=1 BSQ_XCHG_TIMEOUT_S=120 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29620 + n)) bench.py --gpus $n --steps 3 --warmup 1 --checksums --reads 200000 \
    --no-cpu-baseline --no-codec > $out/n$n.json 2> $out/n$n.err || { tail -30 $out/n$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/n$n.json').read().strip().splitlines()[-1]); print('ranks $n', d['n_gpus'], d['value'], d['checksums'], d.get('parity_sample'), d.get('exchange'))"
done
for r in 0 1 2 3; do
  timeout -k 10 300 python bench.py --timed-only --checksums --reads 200000 --steps 3 --warmup 1 --seed-offset $r > $out/one_$r.json 2> $out/one_$r.err || exit 1
  python3 -c "import json; d=json.load(open('$out/one_$r.json')); print('one-GPU seed-offset $r', d['checksums'])"
done
