"""Probe (GPU box): two RCCL ranks on one device when each claims its own host id (NCCL_HOSTID) and RCCL connects them
over the loopback socket transport.  Run as
    timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29512 tools/probe_rccl_hostid.py
Prints one line per rank: an all-reduce, a grouped send/recv to rank 0, and the result."""
import os

rank = int(os.environ["RANK"])
os.environ["NCCL_HOSTID"] = f"probe-rank{rank}"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
os.environ.setdefault("NCCL_IB_DISABLE", "1")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", device_id=dev)
x = torch.full((1024,), float(rank + 1), device=dev)
dist.all_reduce(x)
ok_ar = bool((x == 3).all())
if rank == 0:
    y = torch.zeros(1 << 20, device=dev)
    dist.recv(y, src=1)
    ok_p2p = bool((y == 7).all())
else:
    dist.send(torch.full((1 << 20,), 7.0, device=dev), dst=0)
    ok_p2p = True
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce {ok_ar} send/recv {ok_p2p}", flush=True)
dist.destroy_process_group()
