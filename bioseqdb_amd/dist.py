"""Read-sharded multi-GPU driver (one process per GPU, torch.distributed over RCCL or gloo).

The SQL path is embarrassingly parallel over query rows (extension.cpp:362-370 aligns one cursor row
at a time and libbwa keeps no cross-read state except the lrand48 position, Q10).  Each rank takes a
contiguous slice of the reads, aligns it on its own GPU against its own replica of the index, and the
hit records travel to rank 0 (the calling backend) in one gather, which preserves read order
(rank order == read order, Q16).  No other collective sits on the data path.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def shard(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous read range [lo, hi) of `rank` among `world` ranks."""
    return n * rank // world, n * (rank + 1) // world


def first_call_of(rank: int, world: int, n_total: int, base: int = 0) -> int:
    """lrand48 stream position of the shard's first read: as if one backend aligned all reads in order."""
    return base + shard(n_total, rank, world)[0]


def gather_records(local: np.ndarray, group=None, device=None, dst: int = 0) -> List[np.ndarray]:
    """Gather variable-length uint8 record buffers to rank `dst` (the calling backend), in rank order.

    Returns the per-rank buffers on `dst` and [] elsewhere.  Works with the "nccl" (RCCL, tensors on
    `device`) and "gloo" (CPU tensors) backends: one all-gather of the byte counts, one gather of the
    buffers padded to the largest -- only the caller receives rows, as in the SQL path."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    me = dist.get_rank(group)
    dev = device if device is not None else torch.device("cpu")
    n = torch.tensor([local.nbytes], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes_i = [int(s.item()) for s in sizes]
    mx = max(max(sizes_i), 1)
    buf = torch.zeros(mx, dtype=torch.uint8, device=dev)
    if local.nbytes:
        buf[:local.nbytes].copy_(torch.from_numpy(np.ascontiguousarray(local).view(np.uint8).reshape(-1)))
    out = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(world)] if me == dst else None
    dist.gather(buf, out, dst=dst, group=group)
    if me != dst:
        return []
    return [o[:s].cpu().numpy() for o, s in zip(out, sizes_i)]


def replicate_index(L, idx, gpu: int, src: int = 0, group=None):
    """One index build for the whole job: rank `src` passes its built host index
    `idx`, every other rank passes None.  The root uploads into torch-allocated device buffers, the
    metadata blob and every device table are broadcast (RCCL over xGMI with the "nccl" backend), and the
    other ranks import them.  Returns (index handle, buffers to keep alive while the index is used)."""
    import ctypes

    import torch
    import torch.distributed as dist

    from ._native import N_TABLES, Table, check

    rank = dist.get_rank(group)
    if rank == src:
        sizes = (ctypes.c_uint64 * N_TABLES)()
        mb = ctypes.c_uint64()
        check(L.bsq_index_layout(idx, sizes, None, ctypes.byref(mb)))
        meta = ctypes.create_string_buffer(mb.value)
        check(L.bsq_index_layout(idx, sizes, meta, ctypes.byref(mb)))
        obj = [list(sizes), bytes(meta.raw)]
    else:
        obj = [None, None]
    dist.broadcast_object_list(obj, src=src, group=group)
    sizes, meta = obj
    dev = torch.device("cuda", gpu)
    bufs = [torch.empty(int(b), dtype=torch.uint8, device=dev) if b else None for b in sizes]
    tables = (Table * N_TABLES)(*[Table(t.data_ptr() if t is not None else None, int(b)) for t, b in zip(bufs, sizes)])
    if rank == src:
        check(L.bsq_index_upload_into(idx, gpu, tables, N_TABLES))
    torch.cuda.synchronize(dev)
    for t in bufs:
        if t is not None:
            dist.broadcast(t, src=src, group=group)
    torch.cuda.synchronize(dev)
    if rank != src:
        out = ctypes.c_void_p()
        mbuf = ctypes.create_string_buffer(meta, len(meta))
        check(L.bsq_index_import(mbuf, len(meta), gpu, tables, N_TABLES, ctypes.byref(out)))
        idx = out
    return idx, bufs


def merge_rows(per_rank: Sequence[Sequence[tuple]]) -> List[tuple]:
    """Concatenate per-rank result rows in rank (= read) order."""
    out: List[tuple] = []
    for rows in per_rank:
        out.extend(rows)
    return out
