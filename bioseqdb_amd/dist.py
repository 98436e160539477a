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


class RecordExchange:
    """The exchange step of a sharded job, pipelined (bench.py --gpus N): the hit records
    of step k travel to rank `dst` (the calling backend) while step k+1 aligns.

    post(parts) takes this rank's record segments of one step (host uint8 arrays, in read order):
      * the byte counts are all-gathered (tiny, host-visible: the receive buffers are sized from them);
      * the segments are packed into this rank's send buffer -- in HBM for RCCL (host-to-device copies on a side
        stream), in host memory for gloo -- and gathered into `dst`'s receive buffers asynchronously (RCCL over
        xGMI on a multi-GPU node);
      * on `dst` the received buffers are copied into pinned host memory after the gather (same side stream), so
        the rows reach the caller's host without a host-side wait in the step.
    post() first completes the previous exchange (its buffers are reused); finish() completes the last one.
    result() on `dst` returns the per-rank byte arrays of the last completed exchange, in rank (= read) order.
    """

    def __init__(self, device=None, group=None, dst: int = 0):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group, self.dst = torch, dist, group, dst
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.dev = device if device is not None else torch.device("cpu")
        self.gpu = self.dev.type == "cuda"
        self.stream = torch.cuda.Stream(device=self.dev) if self.gpu else None
        self.send = None
        self.recv = None
        self.host = None
        self.work = None
        self.event = None
        self.sizes = None
        self.done_sizes = None
        self.bytes_moved = 0

    def _grow(self, buf, n, pinned_host=False):
        torch = self.torch
        if buf is not None and buf.numel() >= n:
            return buf
        n = max(int(n * 1.25), 1)
        if pinned_host:
            return torch.empty(n, dtype=torch.uint8, pin_memory=True)
        return torch.empty(n, dtype=torch.uint8, device=self.dev)

    def post(self, parts: Sequence[np.ndarray]) -> None:
        """Exchange host record segments (read order)."""
        torch = self.torch

        def fill(send):
            off = 0
            for p in parts:
                if p.nbytes:
                    src = torch.from_numpy(np.ascontiguousarray(p).view(np.uint8).reshape(-1))
                    send[off:off + p.nbytes].copy_(src)
                    off += p.nbytes
        self.post_fill(int(sum(p.nbytes for p in parts)), fill)

    def post_fill(self, n: int, fill) -> None:
        """Exchange n bytes that fill(send_buffer) writes into bytes [0, n) of the send buffer (on this rank's
        exchange device) and that are complete when it returns (e.g. bsq_batch_copy_records per batch)."""
        torch, dist = self.torch, self.dist
        self.finish()
        cnt = torch.tensor([n], dtype=torch.int64, device=self.dev)
        allc = [torch.zeros(1, dtype=torch.int64, device=self.dev) for _ in range(self.world)]
        dist.all_gather(allc, cnt, group=self.group)
        sizes = [int(c.item()) for c in allc]
        mx = max(max(sizes), 1)
        self.send = self._grow(self.send, mx)
        me_dst = self.rank == self.dst
        if me_dst:
            if self.recv is None or len(self.recv) != self.world or self.recv[0].numel() < mx:
                self.recv = [self._grow(None, mx) for _ in range(self.world)]
            if self.gpu and (self.host is None or any(h.numel() < s for h, s in zip(self.host, sizes))):
                self.host = [self._grow(None, max(s, 1), pinned_host=True) for s in sizes]
        if self.gpu:
            torch.cuda.current_stream(self.dev).synchronize()   # the send buffer's allocation / last use
        fill(self.send)
        ctx = torch.cuda.stream(self.stream) if self.gpu else _nullctx()
        with ctx:
            recv = [r[:mx] for r in self.recv] if me_dst else None
            self.work = dist.gather(self.send[:mx], recv, dst=self.dst, group=self.group, async_op=True)
            if self.gpu:
                # on every rank: the side stream (and the event recorded on it) follows the gather, so finish()
                # waiting on the event means the send buffer may be refilled and the receive buffers read
                self.work.wait()
                if me_dst:
                    for h, r, s in zip(self.host, self.recv, sizes):
                        if s:
                            h[:s].copy_(r[:s], non_blocking=True)
                self.event = torch.cuda.Event()
                self.event.record(self.stream)
        self.sizes = sizes
        self.bytes_moved += sum(sizes) if me_dst else n

    def finish(self) -> None:
        if self.work is None:
            return
        self.work.wait()
        if self.event is not None:
            self.event.synchronize()
        self.work, self.event = None, None
        self.done_sizes = self.sizes

    def result(self) -> List[np.ndarray]:
        """`dst`: the per-rank record bytes of the last finished exchange (valid until the next post); else []."""
        if self.rank != self.dst or self.done_sizes is None:
            return []
        bufs = self.host if self.gpu else self.recv
        return [b[:s].numpy() for b, s in zip(bufs, self.done_sizes)]


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


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
