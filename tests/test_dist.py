"""Multi-rank read sharding + gather of hit records, world_size 2 on gloo (CPU)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from bioseqdb_amd import dist as D


def test_shard_covers_all_reads_in_order():
    for n in (0, 1, 7, 1000, 1001):
        for w in (1, 2, 3, 8):
            parts = [D.shard(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            assert all(D.first_call_of(r, w, n, 10) == 10 + parts[r][0] for r in range(w))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(rank)
    local = rng.integers(0, 255, size=100 + 37 * rank, dtype=np.uint8)   # ragged per-rank record bytes
    got = D.gather_records(local)
    q.put((rank, [g.tobytes() for g in got], local.tobytes()))
    dist.destroy_process_group()


def test_gather_records_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    locals_ = [r[2] for r in res]
    for rank, got, _ in res:
        if rank == 0:
            assert got == locals_, rank       # the caller sees every rank's records in rank (= read) order
        else:
            assert got == [], rank            # only the calling backend receives rows


def test_merge_rows():
    assert D.merge_rows([[(1,), (2,)], [], [(3,)]]) == [(1,), (2,), (3,)]
