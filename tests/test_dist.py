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


def _xchg_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = D.RecordExchange()
    out = []
    for step in range(4):   # ragged per-rank, per-step record bytes in 1-3 segments
        rng = np.random.default_rng(100 * step + rank)
        parts = [rng.integers(0, 255, size=int(rng.integers(0, 5000)), dtype=np.uint8) for _ in range(1 + (step + rank) % 3)]
        x.post(parts)   # completes the previous step's exchange first
        q.put(("sent", rank, step, b"".join(p.tobytes() for p in parts)))
        x.finish()
        out.append([r.tobytes() for r in x.result()])
    q.put(("got", rank, out))
    dist.destroy_process_group()


def test_record_exchange_pipelined_world3_gloo():
    """RecordExchange (the bench's pipelined exchange step): after each finish, rank 0 holds every rank's bytes of
    that step in rank order; other ranks hold nothing."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_xchg_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    msgs = [q.get(timeout=120) for _ in range(world * 5)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    sent = {(m[1], m[2]): m[3] for m in msgs if m[0] == "sent"}
    got = {m[1]: [o for o in m[2] if o != []] for m in msgs if m[0] == "got"}
    assert all(got[r] == [] for r in range(1, world))
    assert len(got[0]) == 4
    for step in range(4):
        assert got[0][step] == [sent[(r, step)] for r in range(world)]


def test_merge_rows():
    assert D.merge_rows([[(1,), (2,)], [], [(3,)]]) == [(1,), (2,), (3,)]


def _protocol_worker(rank, world, port, q):
    """The multi-process protocol of bench.py --gpus N / dist.py with the oracle standing in for the GPU aligner:
    shard the reads, align the shard from its own lrand48 position, gather the rows to rank 0."""
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(__file__))
    import oracle_py as O
    from parity_util import _oracle_batch_tsv
    from bioseqdb_amd import NucleotideSequence, effective_opts, synth
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ref = synth.make_reference(120_000, n_rows=2, n_run_every=50_000, n_run_len=80)
    reads = synth.make_reads(ref, 301, seed=3)
    oi = O.OracleIndex()
    for i, t in enumerate(ref.texts()):
        oi.add_ref(i + 1, O.Nuclseq(t.decode()).raw)
    oi.build()
    oo = O.opts_from(effective_opts(None, 2))
    raws = [NucleotideSequence.from_text(reads.text(i)).raw for i in range(reads.n)]
    base = 1000   # this backend's lrand48 position before the call
    lo, hi = D.shard(reads.n, rank, world)
    text, counts = _oracle_batch_tsv(oi, oo, raws[lo:hi], D.first_call_of(rank, world, reads.n, base), threads=1)
    rec = np.frombuffer(np.array(counts, dtype=np.int64).tobytes() + text.encode("latin-1"), dtype=np.uint8)
    got = D.gather_records(rec)
    whole = _oracle_batch_tsv(oi, oo, raws, base, threads=2) if rank == 0 else None
    q.put((rank, [g.tobytes() for g in got], whole, [D.shard(reads.n, r, world) for r in range(world)]))
    dist.destroy_process_group()


def test_sharded_protocol_equals_one_backend_gloo():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_protocol_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, parts, (whole_text, whole_counts), shards = res[0]
    assert len(parts) == world and all(r[1] == [] for r in res[1:])
    text, counts = "", []
    for buf, (lo, hi) in zip(parts, shards):
        c = np.frombuffer(buf[:8 * (hi - lo)], dtype=np.int64).tolist()
        counts += c
        text += buf[8 * (hi - lo):].decode("latin-1")
    assert counts == whole_counts                  # rows per read, read order
    assert text == whole_text and len(text) > 1000  # identical rows: lrand48 positions continue across ranks
