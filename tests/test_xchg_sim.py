"""The multi-rank record exchange (bsq_xchg) rehearsed on the CPU: tests/xchg_sim.cpp runs the real
orchestration of bioseqdb_amd/csrc/exchange_core.h -- the Core that exchange.cpp drives over RCCL -- with threads as
ranks over a host-memory transport that enforces NCCL's matching rules.  World sizes 2..8 (the driver's curve,
which no one-GPU box can run), ragged and empty shares, zero-hit ranks, the staged host-view branch, lanes finishing
their rounds in shuffled order, and a failure injected on one rank (every rank must stop at that (round, lane),
nothing may hang).  Built with ASan + UBSan.  Reference loop being sharded: bioseqdb/extension.cpp:362-370."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def sim(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("xchg") / "xchg_sim")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-Wall", "-Werror", "-pthread",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                    "-o", exe, os.path.join(HERE, "xchg_sim.cpp")], check=True)
    return exe


def _run(exe, *args):
    p = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=120)
    return p.returncode, p.stdout + p.stderr


@pytest.mark.parametrize("world,lanes,rounds", [(2, 1, 3), (2, 4, 5), (3, 4, 6), (4, 4, 4), (8, 4, 6), (8, 6, 3)])
def test_exchange_rounds_match_and_assemble(sim, world, lanes, rounds):
    rc, out = _run(sim, world, lanes, rounds)
    assert rc == 0 and out.rstrip().endswith("OK"), out
    assert "VIOLATION" not in out
    # every rank > 0 sent once per (round, lane); some rounds took the staged branch
    assert f"sends {(world - 1) * lanes * rounds} recvs {(world - 1) * lanes * rounds}" in out


@pytest.mark.parametrize("world,lanes,rounds,fr,fl,fk", [(3, 4, 6, 0, 0, 0), (3, 4, 6, 2, 3, 5), (8, 4, 6, 5, 2, 3),
                                                          (8, 4, 5, 7, 3, 4), (2, 1, 4, 1, 0, 2)])
def test_failure_on_one_rank_stops_every_rank(sim, world, lanes, rounds, fr, fl, fk):
    rc, out = _run(sim, world, lanes, rounds, fr, fl, fk)
    assert rc == 0 and "OK (failure propagated)" in out, out
    tag = f"rank {fr} lane {fl} round {fk} failed"
    assert sum(1 for line in out.splitlines() if line.startswith("rank ") and tag in line) == world, out


@pytest.mark.parametrize("world,lanes,rounds,fl,fk", [(2, 1, 4, 0, 1), (4, 1, 5, 0, 2), (3, 2, 4, 1, 1)])
def test_rank0_receive_failure_does_not_hang(sim, world, lanes, rounds, fl, fk):
    """a lane whose batch waits on a send rank 0 never matched publishes nothing; the other
    ranks' exchange threads must give up (Transport::poll's deadline) instead of waiting forever.  One lane and
    several rounds is the shape where no other wait of the exchange thread has a deadline."""
    rc, out = _run(sim, world, lanes, rounds, 0, fl, fk, "recv")
    assert rc == 0 and "OK (receive failure, no hang)" in out, out
