#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: aligned reads/s, 150 bp synthetic reads vs a 100 Mbp synthetic
reference, full BWA-MEM seed + extend + CIGAR (configs[2], "C3"), on N MI355X GPUs.

--config c2 measures configs[1] (FM-index seeding only, mem_collect_intv) and --config c4 configs[3]
(10M reads vs a 3 Gbp reference of 24 rows x 125 Mbp: 64-bit rows, index > Infinity Cache, the batch
runs in 1M-read workspace chunks); the default (no flags) is C3.

One step = one pass of the whole alignment path (libbsq: smem -> chain -> extend -> reg2aln -> pack ->
D2H of the hit records) over one batch of reads already resident in HBM; with N > 1 each rank aligns
its own batch (weak scaling, read-sharded) and the hit records are gathered to rank 0 over RCCL
(the exchange step of the SQL path: all rows return to the calling backend).

Prints ONE JSON line on rank 0 with `roofline` (dominant kernel, algorithmic bytes / HIP-event time on
the batch stream) and `cpu_baseline` (the CPU oracle on this host's cores, bounded sample, rank 0 at
N = 1 only; its outputs are also checksummed against the GPU's for the same reads).
"""
from __future__ import annotations

import os
import sys

# HIP hardware queues of this process (the runtime's default is 4): the concurrent batches below each
# own a stream, and 8 queues let 4 of them run without sharing a queue (+3 % over 3 batches on 4 queues).
# RCCL communicators (a device group, the torchrun exchange lanes) take queues of their own: with 8, two batch
# streams then share one and the step loses 15-20 % (one-device group at C3: 42.6 M reads/s on 8 queues, 49.4 M on
# 16 -- the N = 1 line's rate).  Set before anything loads the HIP runtime (the box exports 4; BSQ_HW_QUEUES
# overrides this choice).
_RCCL_IN_PROCESS = (int(os.environ.get("WORLD_SIZE", "1")) > 1 or "--exchange-world1" in sys.argv[1:]
                    or "--group-devices" in sys.argv[1:]
                    or any(a.startswith("--gpus") and (a.split("=")[1:] or ["1"])[0] != "1" for a in sys.argv[1:])
                    or ("--gpus" in sys.argv[1:] and sys.argv[sys.argv.index("--gpus") + 1:][:1] != ["1"]))
if os.environ.get("BSQ_HW_QUEUES") != "lib":   # "lib": leave the choice to libbsq's load-time default (8 when unset)
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("BSQ_HW_QUEUES", "16" if _RCCL_IN_PROCESS else "8")
# BSQ_REHEARSE_SHARED_GPU=1 (one-GPU rehearsal of the driver's torchrun run, tools/rehearse_rccl.sh): RCCL refuses two ranks on
# one device ("Duplicate GPU detected", judged by host id + bus id), so every rank claims a host of its own and RCCL
# connects them over its socket transport on the loopback device -- the native exchange (all-gathers, send/recv of the
# wire records, rank 0's expansion) then runs for real between processes; rates are meaningless (one shared GPU)
if os.environ.get("BSQ_REHEARSE_SHARED_GPU") == "1" and int(os.environ.get("WORLD_SIZE", "1")) > 1:
    os.environ["NCCL_HOSTID"] = "bsq-rehearsal-rank" + os.environ.get("RANK", "0")
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
# the native record exchange gives up (and aborts its communicator on every rank) after this long without progress
# from the other ranks; a timed step is ~20 ms, so 3 minutes means a broken run, and the job should end, not hang
os.environ.setdefault("BSQ_XCHG_TIMEOUT_S", "180")

import argparse  # noqa: E402
import ctypes  # noqa: E402
import json  # noqa: E402
import time  # noqa: E402

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from bioseqdb_amd import synth  # noqa: E402
from bioseqdb_amd import _native as N  # noqa: E402

METRIC = "aligned reads/sec (150 bp vs 100 Mbp ref) at 1/2/4/8 MI355X; bit-exact vs libbwa"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# stage -> the main-pass kernel its HIP events bracket (libbsq run_stages)
STAGE_KERNEL = {"smem": "k_codes_wave+k_smem_lds",
                "chain": "k_chain_s+k_chain", "extend": "k_ext_key+sort+k_extend",
                "reg2aln": "k_r2a_key+sort+k_reg2aln_diag+g16+g32+w"}
# per-launch HBM traffic from the committed PMC passes (tools/profile_round.sh + tools/traffic_from_pmc.py,
# FETCH_SIZE corrected by the calib_fetch.hip gather calibration); PMC cannot be collected in-process
TRAFFIC_JSON = {"c3": os.path.join(ROOT, "profiles", "traffic.json"),
                "c2": os.path.join(ROOT, "profiles", "traffic_c2.json"),
                "c4": os.path.join(ROOT, "profiles", "traffic_c4.json")}


def traffic_for(stage: str, reads: int, config: str = "c3"):
    """PMC traffic of `stage` scaled to a launch of `reads` reads (the committed per-launch figure of the
    profiled lone launches), and the profile round it comes from."""
    try:
        t = json.load(open(TRAFFIC_JSON[config]))
        k = t["kernels"][stage]
        return k["traffic_bytes"] * reads / t["reads_per_launch"], t["round"]
    except (OSError, KeyError, ValueError):
        return None, None


# VALU lane-instruction issue peak: 256 CUs x 4 SIMDs x 32 lanes per clock x 2.4 GHz (MI355X_MICROARCH.md: 157.3 TFLOPS
# FP32 vector = this rate x 2 flops per FMA)
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9
# VALU instructions per ksw_extend2 DP cell in k_extend<true, 1>: the cell loop is unrolled by two and holds 59 VALU
# (+6 SALU, +6 LDS) instructions (tools/dp_cell_isa.py counts them in the gfx950 ISA)
EXT_VALU_PER_CELL = 29.5
SQ_JSON = {c: os.path.join(ROOT, "profiles", f"sq_{c}.json") for c in ("c2", "c3", "c4")}


def sq_for(config: str):
    try:
        return json.load(open(SQ_JSON[config]))
    except (OSError, KeyError, ValueError):
        return None


def valu_roofline(cells: float, lone_ms: float, sq) -> dict:
    """The extension's VALU roofline: the DP cells of one lone launch x VALU instructions per cell (the useful lane
    instructions) over the launch time, against the VALU lane-issue peak; SQ lane utilisation beside it."""
    useful = cells * EXT_VALU_PER_CELL
    rate = useful / (lone_ms * 1e-3)
    return {"bound": "valu", "dp_cells_per_launch": cells, "valu_per_cell": EXT_VALU_PER_CELL,
            "achieved": round(rate / 1e12, 3), "peak": round(VALU_PEAK_LANE_OPS / 1e12, 2), "unit": "T lane-instr/s",
            "frac": round(rate / VALU_PEAK_LANE_OPS, 4),
            "sq_lane_util": (sq or {}).get("valu_lane_util"), "sq_valu_busy": (sq or {}).get("valu_busy")}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Heartbeat:
    """A line on stderr every `period` s naming the current phase (long C4 setups stay visibly alive)."""

    def __init__(self, tag: str, period: float = 60.0):
        import threading
        self.phase, self.t0, self.tag = "start", time.time(), tag
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._run, args=(period,), daemon=True)
        self._th.start()

    def _run(self, period):
        while not self._stop.wait(period):
            log(f"[{self.tag}] {self.phase} ... {time.time() - self.t0:.0f}s")

    def stop(self):
        self._stop.set()


def json_out():
    """The bench's stdout carries only its one JSON line: fd 1 is pointed at stderr for the rest of the process
    (RCCL prints version banners on stdout when communicators initialise) and the line goes to a saved copy."""
    global _OUT
    if _OUT is None:
        sys.stdout.flush()
        _OUT = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)
    return _OUT


_OUT = None


def host_cpus() -> dict:
    """The host cores this process may use: the affinity mask, capped by the cgroup CPU quota (the GPU
    box's quota is 16 CPUs of a 256-thread host, which nproc reports), plus the CPU model."""
    n_aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"usable": min(n_aff, quota) if quota else n_aff, "affinity_cpus": n_aff, "cgroup_quota_cpus": quota,
            "machine_cpus": os.cpu_count(), "model": model}


def default_opts(n_refs: int) -> N.Opts:
    # effective SQL defaults incl. the bwa_opts() field-order quirk (Q1): e_del=6, o_ins=1
    return N.Opts(19, max(500, 2 * n_refs), 1, 4, 5, 5, 100, 100, 6, 6, 1, 1)


CONFIGS = {
    "c1": dict(reads=10_000, ref_bp=1_000_000, rows=1, seeding=False, metric=METRIC,
               label="C1: 10k 150 bp reads vs 1 Mbp synthetic reference, full seed + extension + CIGAR (BASELINE.json "
                     "configs[0]: the reference's own CPU-runnable case; latency-bound at this size)"),
    "c3": dict(reads=1_000_000, ref_bp=100_000_000, rows=1, seeding=False, metric=METRIC,
               label="C3: 150 bp reads vs 100 Mbp synthetic reference, full seed + banded SW extension + CIGAR "
                     "(BASELINE.json configs[2]); bwa_opts() SQL defaults"),
    "c2": dict(reads=1_000_000, ref_bp=100_000_000, rows=1, seeding=True,
               metric="seeded reads/sec (150 bp vs 100 Mbp ref, FM-index seeding only) on 1 MI355X",
               label="C2: 150 bp reads vs 100 Mbp synthetic reference, FM-index seeding only (mem_collect_intv: "
                     "SMEM passes 1+2 + seed strategy; BASELINE.json configs[1]); intervals left in HBM"),
    "c4": dict(reads=10_000_000, ref_bp=3_000_000_000, rows=24, seeding=False,
               metric="aligned reads/sec (150 bp vs 3 Gbp ref) on 1 MI355X; bit-exact vs libbwa",
               label="C4: 150 bp reads vs a 3 Gbp synthetic reference (24 rows x 125 Mbp; 64-bit rows), full "
                     "seed + extension + CIGAR (BASELINE.json configs[3]); 1M-read workspace chunks"),
}

_FNV_P = np.uint64(0x100000001B3)


def fnv_vec(h: np.ndarray, v: np.ndarray) -> np.ndarray:
    v = v.astype(np.uint64)
    with np.errstate(over="ignore"):
        for i in range(8):
            h = (h ^ ((v >> np.uint64(8 * i)) & np.uint64(0xFF))) * _FNV_P
    return h


# bsq_hit as a numpy record (np.ctypeslib on a ctypes.Structure pointer warns about its PEP 3118 format)
HIT_DTYPE = np.dtype({"names": [f[0] for f in N.Hit._fields_],
                      "formats": [np.dtype(f[1]) for f in N.Hit._fields_],
                      "offsets": [getattr(N.Hit, f[0]).offset for f in N.Hit._fields_],
                      "itemsize": ctypes.sizeof(N.Hit)})


def hits_array(ptr, n: int) -> np.ndarray:
    buf = (ctypes.c_uint8 * (n * ctypes.sizeof(N.Hit))).from_address(ctypes.addressof(ptr.contents))
    return np.frombuffer(buf, dtype=HIT_DTYPE, count=n)


def gpu_checksum_vec(H, n_reads: int, read_base: int = 0) -> int:
    """The oracle's orc_align_batch checksum (per-read FNV, summed), vectorised over reads; the batch's
    read r is read read_base + r of the oracle's run."""
    off = np.ctypeslib.as_array(H.read_off, shape=(n_reads + 1,)).astype(np.int64)
    nh = int(off[n_reads] - off[0])
    hits = hits_array(H.hits, nh) if nh else None
    ncig = int(H.n_cigar)
    cig = np.ctypeslib.as_array(H.cigar, shape=(max(ncig, 1),)) if ncig else np.zeros(1, np.uint32)
    h = fnv_vec(np.full(n_reads, 0xCBF29CE484222325, dtype=np.uint64),
                np.arange(read_base, read_base + n_reads, dtype=np.uint64))
    cnt = off[1:] - off[:-1]
    for k in range(int(cnt.max()) if n_reads else 0):
        m = cnt > k
        x = hits[(off[:-1][m] + k) - off[0]]
        hm = h[m]
        for col in (x["rb"].astype(np.int64).view(np.uint64), x["re"].astype(np.int64).view(np.uint64),
                    x["qb"].astype(np.uint32), x["qe"].astype(np.uint32), x["score"].astype(np.uint32),
                    np.where(x["is_secondary"] != 0, 0x100, 0).astype(np.uint64)):
            hm = fnv_vec(hm, col)
        nc = x["n_cigar"].astype(np.int64)
        co = x["cigar_off"].astype(np.int64)
        for c in range(int(nc.max()) if len(nc) else 0):
            mc = nc > c
            hm[mc] = fnv_vec(hm[mc], cig[co[mc] + c])
        h[m] = hm
    with np.errstate(over="ignore"):
        return int(h.sum(dtype=np.uint64))


def intv_checksum_vec(off: np.ndarray, iv: np.ndarray, n_reads: int) -> int:
    """The oracle's orc_seed_batch checksum over (x[0], x[2], info), vectorised over reads."""
    h = fnv_vec(np.full(n_reads, 0xCBF29CE484222325, dtype=np.uint64), np.arange(n_reads, dtype=np.uint64))
    cnt = off[1:n_reads + 1] - off[:n_reads]
    for k in range(int(cnt.max()) if n_reads else 0):
        m = cnt > k
        row = iv[off[:n_reads][m] + k]
        hm = h[m]
        for col in (row[:, 0], row[:, 2], row[:, 3]):
            hm = fnv_vec(hm, col)
        h[m] = hm
    with np.errstate(over="ignore"):
        return int(h.sum(dtype=np.uint64))


def fnv(h: int, v: int) -> int:
    for i in range(8):
        h ^= (v >> (8 * i)) & 0xFF
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def gpu_checksum(hits: "N.Hits", n_reads: int) -> int:
    """Same per-read FNV hash the oracle's orc_align_batch computes (order-independent sum)."""
    H = hits
    ck = 0
    for r in range(n_reads):
        h = fnv(0xCBF29CE484222325, r)
        for k in range(H.read_off[r], H.read_off[r + 1]):
            x = H.hits[k]
            for v in (x.rb, x.re, x.qb & 0xFFFFFFFF, x.qe & 0xFFFFFFFF, x.score & 0xFFFFFFFF,
                      0x100 if x.is_secondary else 0):
                h = fnv(h, v & 0xFFFFFFFFFFFFFFFF)
            for c in range(x.n_cigar):
                h = fnv(h, H.cigar[x.cigar_off + c])
        ck = (ck + h) & 0xFFFFFFFFFFFFFFFF
    return ck


def reads_as_nuclseq(L, reads):
    """nuclseq varlenas of the batch's reads (sequence.h:18-38), for the host rendering measurement: the
    reads without N packed in numpy (padding bases as nuclseq_from_text draws them), the rest through
    bsq_nuclseq_from_text.  Returns (buffers to keep alive, ctypes array of pointers)."""
    n = reads.n
    lens = np.diff(reads.offsets)
    ptrs = (ctypes.c_void_p * max(n, 1))()
    keep = []
    L0 = int(lens[0]) if n else 0
    plain = np.zeros(n, dtype=bool)
    if n and L0 and (lens == L0).all():
        codes = reads.codes.reshape(n, L0)
        plain = (codes < 4).all(axis=1)
        nb = (L0 + 3) // 4
        pad = np.zeros((n, nb * 4), dtype=np.uint8)
        pad[:, :L0] = codes
        x = L0 % 2147483647 or 1   # std::minstd_rand(holes_num ^ len) with no holes
        for j in range(L0, nb * 4):
            x = x * 48271 % 2147483647
            pad[:, j] = x & 3
        q = pad.reshape(n, nb, 4).astype(np.uint8)
        pac = (q[:, :, 0] << 6 | q[:, :, 1] << 4 | q[:, :, 2] << 2 | q[:, :, 3]).astype(np.uint8)
        size = 12 + nb
        buf = np.zeros((n, size), dtype=np.uint8)
        buf[:, 0:4] = np.frombuffer(np.uint32(size << 2).tobytes(), np.uint8)
        buf[:, 8:12] = np.frombuffer(np.uint32(L0).tobytes(), np.uint8)
        buf[:, 12:] = pac
        keep.append(buf)
        base = buf.ctypes.data
        for i in np.nonzero(plain)[0]:
            ptrs[int(i)] = base + int(i) * size
    for i in np.nonzero(~plain)[0]:
        t = reads.text(int(i)).encode()
        size = ctypes.c_size_t()
        p = L.bsq_nuclseq_from_text(t, len(t), ctypes.byref(size))
        b = ctypes.create_string_buffer(ctypes.string_at(p, size.value), size.value)
        L.bsq_free(p)
        keep.append(b)
        ptrs[int(i)] = ctypes.addressof(b)
    return keep, ptrs


def lone_launch(L, idx, opts, codes, offs, n, first_call):
    """Every stage of the path as one lone launch over n reads (one batch, nothing else on the GPU), after a
    warm-up run: per-stage HIP-event ms and issued bytes on the batch stream."""
    wb = ctypes.c_void_p()
    N.check(L.bsq_batch_create(idx, n, int(offs[n] - offs[0]), ctypes.byref(wb)))
    try:
        N.check(L.bsq_batch_set_reads(wb, codes.ctypes.data, offs.ctypes.data, n))
        for _ in range(2):   # warm-up + measured
            N.check(L.bsq_batch_run(wb, ctypes.byref(opts), first_call))
        ms = (ctypes.c_float * 6)()
        L.bsq_batch_stage_ms(wb, ms, 6)
        by = (ctypes.c_double * 6)()
        L.bsq_batch_stage_bytes(wb, by, 6)
        wk = (ctypes.c_double * 6)()
        L.bsq_batch_stage_work(wb, wk, 6)
        return [float(x) for x in ms], [float(x) for x in by], [float(x) for x in wk]
    finally:
        L.bsq_batch_free(wb)


def oracle_index(L, idx, ref_ns):
    """The CPU oracle's index over the same reference rows, its FM tables from the device-built suffix array
    (the checker for parity and the CPU baseline; test infrastructure, never on the product path).  The SA is
    certified twice before the oracle uses it, so the two sides cannot share a wrong one: on the device
    (bsq_index_certify_sa) and on the host by the oracle itself (range, one primary row, adjacent suffixes
    strictly increasing).  Both certificates go into SA_CERT (the line's `sa_certificate`)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O
    oi = O.OracleIndex()
    for buf in ref_ns:
        oi.add_ref(len(oi._keep) + 1, bytes(buf.raw))
    n_suf, bad = ctypes.c_uint64(), ctypes.c_uint64()
    t0 = time.perf_counter()
    N.check(L.bsq_index_certify_sa(idx, ctypes.byref(n_suf), ctypes.byref(bad)))
    SA_CERT["device"] = {"suffixes": int(n_suf.value), "violations": int(bad.value),
                         "s": round(time.perf_counter() - t0, 3)}
    if bad.value:
        raise SystemExit(f"device SA certificate: {bad.value} violations over {n_suf.value} suffixes")
    eb = ctypes.c_int()
    N.check(L.bsq_index_download(idx))   # host copy of the SA for the oracle's index
    sa = L.bsq_index_sa_data(idx, ctypes.byref(eb))
    SA_CERT["host"] = oi.build_from_sa(sa, eb.value)
    return O, oi


SA_CERT = {}


def cpu_baseline(O, oi, oo, codes, offs, n_reads, threads, seeding, seconds, first_call):
    """The oracle timed on this host: a warm-up that sizes the sample, then the median of 3 runs
    on `threads` threads (~seconds/3 each) and the median of 3 single-thread runs (~seconds/6 each)."""
    def run(n, th):
        ck = ctypes.c_uint64()
        t = time.perf_counter()
        if seeding:
            nreg = O.lib().orc_seed_batch(oi.h, ctypes.byref(oo), codes.ctypes.data, offs.ctypes.data, n, th,
                                          ctypes.byref(ck))
        else:
            nreg = O.lib().orc_align_batch(oi.h, ctypes.byref(oo), codes.ctypes.data, offs.ctypes.data, n, first_call,
                                           th, ctypes.byref(ck))
        return time.perf_counter() - t, nreg, ck.value

    n0 = min(2000, n_reads)
    dt, _, _ = run(n0, threads)
    sample = int(min(n_reads, max(n0, n0 / max(dt, 1e-6) * seconds / 3)))
    times = []
    for _ in range(3):
        dt, nreg, ck = run(sample, threads)
        times.append(dt)
    ab = (ctypes.c_uint64 * 4)()
    O.lib().orc_algo_bytes(ab)   # SURVEY.md 8(d) bytes of the sample, counted on libbwa's layout
    m0 = min(300, n_reads)
    dt, _, _ = run(m0, 1)
    n1 = int(min(n_reads, max(m0, m0 / max(dt, 1e-6) * seconds / 6)))
    times1 = [run(n1, 1)[0] for _ in range(3)]
    med, med1 = sorted(times)[1], sorted(times1)[1]
    return {"sample": sample, "times": times, "nreg": nreg, "ck": ck, "ab": list(ab), "n1": n1, "times1": times1,
            "value": round(sample / med, 1), "value_1thread": round(n1 / med1, 1)}


def exchange_budget(L, idx, batches, step_ms: float) -> dict:
    """The torchrun exchange's ingress at rank 0 (the rows of every rank reach the caller's
    tuplestore, bioseqdb/extension.cpp:362-370), budgeted from one GPU: this rank's records of one step in the wire
    form the exchange sends (bsq_xchg_wire_check: the send path's device pack, rank 0's host expansion, compared
    byte for byte with the batch's view) and as bsq_hit records, and the measured pinned D2H rate of one PCIe link --
    rank 0's link carries the 7 peers' wire records plus its own records at 8 GPUs."""
    wire = raw = bad = 0
    for b in batches:
        wb, rb, mm = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        N.check(L.bsq_xchg_wire_check(b, idx, ctypes.byref(wb), ctypes.byref(rb), ctypes.byref(mm)))
        wire += wb.value
        raw += rb.value
        bad += mm.value
    # the HIP runtime libbsq already uses (torch's lazy CUDA init is not safe here after the batches' HIP use)
    hip = ctypes.CDLL("libamdhip64.so.7")   # libbsq's DT_NEEDED: the same loaded runtime
    nbytes, reps = 256 << 20, 8
    src, dst = ctypes.c_void_p(), ctypes.c_void_p()
    if hip.hipMalloc(ctypes.byref(src), ctypes.c_size_t(nbytes)) or hip.hipHostMalloc(ctypes.byref(dst), ctypes.c_size_t(nbytes), 0):
        raise RuntimeError("exchange budget: HIP allocation failed")
    D2H = 2   # hipMemcpyDeviceToHost
    hip.hipMemcpy(dst, src, ctypes.c_size_t(nbytes), D2H)
    t = time.perf_counter()
    for _ in range(reps):
        if hip.hipMemcpy(dst, src, ctypes.c_size_t(nbytes), D2H):
            raise RuntimeError("exchange budget: hipMemcpy failed")
    rate = reps * nbytes / (time.perf_counter() - t)
    hip.hipFree(src)
    hip.hipHostFree(dst)
    out = {"bytes_per_step_rank_wire": wire, "bytes_per_step_rank_raw": raw,
           "wire_saving": round(1 - wire / raw, 3) if raw else None, "wire_roundtrip_mismatches": bad,
           "d2h_pinned_GBps": round(rate / 1e9, 2), "step_ms_1gpu": round(step_ms, 3)}
    for n in (2, 4, 8):   # rank 0's link: (n - 1) peers' wire records + its own records, per step
        ing = (n - 1) * wire + raw
        out[f"rank0_ingress_{n}gpu"] = {"bytes_per_step": ing, "d2h_ms_per_step": round(ing / rate * 1e3, 3),
                                        "frac_of_step": round(ing / rate * 1e3 / step_ms, 3),
                                        "raw_records_d2h_ms": round(n * raw / rate * 1e3, 3)}
    return out


def make_roofline(dom, di, stage_ms, stage_bytes, reads_per_launch, iso, iso_reads, per_read, tr, S):
    """The bench line's `roofline` for the dominant stage: the lone launch over all the step's reads when there
    is one (the kernel's own time), with the shared-CU figure of the timed concurrent batches beside it.
    `achieved` = SURVEY.md 8(d) algorithmic bytes per launch (oracle-counted per read x reads) / launch time."""
    def fig(ms, issued, n):
        d = {"reads_per_launch": int(round(n)), "launch_ms": round(ms, 3), "issued_bytes_per_launch": issued,
             "issued_gbs": round(issued / (ms * 1e-3) / 1e9, 2) if ms > 0 else 0.0}
        alg = per_read[di] * n if per_read else issued
        d["algorithmic_bytes_per_launch"] = alg
        d["achieved"] = round(alg / (ms * 1e-3) / 1e9, 2) if ms > 0 else 0.0
        d["frac"] = round(d["achieved"] / HBM_PEAK_GBS, 5)
        return d
    conc = fig(float(stage_ms[di]), float(stage_bytes[di]), reads_per_launch)
    head = fig(float(iso[0][di]), float(iso[1][di]), iso_reads) if iso else conc
    t, t_round = tr(dom, head["reads_per_launch"])
    roof = {"bound": "hbm", "kernel": STAGE_KERNEL[dom], "peak": HBM_PEAK_GBS, "unit": "GB/s", **head,
            "traffic": t,
            # the HBM bytes the launch really moved (PMC) per second of the same launch, as a fraction of peak
            "traffic_frac": (round(t / (head["launch_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                             if t and head["launch_ms"] > 0 else None),
            "traffic_source": (f"{t_round} rocprofv3 PMC FETCH_SIZE + WRITE_SIZE passes of lone launches, per launch"
                               if t else "not measured for this shape"),
            "basis": ("lone launch: one batch of all the step's reads with nothing else on the GPU (HIP events on the "
                      "batch stream)" if iso else f"{S} concurrent batches (no lone launch in this run)"),
            "bytes": "SURVEY.md 8(d) algorithmic bytes" if per_read else "bytes the kernels issue (no oracle sample)"}
    if iso and S > 1:
        roof["concurrent"] = dict(conc, note=f"{S} concurrent batches of the timed step: the kernel's duration while it "
                                             "shares the CUs with the other batches' stages")
    return roof


def run_group(args, cfg) -> int:
    """--gpus N from one process (no launcher): the devices driven the way a Postgres backend drives them
    (bsq_group): the index built once on the first device and broadcast over RCCL, member k
    aligning its own reads (seed READ_SEED + k, weak scaling) as concurrent shares on its device, each member's
    records copied to pinned host memory over its own PCIe link.  One step = one bsq_group_run over the
    members' reads already staged on their devices; it ends when every record is in host memory (segments in
    read order).  The merged single view is timed separately (`merge_ms`)."""
    L = N.lib()
    G = args.gpus if not args.group_devices else len(args.group_devices.split(","))
    devs = [int(x) for x in args.group_devices.split(",")] if args.group_devices else list(range(G))
    if args.gpus > 1 and len(devs) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but --group-devices lists {len(devs)} members")
    ndev = L.bsq_device_count()
    if ndev < max(devs) + 1:
        raise SystemExit(f"--gpus {G}: {ndev} HIP device(s) visible, devices {devs} requested")
    if cfg["seeding"]:
        raise SystemExit("the device group runs the full path (configs c3/c4)")
    hb = Heartbeat("bench group")
    hb.phase = "generating the reference and reads"
    ref = synth.make_reference(args.ref_bp, n_rows=cfg["rows"])
    member_reads = [synth.make_reads(ref, args.reads, length=args.read_len, seed=synth.READ_SEED + k + args.seed_offset)
                    for k in range(G)]
    idx = ctypes.c_void_p()
    N.check(L.bsq_index_create(ctypes.byref(idx)))
    ref_ns = []
    for i, t in enumerate(ref.texts()):
        size = ctypes.c_size_t()
        p = L.bsq_nuclseq_from_text(t, len(t), ctypes.byref(size))
        buf = ctypes.create_string_buffer(ctypes.string_at(p, size.value), size.value)
        L.bsq_free(p)
        ref_ns.append(buf)
        N.check(L.bsq_index_add_ref(idx, i + 1, ctypes.addressof(buf)))
    hb.phase = "building the index on the first member's GPU"
    t0 = time.time()
    N.check(L.bsq_index_build_device(idx, devs[0]))
    t_build = time.time() - t0
    opts = default_opts(int(L.bsq_index_n_refs(idx)))
    g = ctypes.c_void_p()
    darr = (ctypes.c_int * G)(*devs)
    N.check(L.bsq_group_create(darr, G, ctypes.byref(g)))
    N.check(L.bsq_group_set_slots(g, max(1, args.streams)))
    via_first = args.exchange == "via-first"
    N.check(L.bsq_group_set_exchange(g, 1 if via_first else 0))
    hb.phase = "replicating the index over the group"
    bc_ms = ctypes.c_double()
    N.check(L.bsq_group_replicate(g, idx, ctypes.byref(bc_ms)))
    # the members' reads as one cursor batch of nuclseq varlenas (member k: reads [k*n, (k+1)*n))
    keep, n_tot = [], G * args.reads
    ptrs = (ctypes.c_void_p * n_tot)()
    for k, r in enumerate(member_reads):
        kk, pk = reads_as_nuclseq(L, r)
        keep += [kk, pk]
        ctypes.memmove(ctypes.addressof(ptrs) + k * args.reads * ctypes.sizeof(ctypes.c_void_p), pk,
                       args.reads * ctypes.sizeof(ctypes.c_void_p))
    first_call = args.seed_offset * args.reads
    hb.phase = "aligning"
    N.check(L.bsq_group_run(g, ctypes.byref(opts), ptrs, n_tot, first_call))   # stages every member's reads
    if args.warmup > 1:
        N.check(L.bsq_group_run_rounds(g, ctypes.byref(opts), n_tot, first_call, args.warmup - 1))
    # the timed steps: by default one stream of rounds per member (bsq_group_run_rounds: each share starts its next
    # step as soon as its previous one is taken -- the N = 1 line's schedule); --lockstep: a group run per step
    t0 = time.perf_counter()
    if args.lockstep:
        for _ in range(args.steps):
            N.check(L.bsq_group_run(g, ctypes.byref(opts), None, n_tot, first_call))
    else:
        N.check(L.bsq_group_run_rounds(g, ctypes.byref(opts), n_tot, first_call, args.steps))
    elapsed = time.perf_counter() - t0
    t1 = time.perf_counter()
    H = L.bsq_group_hits(g)
    merge_ms = (time.perf_counter() - t1) * 1e3
    if not H:
        raise N.BsqError(N.BSQ_E_NOMEM, L.bsq_last_error().decode())
    H = H.contents
    value = n_tot * args.steps / elapsed
    segs = (ctypes.POINTER(N.Hits) * 1024)()
    slo = (ctypes.c_int32 * 1024)()
    n_seg = L.bsq_group_segments(g, segs, slo, 1024)
    result = {
        "metric": cfg["metric"], "value": round(value, 1), "unit": "reads/s", "n_gpus": G, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int32", "data": "synthetic",
        "config": {
            "workload": cfg["label"], "reads_per_gpu": args.reads, "read_len": args.read_len, "ref_bp": args.ref_bp,
            "parallelism": f"read-sharded x{G} in one process (bsq_group: index broadcast over RCCL, each member's "
                           "records to host memory over its own PCIe link)",
            "devices": devs, "distinct_devices": len(set(devs)), "shares_per_member": max(1, args.streams),
            "segments": n_seg, "hits_per_step": int(H.n_hits),
            "step_schedule": ("barrier after every step (bsq_group_run per step)" if args.lockstep else
                              "stream of rounds per member share over the timed steps (bsq_group_run_rounds)"),
        },
        "exchange": {"path": ("members' records by peer DMA over xGMI into member 0's HBM, then member 0's PCIe D2H, "
                              "inside the step (BSQ_XCHG_VIA_FIRST)" if via_first else
                              "each member's records over its own PCIe link, pinned D2H inside the step "
                              "(BSQ_XCHG_LINKS)") + "; segments in read order, merged view after the timed region",
                     "mode": args.exchange, "merge_ms": round(merge_ms, 3), "broadcast_ms": round(bc_ms.value, 2),
                     "record_bytes_per_step": int(H.n_hits) * ctypes.sizeof(N.Hit) + int(H.n_cigar) * 4},
        "index_build_s": round(t_build, 2),
    }
    if args.checksums:   # member k's rows with member-local read indices (= a one-GPU run with --seed-offset k)
        cks = [0] * G
        for i in range(n_seg):
            k = slo[i] // args.reads
            v = segs[i].contents
            cks[k] += gpu_checksum_vec(v, int(v.n_reads), slo[i] - k * args.reads)
        result["checksums"] = [c & 0xFFFFFFFFFFFFFFFF for c in cks]
    # parity of the first and the last member against the CPU oracle on a sample of their reads, and SURVEY.md
    # 8(d)'s per-read bytes counted on it (a check, not a CPU baseline: that is the N = 1 line's)
    per_read = None
    if not args.no_cpu_baseline:
        hb.phase = "oracle parity sample"
        O, oi = oracle_index(L, idx, ref_ns)
        oo = O.opts_from(opts)
        th = host_cpus()["usable"]
        par = []
        for k in sorted({0, G - 1}):
            r = member_reads[k]
            m = min(2000, r.n)
            c_ = np.ascontiguousarray(r.codes)
            o_ = np.ascontiguousarray(r.offsets)
            ck = ctypes.c_uint64()
            O.lib().orc_align_batch(oi.h, ctypes.byref(oo), c_.ctypes.data, o_.ctypes.data, m,
                                    first_call + k * args.reads, th, ctypes.byref(ck))
            if k == 0:
                ab = (ctypes.c_uint64 * 4)()
                O.lib().orc_algo_bytes(ab)
                per_read = [ab[0] / m + (args.read_len + 3) // 4, ab[1] / m, ab[2] / m, ab[3] / m]
            gck = 0
            for i in range(n_seg):
                loc = slo[i] - k * args.reads   # segment start within member k
                if slo[i] // args.reads != k or loc >= m:
                    continue
                v = segs[i].contents
                gck += gpu_checksum_vec(v, min(int(v.n_reads), m - loc), loc)
            par.append({"member": k, "reads": m, "checksum_match": (gck & 0xFFFFFFFFFFFFFFFF) == ck.value})
        result["parity_sample"] = par
    # roofline of the dominant stage: member 0's reads as one lone launch on its device
    hb.phase = "isolated single-batch launch"
    r0 = member_reads[0]
    codes = np.ascontiguousarray(r0.codes)
    offs = np.ascontiguousarray(r0.offsets)
    names = [L.bsq_stage_name(i).decode() for i in range(6)]
    iso = None if args.no_isolated else lone_launch(L, idx, opts, codes, offs, r0.n, first_call)
    if iso:
        di = max(range(4), key=lambda i: iso[0][i])
        tr = (lambda stage, n: traffic_for(stage, n, args.config)) if (args.reads == cfg["reads"] and args.ref_bp == cfg["ref_bp"]) \
            else (lambda stage, n: (None, None))
        result["roofline"] = make_roofline(names[di], di, iso[0], iso[1], r0.n, iso, r0.n, per_read, tr, 1)
        result["kernels"] = {STAGE_KERNEL[names[i]]: {"lone_ms": round(iso[0][i], 3)} for i in range(4)}
    hb.stop()
    if SA_CERT:
        result["sa_certificate"] = dict(SA_CERT)
    # introsort scans stopped by the bound rather than the sentinel over every run in this process (must be 0)
    result["sort_guard"] = int(L.bsq_sort_guard_total())
    print(json.dumps(result), file=json_out(), flush=True)
    L.bsq_group_free(g)
    L.bsq_index_free(idx)
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS),
                    help="c3 (default, the BASELINE metric), c2 (seeding only), c4 (3 Gbp reference)")
    ap.add_argument("--reads", type=int, default=None, help="reads per GPU per step (default: the config's)")
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--ref-bp", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-codec", action="store_true", help="skip the bulk nuclseq codec measurement")
    ap.add_argument("--no-isolated", action="store_true",
                    help="skip the untimed lone launch of the dominant stage")
    ap.add_argument("--timed-only", action="store_true",
                    help="only the timed steps (profiling passes): no CPU baseline, codec, isolated launch, rendering "
                         "or one-shot call, so every dispatch of a stage kernel is a timed-step launch")
    ap.add_argument("--streams", type=int, default=4,
                    help="concurrent batches per GPU (bsq_batch_run_many); each aligns 1/S of the reads")
    ap.add_argument("--index-build", default="device", choices=["device", "host"],
                    help="where the index is built before the timed region (device: bsq_index_build_device)")
    ap.add_argument("--exchange-world1", action="store_true",
                    help="run the N > 1 exchange path with a process group of one rank (tests it on a one-GPU box)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1 exchange backend (nccl = RCCL over xGMI; gloo only to rehearse on one GPU)")
    ap.add_argument("--group-devices", default=None,
                    help="in-process group (--gpus N without torchrun): comma-separated device of each member "
                         "(default 0..N-1; a repeated device makes replicas on one GPU, for tests)")
    ap.add_argument("--exchange", default="links", choices=["links", "via-first"],
                    help="in-process group: records to host over every member's own link (links) or gathered over "
                         "xGMI into member 0 first (via-first)")
    ap.add_argument("--lockstep", action="store_true",
                    help="a barrier after every timed step (bsq_batch_run_many per step) instead of one stream of "
                         "batch runs over the K steps")
    ap.add_argument("--cursor-only", action="store_true",
                    help="after the timed steps, only the pipelined cursor measurement (profiling the drop-in loop)")
    ap.add_argument("--cursor-depth", type=int, default=16,
                    help="fetches in flight in the sql_cursor measurement (BwaIndex::pipeline_depth's default)")
    ap.add_argument("--seed-offset", type=int, default=0,
                    help="rank (or member) k aligns the reads of seed READ_SEED + k + offset, lrand48 position "
                         "(k + offset) * reads: lets a one-GPU run reproduce any member of a multi-GPU run")
    ap.add_argument("--checksums", action="store_true",
                    help="add the oracle-format checksum of every rank/member's full read set to the line")
    args = ap.parse_args()
    json_out()
    if args.timed_only:
        args.no_cpu_baseline = args.no_codec = args.no_isolated = True
    if args.cursor_only:
        args.no_cpu_baseline = args.no_codec = args.no_isolated = True
    cfg = CONFIGS[args.config]
    args.reads = args.reads or cfg["reads"]
    args.ref_bp = args.ref_bp or cfg["ref_bp"]
    default_shape = args.reads == cfg["reads"] and args.ref_bp == cfg["ref_bp"]

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and (args.gpus > 1 or args.group_devices) and not args.exchange_world1:
        # N GPUs from one process, the way a Postgres backend drives them (bsq_group): no torchrun needed
        return run_group(args, cfg)
    if world > 1 and args.gpus not in (1, world):
        raise SystemExit(f"--gpus {args.gpus} under a launcher with WORLD_SIZE={world}: one rank per GPU expected")
    dist = None
    gpu = local
    xdev = None   # device of the exchange tensors
    if world > 1 or args.exchange_world1:
        import torch
        import torch.distributed as dist
        ndev = torch.cuda.device_count()   # does not initialise the GPU
        gpu = local % max(ndev, 1)         # one GPU per rank; several ranks share one only in a gloo rehearsal
        torch.cuda.set_device(gpu)
        if args.dist_backend == "nccl":
            xdev = torch.device("cuda", gpu)
            dist.init_process_group("nccl", device_id=xdev)
        else:
            xdev = torch.device("cpu")
            dist.init_process_group("gloo")
    L = N.lib()
    hb = Heartbeat(f"bench r{rank}")
    hb.phase = "generating the reference and reads"
    t0 = time.time()
    ref = synth.make_reference(args.ref_bp, n_rows=cfg["rows"])
    reads = synth.make_reads(ref, args.reads, length=args.read_len, seed=synth.READ_SEED + rank + args.seed_offset)
    t_gen = time.time() - t0

    # ---- index: built once (host, the step before the hot path), then in HBM on every GPU ----
    idx = ctypes.c_void_p()
    ref_ns = []
    t_build = 0.0
    if rank == 0:
        N.check(L.bsq_index_create(ctypes.byref(idx)))
        for i, t in enumerate(ref.texts()):
            size = ctypes.c_size_t()
            p = L.bsq_nuclseq_from_text(t, len(t), ctypes.byref(size))
            buf = ctypes.create_string_buffer(ctypes.string_at(p, size.value), size.value)
            L.bsq_free(p)
            ref_ns.append(buf)
            N.check(L.bsq_index_add_ref(idx, i + 1, ctypes.addressof(buf)))
        t0 = time.time()
        if args.index_build == "device":   # suffix sort + BWT in HBM, leaves it uploaded
            hb.phase = "building the index on the GPU"
            N.check(L.bsq_index_build_device(idx, gpu))
        else:
            hb.phase = "building the index on the host"
            N.check(L.bsq_index_build(idx, 0))
        t_build = time.time() - t0
    t0 = time.time()
    index_bufs = None
    if dist is None:
        hb.phase = "uploading the index"
        N.check(L.bsq_index_upload(idx, gpu))   # no-op for a device-built index
    else:   # one build, device tables broadcast to every rank (RCCL over xGMI)
        hb.phase = "replicating the index"
        from bioseqdb_amd import dist as D
        idx, index_bufs = D.replicate_index(L, idx if rank == 0 else None, gpu)
    t_upload = time.time() - t0
    opts = default_opts(int(L.bsq_index_n_refs(idx)))

    # ---- batches: reads resident in HBM before timing.  S batches over contiguous read ranges run
    # concurrently (bsq_batch_run_many: one stream + host thread each); the stages of one fill the tails
    # and host gaps of the others.  Every read is aligned exactly once per step. ----
    S = 1 if cfg["seeding"] else max(1, args.streams)
    lo_k = [reads.n * k // S for k in range(S + 1)]
    subs = [reads.subset(lo_k[k], lo_k[k + 1]) for k in range(S)]
    batches = []
    keep_arrays = []
    for sub in subs:
        b = ctypes.c_void_p()
        N.check(L.bsq_batch_create(idx, sub.n, int(sub.offsets[-1]), ctypes.byref(b)))
        c_ = np.ascontiguousarray(sub.codes)
        o_ = np.ascontiguousarray(sub.offsets)
        keep_arrays += [c_, o_]
        N.check(L.bsq_batch_set_reads(b, c_.ctypes.data, o_.ctypes.data, sub.n))
        batches.append(b)
    batch = batches[0]
    codes = np.ascontiguousarray(reads.codes)     # the whole batch, for the CPU baseline
    offs = np.ascontiguousarray(reads.offsets)
    # lrand48 stream position as one backend aligning all ranks' reads in order
    first_call = (rank + args.seed_offset) * reads.n
    b_arr = (ctypes.c_void_p * S)(*[b.value for b in batches])
    fc_arr = (ctypes.c_uint64 * S)(*[first_call + lo_k[k] for k in range(S)])
    log(f"[bench r{rank}] gen {t_gen:.1f}s index build {t_build:.1f}s upload {t_upload:.2f}s "
        f"seq_len {L.bsq_index_seq_len(idx)}")

    def step():
        if cfg["seeding"]:
            N.check(L.bsq_batch_seed(batch, ctypes.byref(opts)))
            return
        if S == 1:
            N.check(L.bsq_batch_run(batch, ctypes.byref(opts), first_call))
        else:
            N.check(L.bsq_batch_run_many(b_arr, S, ctypes.byref(opts), fc_arr))
        if dist is not None:   # exchange step: hit records + CIGARs of every rank to the caller (rank 0)
            if xchg.gpu:   # device records straight into the RCCL send buffer; the gather overlaps the next step
                sz = []
                for b in batches:   # batch order == read order
                    nb = ctypes.c_int64()
                    N.check(L.bsq_batch_copy_records(b, None, 0, ctypes.byref(nb)))
                    sz.append(nb.value)

                def fill(send):
                    off = 0
                    for b, nb in zip(batches, sz):
                        got = ctypes.c_int64()
                        N.check(L.bsq_batch_copy_records(b, ctypes.c_void_p(send.data_ptr() + off), nb, ctypes.byref(got)))
                        off += nb
                xchg.post_fill(sum(sz), fill)
            else:
                parts = []
                for b in batches:
                    H = L.bsq_batch_hits(b).contents
                    nb = H.n_hits * ctypes.sizeof(N.Hit)
                    nc = H.n_cigar * 4
                    parts.append(np.ctypeslib.as_array(ctypes.cast(H.hits, ctypes.POINTER(ctypes.c_uint8)), shape=(max(nb, 1),))[:nb])
                    parts.append(np.ctypeslib.as_array(ctypes.cast(H.cigar, ctypes.POINTER(ctypes.c_uint8)), shape=(max(nc, 1),))[:nc])
                xchg.post(parts)

    xchg = None    # the Python exchange (gloo rehearsal only)
    nx = None      # the native exchange: bsq_xchg lanes over RCCL, one per batch
    if dist is not None and args.dist_backend == "nccl" and not cfg["seeding"]:
        import torch
        IDB = 128   # BSQ_XCHG_ID_BYTES
        ids = torch.zeros(IDB, dtype=torch.uint8, device=xdev)
        if rank == 0:
            raw = ctypes.create_string_buffer(IDB)
            N.check(L.bsq_xchg_unique_id(raw))
            ids.copy_(torch.frombuffer(bytearray(raw.raw), dtype=torch.uint8))
        dist.broadcast(ids, src=0)
        idb = ctypes.create_string_buffer(bytes(ids.cpu().numpy()), IDB)
        nx = ctypes.c_void_p()
        hb.phase = "joining the exchange communicator"
        N.check(L.bsq_xchg_create(world, rank, gpu, idb, S, ctypes.byref(nx)))
        N.check(L.bsq_xchg_set_index(nx, idx))   # rank 0 expands the received wire records with its anns
    elif dist is not None:
        from bioseqdb_amd import dist as D
        xchg = D.RecordExchange(device=xdev)
    hb.phase = "aligning"
    moved0 = ctypes.c_int64()
    if nx is not None:
        N.check(L.bsq_batch_run_rounds_x(b_arr, S, ctypes.byref(opts), fc_arr, args.warmup, nx))
        N.check(L.bsq_xchg_finish(nx, ctypes.byref(moved0), None))
    else:
        for _ in range(args.warmup):
            step()
    if xchg is not None:
        xchg.finish()
    stage_ms = np.zeros(6)
    stage_bytes = np.zeros(6)
    stage_work = np.zeros(6)
    if dist is not None:
        import torch
        dist.barrier()
        torch.cuda.synchronize()
    # Without a launcher the K steps run as one stream of batch runs (bsq_batch_run_rounds): each batch starts
    # its next step as soon as its previous one ends, so one batch's seeding overlaps the others' DP tails
    # instead of every step draining to a barrier; every step still aligns all the reads once, and the last
    # step's records are checked below.  --lockstep: a barrier after every step (bsq_batch_run_many per step).
    # Under torchrun (RCCL) every rank runs the same stream of rounds, each batch's records going to rank 0 over its
    # exchange lane after every round (bsq_batch_run_rounds_x).
    rounds = (dist is None or nx is not None) and S > 1 and not cfg["seeding"] and not args.lockstep
    t0 = time.perf_counter()
    if rounds:
        N.check(L.bsq_batch_run_rounds_x(b_arr, S, ctypes.byref(opts), fc_arr, args.steps, nx))
    for _ in range(1 if rounds else args.steps):
        if not rounds:
            if nx is not None:
                N.check(L.bsq_batch_run_rounds_x(b_arr, S, ctypes.byref(opts), fc_arr, 1, nx))
                N.check(L.bsq_xchg_finish(nx, None, None))
            else:
                step()
        for b in batches:   # per-launch figures: averaged over the S concurrent launches of each stage
            ms = (ctypes.c_float * 6)()
            L.bsq_batch_stage_ms(b, ms, 6)
            by = (ctypes.c_double * 6)()
            L.bsq_batch_stage_bytes(b, by, 6)
            wk = (ctypes.c_double * 6)()
            L.bsq_batch_stage_work(b, wk, 6)
            stage_work += np.array(list(wk))
            stage_ms += np.array(list(ms))
            stage_bytes += np.array(list(by))
    moved1, xwait = ctypes.c_int64(), ctypes.c_double()
    if dist is not None:
        import torch
        if nx is not None:   # the last round's records of every rank are in rank 0's host memory
            N.check(L.bsq_xchg_finish(nx, ctypes.byref(moved1), ctypes.byref(xwait)))
        else:
            xchg.finish()   # the last step's records are on the caller's host
        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], device=xdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    stage_ms /= (1 if rounds else max(args.steps, 1)) * S   # rounds: the last step's launches
    stage_bytes /= (1 if rounds else max(args.steps, 1)) * S
    stage_work /= (1 if rounds else max(args.steps, 1)) * S
    reads_per_launch = reads.n / S
    n_hits = sum(int(L.bsq_batch_hits(b).contents.n_hits) for b in batches) if not cfg["seeding"] else 0
    retried = sum(int(L.bsq_batch_retried(b)) for b in batches)
    names = [L.bsq_stage_name(i).decode() for i in range(6)]
    nst = 1 if cfg["seeding"] else 4
    kern = {names[i]: float(stage_ms[i]) for i in range(nst)}
    # measured PMC traffic of lone launches (profiles/traffic*.json) exists for the default config shapes
    tr = (lambda stage, n: traffic_for(stage, n, args.config)) if default_shape else (lambda stage, n: (None, None))
    dom = max(kern, key=kern.get)
    di = names.index(dom)

    # the stages once more as one lone launch over all the reads (one batch, nothing sharing the CUs), outside
    # the timed region: each kernel's own roofline (the headline `roofline`), beside the shared-CU figures of
    # the timed concurrent batches.  With one batch per step the timed launches are lone launches already.
    iso = None
    if world == 1 and S > 1 and not cfg["seeding"] and not args.no_isolated:
        hb.phase = "isolated single-batch launch"
        iso = lone_launch(L, idx, opts, codes, offs, reads.n, first_call)
    elif S == 1:
        iso = (list(stage_ms), list(stage_bytes), list(stage_work))
    if iso:   # the dominant kernel by its own (lone) time: with steps as a stream, the batches' last-step stages
        di = max(range(nst), key=lambda i: iso[0][i])   # overlap in whatever phase they drifted to
        dom = names[di]

    total_reads = args.reads * world
    value = total_reads * args.steps / elapsed
    result = {
        "metric": cfg["metric"],
        "value": round(value, 1),
        "unit": "reads/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {
            "workload": cfg["label"],
            "reads_per_gpu": args.reads, "read_len": args.read_len, "ref_bp": args.ref_bp,
            "parallelism": f"read-sharded x{world}" + (" (one process per GPU, RCCL record gather)" if world > 1 else ""),
            "hits_per_step_rank0": n_hits, "streams": S, "reads_per_launch": int(round(reads_per_launch)),
            "step_schedule": ("stream of batch runs over the timed steps (bsq_batch_run_rounds; stage times of the "
                              "last step)" if rounds else "barrier after every step"),
        },
        "exchange": ({
            "path": ("bsq_xchg: one RCCL communicator and one exchange thread per rank issuing, in one fixed (round, lane) "
                     "order on every rank, an all-gather of the record counts + status, then every rank's read offsets, "
                     "hits and CIGAR words ncclSend/ncclRecv to rank 0 over xGMI and its pinned D2H there; a lane's next "
                     "round waits only for its own send"),
            "lanes": S, "bytes_per_step": int((moved1.value - moved0.value) / max(args.steps, 1)),
            "bytes_side": "received by rank 0" if rank == 0 else "sent by this rank",
            "host_wait_ms_per_step_per_lane": round(xwait.value / max(args.steps, 1) / S, 3),
        } if nx is not None else None if xchg is None else {
            "path": "gloo gather of host records to rank 0 (rehearsal)",
            "bytes_per_step_rank0": int(xchg.bytes_moved / max(args.steps + args.warmup, 1)) if rank == 0 else None,
        }),
        "kernels": {
            STAGE_KERNEL[nm]: {
                "ms": round(float(stage_ms[i]), 3), "issued_bytes": float(stage_bytes[i]),
                "issued_gbs": round(stage_bytes[i] / (stage_ms[i] * 1e-3) / 1e9, 2) if stage_ms[i] > 0 else 0.0,
                "lone_ms": round(float(iso[0][i]), 3) if iso else None,
                "lone_traffic_bytes": tr(nm, reads.n)[0],
                "lone_traffic_gbs": (round(tr(nm, reads.n)[0] / (iso[0][i] * 1e-3) / 1e9, 2)
                                     if iso and tr(nm, reads.n)[0] and iso[0][i] > 0 else None),
                "lone_traffic_frac": (round(tr(nm, reads.n)[0] / (iso[0][i] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                      if iso and tr(nm, reads.n)[0] and iso[0][i] > 0 else None),
                "work": float(stage_work[i]),
            } for i, nm in enumerate(names[:nst])
        },
        "stages_ms": {names[i]: round(float(stage_ms[i]), 3) for i in range(6)},
        "stages_issued_bytes": {names[i]: float(stage_bytes[i]) for i in range(6)},
        "stages_work": {names[i]: float(stage_work[i]) for i in range(6)},
        "index_build_s": round(t_build, 2),
        "index_build": args.index_build,
        "index_upload_s": round(t_upload, 2),
        "retried_reads": retried,
    }
    # SQ counters of lone launches (tools/sq_round.sh, committed under profiles/) and the extension's VALU roofline
    sq = sq_for(args.config) if default_shape else None
    for i, nm in enumerate(names[:nst]):
        k = result["kernels"][STAGE_KERNEL[nm]]
        if sq and nm in sq["stages"]:
            st = sq["stages"][nm]
            k["sq"] = {x: st[x] for x in ("valu_lane_util", "valu_busy", "wait_frac") if x in st}
            k["sq"]["round"] = sq["round"]
        if nm == "extend" and iso and len(iso) > 2 and iso[0][i] > 0:
            k["valu"] = valu_roofline(iso[2][i], iso[0][i], k.get("sq"))
    if args.checksums and not cfg["seeding"]:
        ck = 0
        for k, b in enumerate(batches):
            ck += gpu_checksum_vec(L.bsq_batch_hits(b).contents, lo_k[k + 1] - lo_k[k], lo_k[k])
        result["checksums"] = [ck & 0xFFFFFFFFFFFFFFFF]
        if nx is not None and rank == 0:   # every other rank's records as rank 0 received them (= a one-GPU run
            for r in range(1, world):      # with --seed-offset r)
                ck = 0
                for k in range(S):
                    v = N.Hits()
                    N.check(L.bsq_xchg_view(nx, k, r, ctypes.byref(v)))
                    ck += gpu_checksum_vec(v, lo_k[k + 1] - lo_k[k], lo_k[k])
                result["checksums"].append(ck & 0xFFFFFFFFFFFFFFFF)

    if world == 1 and not cfg["seeding"] and not args.timed_only:
        hb.phase = "exchange budget"
        result["exchange_budget"] = exchange_budget(L, idx, batches, elapsed / args.steps * 1e3)

    # ---- N > 1: the last rank's records as rank 0 received them, against the CPU oracle on a sample ----
    if nx is not None and world > 1 and rank == 0 and not args.no_cpu_baseline:
        hb.phase = "oracle parity sample of the exchanged records"
        r_last = world - 1
        rr = synth.make_reads(ref, args.reads, length=args.read_len, seed=synth.READ_SEED + r_last + args.seed_offset)
        m = min(2000, lo_k[1])
        O, oi = oracle_index(L, idx, ref_ns)
        oo = O.opts_from(opts)
        c_, o_ = np.ascontiguousarray(rr.codes), np.ascontiguousarray(rr.offsets)
        ck = ctypes.c_uint64()
        O.lib().orc_align_batch(oi.h, ctypes.byref(oo), c_.ctypes.data, o_.ctypes.data, m,
                                (r_last + args.seed_offset) * args.reads, host_cpus()["usable"], ctypes.byref(ck))
        v = N.Hits()
        N.check(L.bsq_xchg_view(nx, 0, r_last, ctypes.byref(v)))
        result["parity_sample"] = {"rank": r_last, "reads": m, "received_by_rank0": True,
                                   "checksum_match": (gpu_checksum_vec(v, m, 0) & 0xFFFFFFFFFFFFFFFF) == ck.value}

    # ---- host materialisation: the last step's rows rendered as bwa_result text ----
    if rank == 0 and not cfg["seeding"] and n_hits and not args.timed_only:
        keep, ptrs = reads_as_nuclseq(L, reads)
        # measured first, right after the timed steps: the renderers and the one-shot call below leave streams and
        # pipelines in the process that a backend running this loop would not have
        # the cursor loop of nuclseq_multi_search_bwa as extension_bsq.cpp runs it: fetches of BSQ_FETCH_ROWS
        # (262144) reads submitted to a bsq_pipeline of depth --cursor-depth (16) (each fetch staged, then its tuples released),
        # the oldest fetch's rows taken when the pipeline is full; with the two nuclseq columns per row
        # (build_tuple_bwa) rendered on the GPU, and without them
        hb.phase = "pipelined cursor fetches"
        fetch, depth, passes = 262144, args.cursor_depth, 4   # a 4M-read cursor: the batch's reads 4 times (16 fetches)

        t_sub, sub_s = [0.0], [0.0]

        def cursor(cols, deferred=True, passes=passes):
            # deferred (the drop-in's loop since round 5, extension_bsq.cpp for_each_fetch_held): fetch k is staged by a
            # pipeline worker, and its tuples are "freed" after fetch k+1 is submitted and k's staging has finished;
            # copy: staged on the caller's thread inside bsq_pipeline_submit (round 4)
            p = ctypes.c_void_p()
            N.check(L.bsq_pipeline_create(idx, depth, ctypes.byref(p)))
            try:
                rows, best = 0, None
                for rep in range(3):   # first pass allocates the slots' workspaces
                    t_sub[0] = 0.0
                    t1 = time.perf_counter()
                    pend, rows, held = 0, 0, -1

                    def take():
                        v = ctypes.POINTER(N.Hits)()
                        N.check(L.bsq_pipeline_next(p, ctypes.byref(v), None, None))
                        N.check(L.bsq_pipeline_release(p))
                        return int(v.contents.n_hits)
                    for lo in [q * reads.n + x for q in range(passes) for x in range(0, reads.n, fetch)]:
                        if pend == depth:
                            rows += take()
                            pend -= 1
                        r0 = lo % reads.n
                        n = min(fetch, reads.n - r0)
                        sp = ctypes.cast(ctypes.addressof(ptrs) + r0 * ctypes.sizeof(ctypes.c_void_p), ctypes.c_void_p)
                        t2 = time.perf_counter()
                        if deferred:
                            tk = ctypes.c_int64()
                            N.check(L.bsq_pipeline_submit_deferred(p, ctypes.byref(opts), sp, n, first_call + lo, cols,
                                                                   ctypes.byref(tk)))
                            if held >= 0:
                                N.check(L.bsq_pipeline_wait_staged(p, held + 1))
                            held = tk.value
                        else:
                            N.check(L.bsq_pipeline_submit(p, ctypes.byref(opts), sp, n, first_call + lo, cols))
                        t_sub[0] += time.perf_counter() - t2
                        pend += 1
                    if held >= 0:
                        N.check(L.bsq_pipeline_wait_staged(p, held + 1))
                    while pend:
                        rows += take()
                        pend -= 1
                    dt = time.perf_counter() - t1
                    if rep > 0 and (best is None or dt < best):
                        best = dt
                        sub_s[0] = t_sub[0]
                return rows, best
            finally:
                L.bsq_pipeline_free(p)

        rows_c, dt_c = cursor(1)
        sub_c = sub_s[0]
        rows_r, dt_r = cursor(0)
        sub_r = sub_s[0]
        rows_cc, dt_cc = cursor(1, deferred=False)
        # the same loop over a 16M-read cursor (61 fetches): the pipeline's fill (the first fetch's staging and upload)
        # and drain (the last fetches running with fewer beside them) amortised, as on a large table
        long_passes = 16
        rows_cl, dt_cl = cursor(1, passes=long_passes)
        rows_rl, dt_rl = cursor(0, passes=long_passes)
        nr = passes * reads.n
        result["sql_cursor"] = {
            "reads": nr, "fetch_rows": fetch, "depth": depth,
            "reads_per_s_with_columns": round(nr / dt_c, 1), "reads_per_s_records_only": round(nr / dt_r, 1),
            "same_row_count": rows_c == passes * n_hits and rows_r == passes * n_hits and rows_cc == passes * n_hits,
            "submit_s": [round(sub_c, 4), round(sub_r, 4)], "loop_s": [round(dt_c, 4), round(dt_r, 4)],
            "copy_staging_reads_per_s_with_columns": round(nr / dt_cc, 1),
            "steady_state": {"reads": long_passes * reads.n,
                             "reads_per_s_with_columns": round(long_passes * reads.n / dt_cl, 1),
                             "reads_per_s_records_only": round(long_passes * reads.n / dt_rl, 1),
                             "same_row_count": rows_cl == long_passes * n_hits and rows_rl == long_passes * n_hits,
                             "loop_s": [round(dt_cl, 4), round(dt_rl, 4)]},
            "note": "bsq_pipeline over fetches of host nuclseq varlenas (deferred submissions: staged by the pipeline's "
                    "workers while the caller submits the next fetch, then upload, alignment, D2H, and with columns the "
                    "two nuclseq columns of every row on the GPU), as extension_bsq.cpp's cursor loop runs it, over a "
                    "cursor of the batch's reads 4 times (lrand48 positions continuing); best of 2 runs after a warm-up "
                    "run; copy_staging_*: the same with the staging on the caller's thread (round 4's loop)"}
        # beside the headline: the drop-in's own call path (the pipelined cursor loop, columns included)
        result["value_sql_call"] = round(nr / dt_c, 1)
        if not args.cursor_only:
            hb.phase = "rendering rows on the host"
            base = ctypes.addressof(ptrs)
            sub_ptrs = [ctypes.cast(base + lo_k[k] * ctypes.sizeof(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p))
                        for k in range(S)]   # sub-batch k's reads (its read_index is local)

            def host_render():
                n = 0
                for k, b in enumerate(batches):
                    p = L.bsq_render_tsv(idx, L.bsq_batch_hits(b), sub_ptrs[k])
                    n += len(ctypes.string_at(p)) if p else 0
                    L.bsq_free(p)
                return n

            def gpu_render():
                n = 0
                tt, tn = ctypes.c_void_p(), ctypes.c_int64()
                for k, b in enumerate(batches):
                    N.check(L.bsq_batch_render(b, sub_ptrs[k], ctypes.byref(tt), ctypes.byref(tn)))
                    n += int(tn.value)
                return n

            t1 = time.perf_counter()
            nbytes = host_render()
            dt_r = time.perf_counter() - t1
            os.environ["BSQ_RENDER_THREADS"] = "1"   # the reference's single-backend rendering, for comparison
            t1 = time.perf_counter()
            host_render()
            dt_1 = time.perf_counter() - t1
            del os.environ["BSQ_RENDER_THREADS"]
            gpu_render()   # warm (buffers)
            t1 = time.perf_counter()
            gbytes = gpu_render()
            dt_g = time.perf_counter() - t1
            result["gpu_render"] = {"rows": n_hits, "seconds": round(dt_g, 4), "rows_per_s": round(n_hits / dt_g, 1),
                                    "text_MB": round(gbytes / 1e6, 1), "same_bytes_as_host": gbytes == nbytes,
                                    "note": "bsq_batch_render: rows rendered on the GPU incl. record upload and text D2H"}

            def gpu_columns():   # build_tuple_bwa's two nuclseq columns per row (bsq_batch_render_nuclseqs)
                out, oo = ctypes.c_void_p(), ctypes.c_void_p()
                for k, b in enumerate(batches):
                    N.check(L.bsq_batch_render_nuclseqs(b, sub_ptrs[k], ctypes.byref(out), ctypes.byref(oo)))
                    L.bsq_free(out)
                    L.bsq_free(oo)

            gpu_columns()   # warm
            t1 = time.perf_counter()
            gpu_columns()
            result["gpu_render"]["nuclseq_columns_rows_per_s"] = round(n_hits / (time.perf_counter() - t1), 1)
            result["host_render"] = {"rows": n_hits, "seconds": round(dt_r, 3), "rows_per_s": round(n_hits / dt_r, 1),
                                     "rows_per_s_1thread": round(n_hits / dt_1, 1),
                                     "text_MB": round(nbytes / 1e6, 1), "threads": min(16, host_cpus()["usable"]),
                                     "note": "bsq_render_tsv of the last step (BwaMatch text, Q3/Q7/Q8 rules); "
                                             "outside the timed region"}
            # the SQL-level call: one bsq_align_batch over the cursor's nuclseq values in
            # host memory -- batch and workspace set-up, device nt4 conversion, alignment, record copy
            hb.phase = "one-shot bsq_align_batch"
            ho = ctypes.POINTER(N.Hits)()
            t1 = time.perf_counter()
            N.check(L.bsq_align_batch(idx, ctypes.byref(opts), ptrs, reads.n, first_call, ctypes.byref(ho)))
            dt_s = time.perf_counter() - t1
            dts = []
            for _ in range(3):   # later calls reuse the index's pipeline (workspaces kept) and result arrays
                L.bsq_hits_free(ho)
                ho = ctypes.POINTER(N.Hits)()
                t1 = time.perf_counter()
                N.check(L.bsq_align_batch(idx, ctypes.byref(opts), ptrs, reads.n, first_call, ctypes.byref(ho)))
                dts.append(time.perf_counter() - t1)
            dt_s2 = sorted(dts)[1]
            result["sql_batch_call"] = {
                "reads": reads.n, "seconds": round(dt_s, 3), "reads_per_s": round(reads.n / dt_s, 1),
                "repeat_call_s": [round(x, 4) for x in dts], "repeat_call_reads_per_s": round(reads.n / dt_s2, 1),
                "same_rows": int(ho.contents.n_hits) == n_hits,
                "note": "bsq_align_batch from nuclseq varlenas in host memory, one call (staging, upload, device nt4 "
                        "conversion, alignment as concurrent shares, D2H, merged result arrays); first call includes "
                        "workspace allocation; repeat = median of 3"}
            L.bsq_hits_free(ho)
            N.check(L.bsq_index_release_pool(idx))   # the one-shot call's workspaces (C4: ~60 GB of HBM)

        del keep, ptrs

    # ---- bulk codec: the reference rows through nuclseq_in on the GPU vs the
    # per-value host codec, outside the timed region ----
    if rank == 0 and not args.no_codec:
        hb.phase = "bulk codec"
        from bioseqdb_amd import loader
        texts = ref.texts()
        toffs = np.zeros(len(texts) + 1, dtype=np.int64)
        toffs[1:] = np.cumsum([len(t) for t in texts])
        tcat = np.frombuffer(b"".join(texts), dtype=np.uint8)
        loader.encode_concat(tcat, toffs)   # warm
        t1 = time.perf_counter()
        raw, voff = loader.encode_concat(tcat, toffs)
        dt_e = time.perf_counter() - t1
        k_e, _ = loader.codec_ms()
        vals = loader._split(raw, voff)
        dt_h = 0.0
        for t in texts:   # the per-value path (bsq_nuclseq_from_text = nuclseq_from_text), one host thread
            size = ctypes.c_size_t()
            t2 = time.perf_counter()
            p = L.bsq_nuclseq_from_text(t, len(t), ctypes.byref(size))
            dt_h += time.perf_counter() - t2
            L.bsq_free(p)
        same = all(v.raw == bytes(h.raw) for v, h in zip(vals, ref_ns)) if ref_ns else None
        loader.nuclseq_out_batch(vals)
        k_d, c_d = loader.codec_ms()
        nb = int(toffs[-1])
        out_b = int(voff[-1])
        result["bulk_codec"] = {
            "bases": nb, "encode_s": round(dt_e, 4), "encode_kernel_ms": round(k_e, 3),
            "encode_kernel_gbs": round((2 * nb + out_b) / (k_e * 1e-3) / 1e9, 1) if k_e > 0 else None,
            "encode_gbases_per_s": round(nb / dt_e / 1e9, 2), "host_gbases_per_s_1thread": round(nb / dt_h / 1e9, 3),
            "decode_kernel_ms": round(k_d, 3), "decode_call_s": round(c_d * 1e-3, 4),
            "same_bytes_as_host": same,
            "note": "bsq_nuclseq_encode_batch on the reference rows (call incl. PCIe both ways); kernel GB/s counts "
                    "the text read twice (count + write passes) and the varlenas written once",
        }
        del raw, vals, tcat

    # ---- CPU baseline: the oracle on this host, bounded sample, rank 0 at N = 1 only ----
    per_read = None
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        hb.phase = "CPU baseline"
        O, oi = oracle_index(L, idx, ref_ns)
        oo = O.opts_from(opts)
        host = host_cpus()
        threads = args.cpu_threads or host["usable"]
        cb = cpu_baseline(O, oi, oo, codes, offs, reads.n, threads, cfg["seeding"], args.cpu_seconds, first_call)
        sample = cb["sample"]
        if cfg["seeding"]:
            ro = ctypes.POINTER(ctypes.c_int64)()
            ivp = ctypes.POINTER(ctypes.c_uint64)()
            nt = ctypes.c_int64()
            N.check(L.bsq_batch_intervals(batch, ctypes.byref(ro), ctypes.byref(ivp), ctypes.byref(nt)))
            soff = np.ctypeslib.as_array(ro, shape=(reads.n + 1,))
            siv = np.ctypeslib.as_array(ivp, shape=(max(int(nt.value), 1) * 4,))[: int(nt.value) * 4].reshape(-1, 4)
            gck = intv_checksum_vec(soff, siv, sample)
        else:
            gck = 0
            for k, b in enumerate(batches):   # sub-batch k holds reads [lo_k[k], lo_k[k+1])
                m = min(sample, lo_k[k + 1]) - lo_k[k]
                if m > 0:
                    gck += gpu_checksum_vec(L.bsq_batch_hits(b).contents, m, lo_k[k])
            gck &= 0xFFFFFFFFFFFFFFFF
        result["cpu_baseline"] = {
            "value": cb["value"], "unit": "reads/s", "cores": threads, "kind": "port",
            "sample": (f"first {sample} reads of the same batch, CPU oracle (oracle/bwa_oracle.c, -O2), {threads} threads "
                       f"= every core this process may use; median of 3 runs after a warm-up "
                       f"(runs {', '.join(f'{t:.2f}' for t in cb['times'])} s); 1 thread: median of 3 over "
                       f"{cb['n1']} reads ({', '.join(f'{t:.2f}' for t in cb['times1'])} s)"),
            "value_1thread": cb["value_1thread"],
            "host": host,
        }
        result["parity_sample"] = {"reads": sample, ("intervals" if cfg["seeding"] else "regions"): int(cb["nreg"]),
                                   "checksum_match": bool(gck == cb["ck"])}
        result["gpu_vs_cpu"] = round(value / cb["value"], 1)
        result["gpu_vs_cpu_1thread"] = round(value / cb["value_1thread"], 1)
        # SURVEY.md 8(d)'s per-read algorithmic bytes (libbwa's own layout, counted by the oracle on this sample)
        reads_bytes_per_read = (args.read_len + 3) // 4   # the packed read (2 bits per base)
        ab = cb["ab"]
        per_read = [ab[0] / sample + reads_bytes_per_read, ab[1] / sample, ab[2] / sample, ab[3] / sample]
        for i, nm in enumerate(names[:nst]):
            k = result["kernels"][STAGE_KERNEL[nm]]
            k["algorithmic_bytes_8d_per_read"] = round(per_read[i], 1)
            k["achieved_gbs_8d"] = (round(per_read[i] * reads_per_launch / (k["ms"] * 1e-3) / 1e9, 2)
                                    if k["ms"] > 0 else 0.0)
            if iso and iso[0][i] > 0:
                k["lone_achieved_gbs_8d"] = round(per_read[i] * reads.n / (iso[0][i] * 1e-3) / 1e9, 2)
        result["roofline_source"] = (f"SURVEY.md 8(d) bytes: oracle-counted on libbwa's layout over the {sample}-read "
                                     "sample (64 B per occ block of bwt_extend, 8 B per SA value, ceil(bases/4) per "
                                     "reference window, + the packed read)")
    result["roofline"] = make_roofline(dom, di, stage_ms, stage_bytes, reads_per_launch, iso, reads.n, per_read, tr, S)
    if SA_CERT:
        result["sa_certificate"] = dict(SA_CERT)
    # introsort scans stopped by the bound rather than the sentinel over every run in this process (must be 0)
    result["sort_guard"] = int(L.bsq_sort_guard_total())
    hb.stop()
    if rank == 0:
        print(json.dumps(result), file=json_out(), flush=True)
    if nx is not None:
        L.bsq_xchg_free(nx)
    for b in batches:
        L.bsq_batch_free(b)
    L.bsq_index_free(idx)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
