"""bench.py's vectorised parity checksums equal the scalar per-read FNV the oracle computes
(orc_align_batch / orc_seed_batch), on random hit and interval layouts."""
import ctypes
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    argv = sys.argv
    sys.argv = ["bench.py"]
    try:
        spec.loader.exec_module(m)
    finally:
        sys.argv = argv
    return m


def _hits(rng, n_reads):
    from bioseqdb_amd import _native as N
    per = rng.integers(0, 4, size=n_reads)
    off = np.concatenate([[0], np.cumsum(per)]).astype(np.int64)
    nh = int(off[-1])
    hits = (N.Hit * max(nh, 1))()
    cig = []
    for k in range(nh):
        h = hits[k]
        h.rb = int(rng.integers(0, 1 << 40)); h.re = h.rb + int(rng.integers(1, 200))
        h.qb = int(rng.integers(-5, 150)); h.qe = int(rng.integers(0, 150)); h.score = int(rng.integers(-30, 151))
        h.is_secondary = int(rng.integers(0, 2))
        nc = int(rng.integers(0, 6))
        h.cigar_off = len(cig); h.n_cigar = nc
        cig.extend(int(v) for v in rng.integers(0, 1 << 32, size=nc, dtype=np.uint64))
    cig_arr = (ctypes.c_uint32 * max(len(cig), 1))(*cig) if cig else (ctypes.c_uint32 * 1)()
    off_arr = (ctypes.c_int64 * (n_reads + 1))(*off.tolist())
    H = N.Hits()
    H.n_reads = n_reads; H.n_hits = nh; H.hits = ctypes.cast(hits, ctypes.POINTER(N.Hit))
    H.read_off = ctypes.cast(off_arr, ctypes.POINTER(ctypes.c_int64)); H.n_cigar = len(cig)
    H.cigar = ctypes.cast(cig_arr, ctypes.POINTER(ctypes.c_uint32))
    return H, (hits, cig_arr, off_arr)


def test_hit_checksum_vectorised_equals_scalar():
    B = _bench()
    rng = np.random.default_rng(5)
    H, keep = _hits(rng, 300)
    assert B.gpu_checksum_vec(H, 300) == B.gpu_checksum(H, 300)
    assert B.gpu_checksum_vec(H, 120) == B.gpu_checksum(H, 120)


def test_interval_checksum_vectorised_equals_scalar():
    B = _bench()
    rng = np.random.default_rng(6)
    n = 200
    per = rng.integers(0, 7, size=n)
    off = np.concatenate([[0], np.cumsum(per)]).astype(np.int64)
    iv = rng.integers(0, 1 << 63, size=(int(off[-1]), 4), dtype=np.uint64)
    exp = 0
    for r in range(n):
        h = B.fnv(0xCBF29CE484222325, r)
        for k in range(off[r], off[r + 1]):
            for v in (iv[k, 0], iv[k, 2], iv[k, 3]):
                h = B.fnv(h, int(v))
        exp = (exp + h) & 0xFFFFFFFFFFFFFFFF
    assert B.intv_checksum_vec(off, iv, n) == exp


def test_roofline_fields():
    """The line's HBM fraction of the PMC traffic (`roofline.traffic_frac`) and the extension's VALU roofline
    (`kernels.k_ext_key+sort+k_extend.valu`): plain ratios of the figures beside them."""
    b = _bench()
    roof = b.make_roofline("smem", 0, [2.0] * 6, [1e9] * 6, 1000, ([4.0] * 6, [2e9] * 6, [0.0] * 6), 1000,
                           [8000.0] * 4, lambda stage, n: (16e9, "rXX"), 1)
    assert roof["traffic"] == 16e9
    assert abs(roof["traffic_frac"] - 16e9 / 4e-3 / 1e9 / b.HBM_PEAK_GBS) < 1e-4
    none = b.make_roofline("smem", 0, [2.0] * 6, [1e9] * 6, 1000, None, 1000, None, lambda stage, n: (None, None), 1)
    assert none["traffic_frac"] is None
    v = b.valu_roofline(1e9, 5.0, {"valu_lane_util": 0.4, "valu_busy": 0.42})
    assert v["frac"] == round(1e9 * b.EXT_VALU_PER_CELL / 5e-3 / b.VALU_PEAK_LANE_OPS, 4)
    assert v["sq_lane_util"] == 0.4 and v["bound"] == "valu"
