"""bsq_index_layout (index replication) on the host: table sizes follow the index's
shape and the metadata blob is self-describing (no GPU needed)."""
import ctypes

from bioseqdb_amd import BwaIndex, NucleotideSequence, synth
from bioseqdb_amd import _native as N


def _index(bp, rows):
    ref = synth.make_reference(bp, n_rows=rows, n_run_every=max(bp // 3, 1000), n_run_len=100)
    pi = BwaIndex()
    for i, t in enumerate(ref.texts()):
        pi.add_ref_sequence(i + 1, NucleotideSequence.from_text(t.decode()))
    pi.build()
    return pi


def test_layout_sizes_and_meta():
    L = N.lib()
    pi = _index(300_000, 3)
    sizes = (ctypes.c_uint64 * N.N_TABLES)()
    mb = ctypes.c_uint64()
    assert L.bsq_index_layout(pi.handle, sizes, None, ctypes.byref(mb)) == 0
    n = L.bsq_index_seq_len(pi.handle)
    l_pac = L.bsq_index_l_pac(pi.handle)
    occ, occ32, sa, pac, ann_off, ann_id, ann_len, kmer = list(sizes)
    assert occ == ((n + 127) // 128 + 1) * 64                       # 64-B blocks of 128 rows (+1 guard)
    assert occ32 == occ and sa == (n + 1) * 4                       # 32-B blocks of 64 rows; u32 SA
    assert pac == (l_pac + 3) // 4 + 16
    assert ann_off == ann_id == 3 * 8 and ann_len == 3 * 4
    assert kmer > 0 and kmer % 16 == 0
    small = ctypes.c_uint64(8)
    buf = ctypes.create_string_buffer(8)
    assert L.bsq_index_layout(pi.handle, sizes, buf, ctypes.byref(small)) != 0   # too small: refused
    meta = ctypes.create_string_buffer(mb.value)
    assert L.bsq_index_layout(pi.handle, sizes, meta, ctypes.byref(mb)) == 0
    assert meta.raw[:7] == b"BSQIDX1"


def test_layout_wide(monkeypatch):
    monkeypatch.setenv("BSQ_FORCE_WIDE", "1")
    L = N.lib()
    pi = _index(100_000, 1)
    sizes = (ctypes.c_uint64 * N.N_TABLES)()
    mb = ctypes.c_uint64()
    assert L.bsq_index_layout(pi.handle, sizes, None, ctypes.byref(mb)) == 0
    n = L.bsq_index_seq_len(pi.handle)
    nblk = (n + 127) // 128 + 1
    # 64-bit rows also get the 32-B blocks (u32 counts relative to 2^22-row superblocks), the superblocks'
    # 64-B absolute counts appended (bsq_device.h SupBlock, one per 2^16 blocks of 64 rows)
    assert sizes[1] == 2 * nblk * 32 + ((2 * nblk >> 16) + 1) * 64
    assert sizes[2] == (n + 1) * 8 and sizes[7] % 32 == 0
