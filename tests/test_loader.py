"""Bulk loader host side: the FASTA reading of bioseqdb-import
(bioseqdb-import/main.cpp:48-71) against a line-by-line restatement, and the codec's argument checks that
run before any device work (no GPU needed)."""
import random

import numpy as np
import pytest

from bioseqdb_amd import _native, loader
from bioseqdb_amd.bwa import InvalidParameterValue, InvalidTextRepresentation


def fasta_restated(data: bytes):
    """main.cpp:48-71 with std::getline semantics: split at '\\n', no empty line after a final '\\n'."""
    out, name, seq = [], b"", b""
    lines = data.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    for line in lines:
        if line[:1] == b">":
            if seq:
                out.append((name, seq))
            seq = b""
            name = line[1:]
        else:
            seq += bytes(c - 32 if 97 <= c <= 122 else c for c in line)
    if seq:
        out.append((name, seq))
    return [(n.decode("utf-8", errors="surrogateescape"), s) for n, s in out]


CASES = [
    b"",
    b"\n",
    b">a\nACGT\n",
    b">a\nACGT",
    b"acgtn\n>x\nAC\ngt\n",                 # sequence before any header: record with an empty name
    b">a\n>b\nAC\n>c\n\n>d\nT\n",          # empty records are dropped with their names
    b">r1 desc\r\nAC\r\nGT\r\n",           # '\r' stays in names and sequence lines (getline)
    b">\nNNNN\n>z\n",
    b">s\nacgtRYkmswbdhvn-.\n\n\nACGT\n",
    ">żółć\nAC\n".encode(),
]


@pytest.mark.parametrize("data", CASES)
def test_fasta_cases(data):
    assert loader.parse_fasta(data) == fasta_restated(data)


def test_fasta_random():
    rng = random.Random(3)
    for _ in range(200):
        parts = []
        for _ in range(rng.randint(0, 12)):
            r = rng.random()
            if r < 0.25:
                parts.append(b">" + bytes(rng.choice(b"abc XYZ\r") for _ in range(rng.randint(0, 6))))
            elif r < 0.35:
                parts.append(b"")
            else:
                parts.append(bytes(rng.choice(b"ACGTNacgtnRY\r") for _ in range(rng.randint(0, 70))))
        data = b"\n".join(parts) + (b"\n" if rng.random() < 0.5 else b"")
        assert loader.parse_fasta(data) == fasta_restated(data)


def test_too_long_is_checked_first_on_the_host():
    # nuclseq_in's length check (extension.cpp:50-51) precedes any device work
    big = np.full(0x7FFFFFFF // 4 + 1, ord("A"), dtype=np.uint8)
    offs = np.array([0, 4, 4 + len(big)], dtype=np.int64)
    data = np.concatenate([np.frombuffer(b"ACGT", np.uint8), big])
    with pytest.raises(InvalidParameterValue, match="provided sequence is too long"):
        loader.encode_concat(data, offs)
    # an invalid character in an earlier text is reported first, as a cursor of nuclseq_in calls would
    data[1] = ord("x")
    with pytest.raises(InvalidTextRepresentation, match="invalid nucleotide in nuclseq_in: 'x'"):
        loader.encode_concat(data, offs)


def test_codec_without_device_fails_loudly(gpu_available):
    if gpu_available:
        pytest.skip("GPU present")
    with pytest.raises(_native.BsqError) as e:
        loader.nuclseq_in_batch(["ACGT"])
    assert e.value.code == _native.BSQ_E_NODEV
