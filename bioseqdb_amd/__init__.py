"""bioseqdb_amd -- MI355X-native BWA-MEM alignment path of bioseqdb (nuclseq_search_bwa /
nuclseq_multi_search_bwa), as HIP kernels behind the C-ABI in include/bsq.h.

Layout:
  csrc/           HIP kernels (align_kernels.hip), host index builder, C-ABI (libbsq.so)
  _native.py      ctypes bindings of every include/bsq.h symbol
  bwa.py          host mirror of the reference interface (BwaIndex, bwa_opts, search functions)
  synth.py        deterministic synthetic reference / read generator
  dist.py         read-sharded multi-GPU driver (one process per GPU, gather of hit records)
"""
from ._native import BsqError, lib  # noqa: F401
from .bwa import (  # noqa: F401
    BWA_RESULT_COLUMNS, BwaIndex, BwaMatch, BwaOptions, NucleotideSequence, bwa_index_from_query, bwa_opts,
    effective_opts, lrand48_calls, nuclseq_multi_search_bwa, nuclseq_search_bwa, reset_lrand48,
)

__all__ = [
    "BsqError", "lib", "BWA_RESULT_COLUMNS", "BwaIndex", "BwaMatch", "BwaOptions", "NucleotideSequence",
    "bwa_index_from_query", "bwa_opts", "effective_opts", "lrand48_calls", "nuclseq_multi_search_bwa",
    "nuclseq_search_bwa", "reset_lrand48",
]
