"""ibwa_amd -- MI355X-native engine for the `ibwa aln` hot path.

Host-side mirror of the reference's aln interface (bwtaln.c / bwtaln.h):
``GapOpt`` (gap_opt_t), read batches (bwa_seq_t), ``.sai`` I/O, and the
device engine behind the C-ABI in include/ibwa_aln.h.
"""
__version__ = "0.1.0"
