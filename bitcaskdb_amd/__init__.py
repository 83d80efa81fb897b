"""bitcaskdb_amd: MI355X-native WAL record codec for bitcaskDB's compaction / recovery scan.

The product is libbcw.so (C-ABI in include/bcw.h, HIP kernels for gfx950 in csrc/). This package
is the Python host mirror of the reference interface (wal.py: the WAL iterators, compaction re-encode,
hint rebuild; index.py: the device-resident index, its rebuild from hint / data WALs and the device
compaction filter) and its ctypes binding (_lib.py).
"""
from . import _lib
from .wal import (Context, Decoded, ErrCorruptedHintRecord, ErrInvalidData, ErrShortFile, ErrWalMismatchBlockSize,
                  ErrWalMismatchCRC, ErrWalMismatchMagic, ErrWalUnknownRecordType, HintRecord, Meta, Record,
                  RefPanic, Wal, WalError, WalFile, compact_one_wal, compute_crc32, default_context, iterate_hint,
                  iterate_record, load_wal, new_hint_by_wal)
from .staging import Stage
from .index import (ErrKeyNotFound, ErrKeySoftDeleted, Index, compact_one_wal_filtered, merged_key, murmur3_sum64,
                    recover_from_wals)

__all__ = ["Context", "Decoded", "ErrCorruptedHintRecord", "ErrInvalidData", "ErrShortFile",
           "ErrWalMismatchBlockSize", "ErrWalMismatchCRC", "ErrWalMismatchMagic", "ErrWalUnknownRecordType",
           "HintRecord", "Meta", "Record", "RefPanic", "Wal", "WalError", "compute_crc32", "default_context",
           "iterate_hint", "iterate_record", "load_wal", "_lib", "WalFile", "compact_one_wal",
           "new_hint_by_wal", "ErrKeyNotFound", "ErrKeySoftDeleted", "Index", "compact_one_wal_filtered",
           "merged_key", "murmur3_sum64", "recover_from_wals", "Stage"]
