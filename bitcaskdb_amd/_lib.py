"""ctypes binding of libbcw.so (include/bcw.h). The HIP extension is mandatory: importing
this module without the built library raises, there is no CPU fallback on the product path."""
from __future__ import annotations

import ctypes as C
import os
import re

# One HIP runtime per process. PyTorch (device memory, streams and torch.distributed in bench.py and the tests) ships
# its own libamdhip64 with the soname libamdhip64.so.7; loaded first, it is the runtime libbcw.so binds to. Loaded
# after libbcw.so it would be a second runtime in the process, and with two processes sharing a GPU the second
# runtime of each finds no device (measured: tools/probe/runtimes.py). Without PyTorch libbcw.so uses /opt/rocm's.
# The preload costs the import time of torch: a process that never uses PyTorch (a CPU-only tool, the Go-side shim's
# tests) sets BCW_NO_TORCH_PRELOAD=1 to skip it; a process that does use PyTorch must then import torch first itself.
if os.environ.get("BCW_NO_TORCH_PRELOAD") != "1":
    try:
        import torch  # noqa: F401
    except ImportError:
        pass

_HERE = os.path.dirname(os.path.abspath(__file__))
# BCW_LIB: an alternative build of the same library (A/B measurements of kernel variants only)
LIB_PATH = os.environ.get("BCW_LIB") or os.path.join(_HERE, "libbcw.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "bcw.h")

u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)


class SuperBlock(C.Structure):
    _fields_ = [("magic", C.c_uint64), ("block_size", C.c_uint64), ("start_off", C.c_uint32),
                ("crc", C.c_uint32), ("create_time", C.c_uint64), ("base_time", C.c_uint64)]


class DecodeParams(C.Structure):
    _fields_ = [("seg_len", C.c_uint64), ("base_time", C.c_uint64), ("start_off", C.c_uint32),
                ("ns_size", C.c_uint32), ("etag_size", C.c_uint32), ("mode", C.c_uint32)]


class RecordTable(C.Structure):
    _fields_ = [("capacity", C.c_uint64), ("foff", u64p), ("size", u64p), ("expire", u64p),
                ("aux0", u64p), ("aux1", u64p), ("key_len", u32p), ("val_len", u32p), ("meta_len", u32p),
                ("first_frag", u32p), ("emit_frag", u32p), ("hdr_size", u8p), ("flags", u8p),
                ("etag_off", u8p), ("status", u8p)]


class DecodeResult(C.Structure):
    _fields_ = [("n_records", C.c_uint64), ("n_records_total", C.c_uint64), ("n_frags", C.c_uint64),
                ("err_frag", C.c_uint64), ("err_file_off", C.c_uint64), ("err_class", C.c_int32),
                ("first_bad_record", C.c_int32), ("n_blocks", C.c_uint64), ("retry_frag_capacity", C.c_uint64),
                ("generation", C.c_uint64)]


class FragTable(C.Structure):
    _fields_ = [("capacity", C.c_uint64), ("data_off", u64p), ("len", u32p), ("stored_crc", u32p),
                ("type", u8p), ("crc_ok", u8p)]


class EncodeParams(C.Structure):
    _fields_ = [("src_len", C.c_uint64), ("dst_base_time", C.c_uint64), ("fid", C.c_uint64), ("wal_pos", C.c_uint64),
                ("hint_pos", C.c_uint64), ("src_start_off", C.c_uint32), ("mode", C.c_uint32), ("ns_size", C.c_uint32),
                ("etag_size", C.c_uint32)]


class EncodeOut(C.Structure):
    _fields_ = [("wal", u8p), ("wal_cap", C.c_uint64), ("hint", u8p), ("hint_cap", C.c_uint64), ("rec_off", u64p),
                ("rec_off_cap", C.c_uint64)]


class EncodeResult(C.Structure):
    _fields_ = [("n_in", C.c_uint64), ("n_written", C.c_uint64), ("wal_end", C.c_uint64), ("hint_end", C.c_uint64),
                ("wal_need", C.c_uint64), ("hint_need", C.c_uint64), ("err_record", C.c_int64),
                ("err_class", C.c_int32), ("src_err_class", C.c_int32), ("wal_events", C.c_uint32),
                ("hint_events", C.c_uint32), ("fits", C.c_uint32), ("_pad", C.c_uint32)]


class ReadParams(C.Structure):
    _fields_ = [("seg_len", C.c_uint64), ("base_time", C.c_uint64), ("ns_size", C.c_uint32),
                ("etag_size", C.c_uint32), ("verify", C.c_uint32), ("_pad", C.c_uint32)]


class IndexResult(C.Structure):
    _fields_ = [("n_in", C.c_uint64), ("n_done", C.c_uint64), ("err_class", C.c_int32), ("_pad", C.c_int32)]


class RecoverFile(C.Structure):
    _fields_ = [("fid", C.c_uint64), ("wal", C.c_void_p), ("wal_p", DecodeParams), ("hint", C.c_void_p),
                ("hint_p", DecodeParams)]


class RecoverStatus(C.Structure):
    _fields_ = [("used", C.c_int32), ("rc", C.c_int32), ("hint_dres", DecodeResult), ("wal_dres", DecodeResult),
                ("hint_ires", IndexResult), ("wal_ires", IndexResult)]


class CompactSrc(C.Structure):
    _fields_ = [("fid", C.c_uint64), ("data", C.c_void_p), ("len", C.c_uint64), ("start_off", C.c_uint32),
                ("_pad", C.c_uint32), ("out", EncodeOut)]


class IndexInfo(C.Structure):
    _fields_ = [("live", C.c_uint64), ("slots_used", C.c_uint64), ("slot_capacity", C.c_uint64),
                ("arena_used", C.c_uint64), ("arena_capacity", C.c_uint64), ("overflow", C.c_uint64),
                ("limited", C.c_uint64), ("evicted", C.c_uint64), ("evicted_bytes", C.c_uint64)]


# the table's column names, C types and numpy dtypes (one place, used by wal.py and bench.py)
TABLE_COLUMNS = [("foff", "u8"), ("size", "u8"), ("expire", "u8"), ("aux0", "u8"), ("aux1", "u8"),
                 ("key_len", "u4"), ("val_len", "u4"), ("meta_len", "u4"), ("first_frag", "u4"),
                 ("emit_frag", "u4"), ("hdr_size", "u1"), ("flags", "u1"), ("etag_off", "u1"), ("status", "u1")]
FRAG_COLUMNS = [("data_off", "u8"), ("len", "u4"), ("stored_crc", "u4"), ("type", "u1"), ("crc_ok", "u1")]

# constants mirrored from bcw.h
BLOCK_SIZE = 32768
HEADER_SIZE = 7
SUPER_BLOCK_SIZE = 40
MODE_RECORD, MODE_HINT = 0, 1
ST_OK, ST_INVALID, ST_PANIC, ST_UNSUPPORTED = 0, 1, 2, 3
ERR_NONE, ERR_CRC, ERR_TYPE, ERR_PANIC, ERR_INTERNAL = 0, 1, 2, 3, 4
SB_OK, SB_SHORT, SB_CRC, SB_MAGIC, SB_BLOCKSIZE = 0, 1, 2, 3, 4
E_INVAL, E_CAPACITY = -1, -4
OPT_CHASE_DIRECT = 1  # bcw_ctx_set_option: k_chase direct-sum workgroup limit (0 forces the look-back)
OPT_DECODE_CHUNKS = 3  # bcw_ctx_set_option: retired (only 1 accepted)
OPT_DECODE_PATH = 2  # bcw_ctx_set_option: retired (only 1 accepted: k_chase + k_crc)
OPT_TEST_ABORT_WAIT = 4  # bcw_ctx_set_option: fault injection (needs BCW_TEST_HOOKS=1): the next decode's k_chase workgroup value-1 gives up its wait
OPT_FILTER_SNAPSHOT = 5  # bcw_ctx_set_option: bcw_compact_wals filters this context's sources against a staging snapshot
OPT_XCD_BALANCE = 6  # bcw_ctx_set_option: k_crc's stream split over the XCDs by their measured rates (default 1)
E_IO = -6
ENC_COMPACT, ENC_HINT = 0, 1
ENC_ERR_NONE, ENC_ERR_SRC, ENC_ERR_EXPIRE, ENC_ERR_PANIC, ENC_ERR_TABLE, ENC_ERR_STALE = 0, 1, 2, 3, 4, 5
IDX_PUT, IDX_DELETE, IDX_SOFT_DELETE = 0, 1, 2
IDX_FOUND, IDX_NOT_FOUND, IDX_SOFT_DELETED = 0, 1, 2
IDX_ERR_FULL = 6
RECOVER_NOT_RUN, RECOVER_HINT, RECOVER_HINT_WAL, RECOVER_WAL = 0, 1, 2, 3
RD_OK, RD_BEYOND, RD_CORRUPTED, RD_CRC, RD_SIZE, RD_TYPE, RD_INCOMPLETE, RD_PANIC = range(8)


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libbcw.so not built ({LIB_PATH}); run __graft_entry__.build() or `make -C bitcaskdb_amd`")
    lib = C.CDLL(LIB_PATH)
    vp = C.c_void_p
    sig = {
        "bcw_abi_version": (C.c_int, []),
        "bcw_strerror": (C.c_char_p, [C.c_int]),
        "bcw_device_count": (C.c_int, []),
        "bcw_ctx_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
        "bcw_ctx_destroy": (C.c_int, [vp]),
        "bcw_ctx_set_stream": (C.c_int, [vp, vp]),
        "bcw_ctx_stream": (vp, [vp]),
        "bcw_ctx_sync": (C.c_int, [vp]),
        "bcw_ctx_device": (C.c_int, [vp]),
        "bcw_ctx_set_profiling": (C.c_int, [vp, C.c_int]),
        "bcw_ctx_set_profiling_sample": (C.c_int, [vp, C.c_int]),
        "bcw_ctx_kernel_times": (C.c_int, [vp, C.POINTER(C.c_double), u64p, C.c_int]),
        "bcw_kernel_name": (C.c_char_p, [C.c_int]),
        "bcw_ctx_reserve_fragments": (C.c_int, [vp, C.c_uint64]),
        "bcw_ctx_set_option": (C.c_int, [vp, C.c_int, C.c_uint64]),
        "bcw_wal_record_size": (C.c_uint64, [C.c_uint64, C.c_uint64]),
        "bcw_wal_block_index_range": (None, [C.c_uint64, C.c_uint64, u64p, u64p, u64p]),
        "bcw_crc32c_masked": (C.c_uint32, [vp, C.c_uint64]),
        "bcw_load_super_block": (C.c_int, [vp, C.c_uint64, C.POINTER(SuperBlock)]),
        "bcw_write_super_block": (None, [vp, C.c_uint64, C.c_uint64]),
        "bcw_max_fragments": (C.c_uint64, [C.c_uint64, C.c_uint32]),
        "bcw_decode_segment_async": (C.c_int, [vp, vp, C.POINTER(DecodeParams), C.POINTER(RecordTable), vp]),
        "bcw_decode_segment": (C.c_int, [vp, vp, C.POINTER(DecodeParams), C.POINTER(RecordTable),
                                         C.POINTER(DecodeResult)]),
        "bcw_decode_fragments_async": (C.c_int, [vp, C.POINTER(FragTable)]),
        "bcw_decode_fragments": (C.c_int, [vp, C.POINTER(FragTable), u64p]),
        "bcw_encode_segment_async": (C.c_int, [vp, vp, C.POINTER(EncodeParams), C.POINTER(RecordTable), vp, vp,
                                               C.POINTER(EncodeOut), vp]),
        "bcw_encode_segment": (C.c_int, [vp, vp, C.POINTER(EncodeParams), vp, C.c_uint64, C.POINTER(EncodeOut),
                                         C.POINTER(EncodeResult)]),
        "bcw_index_create": (C.c_int, [vp, C.c_uint64, C.c_uint64, C.POINTER(vp)]),
        "bcw_index_destroy": (C.c_int, [vp]),
        "bcw_index_reserve": (C.c_int, [vp, C.c_uint64, C.c_uint64]),
        "bcw_index_stats": (C.c_int, [vp, C.POINTER(IndexInfo)]),
        "bcw_index_set_limit": (C.c_int, [vp, C.c_uint64]),
        "bcw_index_apply": (C.c_int, [vp, C.c_uint64, vp, u64p, u8p, u64p, u64p, u64p]),
        "bcw_index_apply_stat": (C.c_int, [vp, C.c_uint64, vp, u64p, u8p, u64p, u64p, u64p, u8p, u64p, u64p]),
        "bcw_index_clear": (C.c_int, [vp]),
        "bcw_index_get": (C.c_int, [vp, C.c_uint64, vp, u64p, u64p, u64p, u64p, u8p]),
        "bcw_index_put_decoded_async": (C.c_int, [vp, vp, C.POINTER(DecodeParams), C.POINTER(RecordTable), vp,
                                                  C.c_uint64, C.c_int, vp]),
        "bcw_compact_filter_async": (C.c_int, [vp, vp, C.POINTER(DecodeParams), C.POINTER(RecordTable), vp,
                                               C.c_uint64, vp, vp]),
        "bcw_index_export": (C.c_int, [vp, vp, C.c_uint64, u64p, u64p, u64p, u64p, C.c_uint64, u64p, u64p]),
        "bcw_index_export_fids": (C.c_int, [vp, u64p, C.c_uint64, vp, C.c_uint64, u64p, u64p, u64p, u64p,
                                            C.c_uint64, u64p, u64p]),
        "bcw_recover_wals": (C.c_int, [vp, C.POINTER(vp), C.c_uint32, C.POINTER(RecoverFile), C.c_uint64,
                                       C.POINTER(RecoverStatus), C.POINTER(C.c_int64)]),
        "bcw_compact_wals": (C.c_int, [vp, C.POINTER(vp), C.c_uint32, C.POINTER(CompactSrc), C.c_uint64,
                                       C.POINTER(EncodeParams), C.POINTER(EncodeResult), C.POINTER(IndexResult),
                                       u64p]),
        "bcw_compact_segment": (C.c_int, [vp, vp, vp, C.POINTER(EncodeParams), C.c_uint64, C.POINTER(EncodeOut),
                                          C.POINTER(EncodeResult), C.POINTER(IndexResult)]),
        "bcw_index_recover_segment": (C.c_int, [vp, vp, vp, C.POINTER(DecodeParams), C.c_uint64, C.c_int,
                                                C.POINTER(DecodeResult), C.POINTER(IndexResult)]),
        "bcw_murmur3_sum64": (C.c_uint64, [vp, C.c_uint64]),
        "bcw_read_records_async": (C.c_int, [vp, vp, C.POINTER(ReadParams), C.c_uint64, vp, vp, vp, vp, vp,
                                             C.POINTER(RecordTable)]),
        "bcw_read_records": (C.c_int, [vp, vp, C.POINTER(ReadParams), C.c_uint64, u64p, u64p, vp, u8p,
                                       C.POINTER(RecordTable)]),
        "bcw_stage_create": (C.c_int, [vp, C.c_uint64, C.c_uint32, C.POINTER(vp)]),
        "bcw_stage_destroy": (C.c_int, [vp]),
        "bcw_stage_read": (C.c_int, [vp, C.c_int, C.c_uint64, C.c_uint64, vp, vp, C.c_uint32]),
        "bcw_stage_write": (C.c_int, [vp, C.c_int, C.c_uint64, vp, C.c_uint64, vp, C.c_uint32]),
        "bcw_peer_enable": (C.c_int, [C.c_int, C.c_int]),
        "bcw_stage_peer": (C.c_int, [vp, vp, vp, C.c_int, C.c_uint64, vp]),
        "bcw_synth_segment": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                                        C.c_int, C.c_uint64, vp, C.c_uint64, u64p, u64p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def header_symbols(path: str = HEADER_PATH) -> list[str]:
    """Every function the C-ABI header declares (used by the symbol-export test)."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bcw_[a-z0-9_]+)\s*\(", text)))
