/*
 * bcw.h -- C-ABI of the MI355X-native bitcaskDB WAL record codec (libbcw.so).
 *
 * Drop-in boundary for the per-record loops of bitcaskDB's compaction / recovery / hint rebuild
 * (wenzhang-dev/bitcaskDB, paths relative to the reference root):
 *   bcw_decode_segment*  replaces  IterateRecord(wal, cb)      record.go:242-266
 *                        i.e.      WalIterator.Next            wal_iterator.go:40-100
 *                        plus      RecordFromBytes             record.go:140-239
 *                        callers   compaction.go:299, hint.go:133, db_impl.go:307
 *   mode BCW_MODE_HINT   replaces  IterateHint(hint, cb)       hint.go:163-188 (+ HintRecord.Decode hint.go:50-84)
 *                        callers   db_impl.go:296, compaction.go:248
 *   bcw_crc32c_masked    replaces  ComputeCRC32                utils.go:24-29
 *   bcw_load_super_block replaces  Wal.loadSuperBlock          wal.go:362-398
 *   bcw_write_super_block          Wal.writeSuperBlock         wal.go:332-360
 *   bcw_encode_segment*  replaces  the compactOneWal loop      compaction.go:294-327
 *     (BCW_ENC_COMPACT)            = Record.Encode              record.go:57-138
 *                                  + WalRewriter.AppendRecord   wal_rewriter.go:39-51 -> Wal.WriteRecord wal.go:490-553
 *                                  + HintWriter.AppendRecord    hint.go:109-117 -> HintRecord.Encode hint.go:32-48
 *     (BCW_ENC_HINT)     replaces  NewHintByWal                 hint.go:123-161
 *                        callers   compaction.go:203-211 (via compactOneWal), db_impl.go:545
 *   bcw_synth_segment    host WAL writer: Wal.WriteRecord wal.go:490-553 over Record.Encode
 *                                  record.go:57-138 (synthetic segments of the benchmark configs)
 *
 * Plain C types only (no torch / HIP types in signatures). Device pointers are `void*`/`uint8_t*`
 * values obtained from hipMalloc (or any HIP allocator). Every call is reentrant: all mutable
 * state lives in the bcw_ctx, one per caller thread (compaction, hint rebuild and recovery may run
 * concurrently). Errors are returned as negative BCW_E* codes; per-record and
 * per-segment outcomes are reported in the result structs, never by aborting.
 */
#ifndef BCW_H
#define BCW_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BCW_ABI_VERSION 2

/* ---- return codes ---- */
#define BCW_OK 0
#define BCW_E_INVAL (-1)      /* bad argument */
#define BCW_E_HIP (-2)        /* a HIP runtime call failed */
#define BCW_E_NOMEM (-3)      /* device / host allocation failed */
#define BCW_E_CAPACITY (-4)   /* output table too small: see bcw_decode_result.n_records_total */
#define BCW_E_NODEVICE (-5)   /* no HIP device */
#define BCW_E_IO (-6)         /* a pread / pwrite failed or hit end of file */

/* ---- reference constants (wal.go:45-58, record.go:44-48) ---- */
#define BCW_BLOCK_SIZE 32768u
#define BCW_HEADER_SIZE 7u
#define BCW_SUPER_BLOCK_SIZE 40u
#define BCW_MAGIC 0x77616C64ull
#define BCW_RECORD_FULL 1
#define BCW_RECORD_FIRST 2
#define BCW_RECORD_MIDDLE 3
#define BCW_RECORD_LAST 4

/* ---- per-record parse status (record.go:140-239 / hint.go:50-84) ---- */
#define BCW_ST_OK 0
#define BCW_ST_INVALID 1     /* errors.New("invalid data") / ErrCorruptedHintRecord */
#define BCW_ST_PANIC 2       /* the Go reference panics on these bytes (slice bounds) */
#define BCW_ST_UNSUPPORTED 3 /* a length >= 2^32 (not representable in this table) */

/* ---- segment-level error class of the first failing fragment (wal_iterator.go:75-96) ---- */
#define BCW_ERR_NONE 0  /* iteration reached EOF (ErrWalIteratorEOF, swallowed by IterateRecord) */
#define BCW_ERR_CRC 1   /* ErrWalMismatchCRC */
#define BCW_ERR_TYPE 2  /* ErrWalUnknownRecordType */
#define BCW_ERR_PANIC 3 /* startOff > file size: the reference panics slicing i.buf[:negative] */
#define BCW_ERR_INTERNAL 4 /* the decode gave up on an internal wait (a library bug): no valid result, no rows */

/* ---- super block load result (wal.go:362-398) ---- */
#define BCW_SB_OK 0
#define BCW_SB_SHORT 1      /* file shorter than 40 bytes (ReadAt -> io.EOF) */
#define BCW_SB_CRC 2        /* ErrWalMismatchCRC */
#define BCW_SB_MAGIC 3      /* ErrWalMismatchMagic */
#define BCW_SB_BLOCKSIZE 4  /* ErrWalMismatchBlockSize */

#define BCW_MODE_RECORD 0 /* data WAL: RecordFromBytes per record */
#define BCW_MODE_HINT 1   /* hint WAL: HintRecord.Decode per record */

typedef struct bcw_super_block {
  uint64_t magic;
  uint64_t block_size;
  uint32_t start_off;
  uint32_t crc;
  uint64_t create_time;
  uint64_t base_time;
} bcw_super_block;

/* Decode parameters. ns_size / etag_size replace the process-global gOpts read by the
 * reference codec (record.go:141,178; hint.go:51). start_off / base_time come from the WAL's
 * super block (LoadWal, wal.go:218-259). */
typedef struct bcw_decode_params {
  uint64_t seg_len;   /* file size in bytes (Wal.Size) */
  uint64_t base_time; /* super block baseTime (IterateRecord passes wal.BaseTime()) */
  uint32_t start_off; /* super block startOff (Wal.offset) */
  uint32_t ns_size;
  uint32_t etag_size;
  uint32_t mode;      /* BCW_MODE_RECORD or BCW_MODE_HINT */
} bcw_decode_params;

/* Struct-of-arrays record table. All arrays are DEVICE pointers with `capacity` entries.
 * Row r describes the r-th record the reference iterator emits (in file order).
 *   record mode: expire = decoded expire incl. baseTime; key/val/meta_len = varint lengths;
 *                hdr_size = data[0]; flags = flag byte; etag_off = offset of the etag field.
 *   hint mode:   key_len, hdr_size = key offset mod 256 (exact when ns_size <= 245; the key starts at
 *                ns_size + the length of the keyLen varint); expire = fid; aux0 = off; aux1 = size.
 * foff is the iterator offset (data start of the record's first non-empty fragment,
 * wal_iterator.go:70-72); callers subtract BCW_HEADER_SIZE as compaction.go:302 does.
 * first_frag / emit_frag are global fragment indices: the record's bytes are the data of
 * fragments [first_frag, emit_frag] (a Full emission: only emit_frag). */
typedef struct bcw_record_table {
  uint64_t capacity;
  uint64_t* foff;
  uint64_t* size;
  uint64_t* expire;
  uint64_t* aux0; /* hint mode only (may be NULL in record mode) */
  uint64_t* aux1; /* hint mode only (may be NULL in record mode) */
  uint32_t* key_len;
  uint32_t* val_len;
  uint32_t* meta_len;
  uint32_t* first_frag;
  uint32_t* emit_frag;
  uint8_t* hdr_size;
  uint8_t* flags;
  uint8_t* etag_off;
  uint8_t* status;
} bcw_record_table;

/* Segment-level outcome, written by the device (async API) or the host (sync API).
 * The Go shim replays rows [0, n_records) in order through the existing callbacks, stops at the
 * first row whose status != BCW_ST_OK (mapped to the reference's error), and otherwise returns
 * the error of err_class (or nil when BCW_ERR_NONE). That reproduces IterateRecord exactly. */
typedef struct bcw_decode_result {
  uint64_t n_records;       /* records emitted before the first failing fragment */
  uint64_t n_records_total; /* records emitted by the whole framing (>= n_records) */
  uint64_t n_frags;         /* fragments parsed by the iterator up to (incl.) err_frag or EOF */
  uint64_t err_frag;        /* global index of the first failing fragment, UINT64_MAX if none */
  uint64_t err_file_off;    /* file offset of that fragment's header (0 if none) */
  int32_t err_class;        /* BCW_ERR_* */
  int32_t first_bad_record; /* first row < n_records with status != OK, or -1 (capped at INT32_MAX) */
  uint64_t n_blocks;
  /* != 0: the context's fragment scratch was too small for this segment; the outputs are invalid.
   * Call bcw_ctx_reserve_fragments(ctx, retry_frag_capacity) and decode again (the sync API does
   * this itself). */
  uint64_t retry_frag_capacity;
  /* decode generation (unique per context and call): bcw_encode_segment_async checks that the result
   * it is given belongs to the context's latest decode, whose fragment table it reads */
  uint64_t generation;
} bcw_decode_result;

/* Fragment table (device arrays, `capacity` entries, global fragment order). */
typedef struct bcw_frag_table {
  uint64_t capacity;
  uint64_t* data_off; /* file offset of the fragment data */
  uint32_t* len;      /* length after the clamp of wal_iterator.go:75 */
  uint32_t* stored_crc;
  uint8_t* type;
  uint8_t* crc_ok;
} bcw_frag_table;

/* ---- library ---- */
int bcw_abi_version(void);
const char* bcw_strerror(int code);
int bcw_device_count(void);

/* ---- context: one HIP stream + device tables + grow-only scratch, bound to one device ---- */
typedef struct bcw_ctx bcw_ctx;
int bcw_ctx_create(int device, bcw_ctx** out);
int bcw_ctx_destroy(bcw_ctx* ctx);
/* Use a caller-owned hipStream_t (passed as void*), e.g. torch.cuda.current_stream().cuda_stream.
 * NULL restores the context's own stream. */
int bcw_ctx_set_stream(bcw_ctx* ctx, void* hip_stream);
void* bcw_ctx_stream(bcw_ctx* ctx);
int bcw_ctx_sync(bcw_ctx* ctx);
int bcw_ctx_device(bcw_ctx* ctx);
/* Per-kernel HIP-event timing of the decode pipeline (events on the launch stream around each
 * selected kernel). `mask`: bit k times kernel id k (see bcw_kernel_name), -1 = all, 0 = off.
 * bcw_ctx_kernel_times synchronises, fills total_ms[k] / launches[k] for kernel ids k < n
 * accumulated since the last call, resets, and returns the number of kernel ids. */
int bcw_ctx_set_profiling(bcw_ctx* ctx, int mask);
/* Time only every `every`-th launch of each selected kernel (default 1: every launch); the others
 * run without events. */
int bcw_ctx_set_profiling_sample(bcw_ctx* ctx, int every);
int bcw_ctx_kernel_times(bcw_ctx* ctx, double* total_ms, uint64_t* launches, int n);
const char* bcw_kernel_name(int kernel_id);
/* Tuning / diagnostic options (bcw_ctx_set_option; BCW_E_INVAL for an unknown option or value):
 *   BCW_OPT_CHASE_DIRECT  k_chase workgroups (64 blocks = 2 MiB each) up to which every workgroup sums all of its
 *                         predecessors' fragment counts directly; larger segments use the decoupled look-back.
 *                         0..BCW_CHASE_DIRECT_MAX (default BCW_CHASE_DIRECT_MAX); 0 forces the look-back at
 *                         every size (the tests drive that branch on small segments with it).
 *   BCW_OPT_DECODE_PATH,  retired in round 4 (the one-launch k_scan and the two-chunk decode lost to k_chase +
 *   BCW_OPT_DECODE_CHUNKS the stream-verify k_crc on every configuration): only the value 1
 *                         is accepted (BCW_OK, no effect), any other returns BCW_E_INVAL.
 *   BCW_OPT_TEST_ABORT_WAIT  fault injection for the test suite, not for production: accepted only when the
 *                         process runs with the environment variable BCW_TEST_HOOKS=1 (else BCW_E_INVAL). In the
 *                         NEXT decode on the context, the k_chase workgroup value - 1 gives up its predecessor wait
 *                         at once (0: none, the default), as a wait that ran past its 200 ms bound would; that decode
 *                         reports BCW_ERR_INTERNAL with no rows. One-shot.
 *   BCW_OPT_FILTER_SNAPSHOT  bcw_compact_wals: 1 = this context filters its sources against a staging copy of the
 *                         index entries that point into them (the path of a context on another device), even when it
 *                         shares the index's device; 0 (default) = a context on the index's device filters against the
 *                         index itself. Both give the same keep masks.
 *   BCW_OPT_XCD_BALANCE   1 (default): the CRC pass splits the segment over the XCDs in proportion to their stream
 *                         rates measured by the previous decode on the context; 0: equal bytes per workgroup. Only
 *                         the work split changes, never a result. */
#define BCW_OPT_CHASE_DIRECT 1
#define BCW_OPT_DECODE_PATH 2
#define BCW_OPT_DECODE_CHUNKS 3
#define BCW_OPT_TEST_ABORT_WAIT 4
#define BCW_OPT_FILTER_SNAPSHOT 5
#define BCW_OPT_XCD_BALANCE 6
#define BCW_CHASE_DIRECT_MAX 1024
/* the largest segment a decode accepts (2^24 blocks of 32 KiB: 512 GiB, beyond one MI355X's 288 GB of HBM);
 * bcw_decode_segment(_async) returns BCW_E_INVAL above it */
#define BCW_MAX_SEGMENT (1ull << 39)
int bcw_ctx_set_option(bcw_ctx* ctx, int option, uint64_t value);
/* Size the context's fragment scratch for at least n fragments on the next decode (after a decode
 * reported retry_frag_capacity). n must be < 2^32 - 16 (BCW_E_INVAL otherwise, nothing stored). */
int bcw_ctx_reserve_fragments(bcw_ctx* ctx, uint64_t n);

/* ---- host helpers (no device work) ---- */
uint32_t bcw_crc32c_masked(const uint8_t* p, uint64_t n);
int bcw_load_super_block(const uint8_t* p, uint64_t n, bcw_super_block* out);
void bcw_write_super_block(uint8_t out[40], uint64_t create_time, uint64_t base_time);
/* Upper bound of records / fragments a segment of seg_len bytes can hold. */
uint64_t bcw_max_fragments(uint64_t seg_len, uint32_t start_off);
/* WalRecordSize (wal.go:61-86): physical footprint (headers, data and any padding the writer puts
 * inside the record's span) of a size-byte payload whose first header is at file offset `offset`
 * (offset >= 40; the reference's uint64 arithmetic wraps below, so does this). */
uint64_t bcw_wal_record_size(uint64_t offset, uint64_t size);
/* WalBlockIndexRange (wal.go:88-97): first block index, its file offset, and the number of blocks the
 * record's span touches (uint64 arithmetic as in the reference). */
void bcw_wal_block_index_range(uint64_t offset, uint64_t size, uint64_t* first_blk_idx, uint64_t* first_blk_off,
                               uint64_t* blk_num);

/* ---- decode ----
 * Async, device-resident: d_seg is a device pointer to the whole file image (super block
 * included), d_result a device pointer to one bcw_decode_result. Launches on the context stream,
 * does not synchronise. If the table is too small, d_result->n_records_total still tells the size
 * needed and rows beyond capacity are not written (check after sync). */
int bcw_decode_segment_async(bcw_ctx* ctx, const uint8_t* d_seg, const bcw_decode_params* p,
                             const bcw_record_table* d_table, bcw_decode_result* d_result);
/* Synchronous, host in / host out: copies seg (host) to the device, decodes, copies the table
 * (host arrays in h_table) and the result back. Returns BCW_E_CAPACITY when h_table is too small. */
int bcw_decode_segment(bcw_ctx* ctx, const uint8_t* h_seg, const bcw_decode_params* p,
                       const bcw_record_table* h_table, bcw_decode_result* h_result);
/* Fragment table of the most recent decode on this context (device arrays), global order. */
int bcw_decode_fragments_async(bcw_ctx* ctx, const bcw_frag_table* d_frags);
/* Same, into host arrays (synchronous). *n_total receives the number of fragments the framing
 * has (rows beyond h_frags->capacity are not copied). After a decode that reported BCW_ERR_INTERNAL both
 * deliver no row (n_total 0): that decode's fragment table and verdicts are not valid. */
int bcw_decode_fragments(bcw_ctx* ctx, const bcw_frag_table* h_frags, uint64_t* n_total);

/* ---- host WAL writer (wal.go:490-553 with Record.Encode record.go:57-138) ----
 * Synthetic segment builder for benchmarks and tests: records of ns ('A'+i%26 bytes), a
 * key_len-byte key (record index LE + splitmix64 bytes) and a value of value_len splitmix64 bytes
 * (value_mode 1: 128*k bytes, k ~ Zipf(1.1) on [1,512]); no etag/expire/meta; createTime =
 * baseTime. Records are appended while the file is shorter than target_bytes (and fewer than
 * max_records if max_records != 0). h_out (host) receives the file image when out_cap suffices;
 * with h_out == NULL only the size is computed. Returns BCW_OK or BCW_E_CAPACITY. */
int bcw_synth_segment(uint64_t target_bytes, uint64_t max_records, uint64_t seed, uint32_t ns_size,
                      uint32_t key_len, uint32_t value_len, int value_mode, uint64_t base_time,
                      uint8_t* h_out, uint64_t out_cap, uint64_t* out_len, uint64_t* out_records);

/* ---- encode: compaction re-encode (compactOneWal) and hint rebuild (NewHintByWal) ---- */
#define BCW_ENC_COMPACT 0 /* kept records re-encoded into the dst WAL + one hint each (compaction.go:294-327) */
#define BCW_ENC_HINT 1    /* a hint per delivered record of a data WAL (hint.go:123-161) */

#define BCW_ENC_ERR_NONE 0
#define BCW_ENC_ERR_SRC 1    /* IterateRecord failed: a bad row (err_record) or a fragment error (err_record -1,
                                src_err_class); everything before it was written, as in the reference */
#define BCW_ENC_ERR_EXPIRE 2 /* Record.Encode: errors.New("invalid expire") (record.go:74) at err_record */
#define BCW_ENC_ERR_PANIC 3  /* Record.Encode panics at err_record: expire delta >= 2^35 overflows
                                `var expireBytes [binary.MaxVarintLen32]byte` (record.go:67,78) */
#define BCW_ENC_ERR_TABLE 4  /* the source table is smaller than the decode's n_records, or the decode reported
                                BCW_ERR_INTERNAL: nothing encoded / applied */
#define BCW_ENC_ERR_STALE 5  /* d_src_result is not the context's latest decode (its fragment table was
                                replaced, e.g. by a hint decode): nothing encoded */

typedef struct bcw_encode_params {
  uint64_t src_len;       /* source WAL file size */
  uint64_t dst_base_time; /* Record.Encode baseTime: dst.Wal().BaseTime() (compaction.go:308) */
  uint64_t fid;           /* hint fid: the dst fid (compaction.go:318) or the data WAL's fid (hint.go:142) */
  uint64_t wal_pos;       /* dst WAL file size before the append (Wal.writeOffset(false), wal.go:482-487), >= 40 */
  uint64_t hint_pos;      /* hint WAL file size before the append, >= 40 */
  uint32_t src_start_off; /* source super block startOff */
  uint32_t mode;          /* BCW_ENC_COMPACT or BCW_ENC_HINT */
  uint32_t ns_size;       /* gOpts.NsSize */
  uint32_t etag_size;     /* gOpts.EtagSize */
} bcw_encode_params;

/* Outputs. wal / hint receive the bytes appended to each file: out[0] is file offset wal_pos /
 * hint_pos (the super block of a new file is bcw_write_super_block's job). rec_off (may be NULL):
 * per source row, the offset WriteRecord returned for the row's record in the dst WAL, UINT64_MAX
 * when not written. Async API: device arrays; rec_off has the source table's capacity (rec_off_cap is
 * ignored). Sync API: host arrays; rec_off has rec_off_cap entries, rows >= n_in are never written,
 * and BCW_E_CAPACITY is returned (result filled, nothing copied) when rec_off_cap < n_in. */
typedef struct bcw_encode_out {
  uint8_t* wal;
  uint64_t wal_cap;
  uint8_t* hint;
  uint64_t hint_cap;
  uint64_t* rec_off;
  uint64_t rec_off_cap;
} bcw_encode_out;

typedef struct bcw_encode_result {
  uint64_t n_in;         /* source rows fully processed before the iteration stopped (error row excluded) */
  uint64_t n_written;    /* records appended (dst WAL and hint WAL) */
  uint64_t wal_end;      /* dst WAL file size after the append */
  uint64_t hint_end;     /* hint WAL file size after the append */
  uint64_t wal_need;     /* bytes appended = wal_end - wal_pos */
  uint64_t hint_need;
  int64_t err_record;    /* source row of the error, -1 if none / a fragment error */
  int32_t err_class;     /* BCW_ENC_ERR_* */
  int32_t src_err_class; /* the decode's BCW_ERR_* */
  uint32_t wal_events;   /* layout events (blocks starting exactly at a record header) */
  uint32_t hint_events;
  uint32_t fits;         /* 0: an output capacity was too small, nothing was written */
  uint32_t _pad;
} bcw_encode_result;

/* Async, device-resident. d_src / d_table / d_src_result must be the inputs and outputs of the most
 * recent bcw_decode_segment_async (BCW_MODE_RECORD) on this context: the encode reads the context's
 * fragment table, and reports BCW_ENC_ERR_STALE (nothing written) when d_src_result->generation is not
 * that decode's. d_keep[i] != 0 keeps source row i (the doFilter verdict, compaction.go:303;
 * ignored for BCW_ENC_HINT). Launches on the context stream; d_result (device) receives the outcome. */
int bcw_encode_segment_async(bcw_ctx* ctx, const uint8_t* d_src, const bcw_encode_params* p,
                             const bcw_record_table* d_table, const bcw_decode_result* d_src_result,
                             const uint8_t* d_keep, const bcw_encode_out* d_out, bcw_encode_result* d_result);
/* Synchronous, host in / host out: decodes h_src, then encodes (n_keep entries of h_keep, missing
 * ones count as dropped). Returns BCW_E_CAPACITY (result filled, nothing copied) when an output is
 * too small: h_result->wal_need / hint_need / n_in tell the sizes. */
int bcw_encode_segment(bcw_ctx* ctx, const uint8_t* h_src, const bcw_encode_params* p, const uint8_t* h_keep,
                       uint64_t n_keep, const bcw_encode_out* h_out, bcw_encode_result* h_result);

/* ---- device index: the bitcaskDB index (index.go) resident in HBM -------------------------------
 * Observable semantics of Index.Get/Put/Delete/SoftDelete (index.go:81-165): a map from MergedKey(ns, key)
 * = ns || key (utils.go:133-139) to (fid, off, size), hashed with murmur3 Sum64 (index.go:15-19). Get
 * reports ErrKeyNotFound, or ErrKeySoftDeleted when off == 0. Unbounded by default (the index grows); the
 * reference's sampled approximate-LRU eviction (map.go:349-420) has a deterministic counterpart,
 * bcw_index_set_limit below. For exact parity with a bounded Go index (IndexLimited below the key count) keep the
 * Go index authoritative and run the device filter against a snapshot of it (bcw_index_clear + bcw_index_apply
 * of its live entries).
 * Batches keep the reference's sequential order: the last operation on a key wins. An index is bound to
 * the context it was created on (its stream and device; the table-driven calls read that context's
 * fragment table of its latest decode). */
typedef struct bcw_index bcw_index;
#define BCW_IDX_PUT 0
#define BCW_IDX_DELETE 1
#define BCW_IDX_SOFT_DELETE 2
#define BCW_IDX_FOUND 0
#define BCW_IDX_NOT_FOUND 1    /* ErrKeyNotFound */
#define BCW_IDX_SOFT_DELETED 2 /* ErrKeySoftDeleted (value still reported) */
#define BCW_IDX_ERR_FULL 6     /* the slot table overflowed (not expected: capacity is managed by the host) */

/* Outcome of a table-driven index call (device struct). err_class: 0, BCW_ENC_ERR_STALE (d_result is not
 * the context's latest decode), BCW_ENC_ERR_TABLE (table smaller than the decode) or BCW_IDX_ERR_FULL. */
typedef struct bcw_index_result {
  uint64_t n_in;   /* rows the iteration delivers: before the first rejected row (record.go:246-263) */
  uint64_t n_done; /* put: rows applied; filter: rows kept */
  int32_t err_class;
  int32_t _pad;
} bcw_index_result;

typedef struct bcw_index_info {
  uint64_t live;          /* keys present (Get finds them, soft-deleted included) */
  uint64_t slots_used;    /* slots claimed (live + deleted keys) */
  uint64_t slot_capacity;
  uint64_t arena_used;    /* key arena bytes */
  uint64_t arena_capacity;
  uint64_t overflow;      /* != 0: an operation found no slot (index inconsistent) */
  uint64_t limited;       /* the capacity bound (bcw_index_set_limit), 0: none */
  uint64_t evicted;       /* keys evicted by the bound so far */
  uint64_t evicted_bytes; /* their value sizes (the WriteStat.FreeBytes of the evictions, index.go:144-165) */
} bcw_index_info;

/* keys / arena_bytes: initial sizing (both grow on demand) */
int bcw_index_create(bcw_ctx* ctx, uint64_t keys, uint64_t arena_bytes, bcw_index** out);
int bcw_index_destroy(bcw_index* ix);
int bcw_index_reserve(bcw_index* ix, uint64_t keys, uint64_t arena_bytes);
int bcw_index_stats(bcw_index* ix, bcw_index_info* out);
/* IndexLimited (db.go:71, db_impl.go:165): bound the index to `limited` keys (0: unbounded, else >= 16), kept as
 * map.go's ShardMap keeps it -- 16 shards by hash % 16, Limited / 16 keys each -- with a deterministic eviction in
 * place of the reference's Rand-sampled one (map.go:395-420; exact parity with Rand is not possible): an entry's
 * expire is the sequence number of the last op that set it, and after every batch (apply, put / recover of a
 * decoded table, the fan-out's ordered puts) each shard over its limit evicts its least recently set entries until
 * it holds its limit. A Get of an evicted key fails (ErrKeyNotFound), so the compaction filter drops its rows. The
 * evictions are counted in bcw_index_info (evicted, evicted_bytes). Applies the bound at once. */
int bcw_index_set_limit(bcw_index* ix, uint64_t limited);
/* Index.Put / Delete / SoftDelete of n merged keys (host arrays; key i = h_keys[h_key_off[i], h_key_off[i+1]),
 * h_ops[i] = BCW_IDX_*), applied in order (the Go shim mirrors DBImpl.writeIndex, db_impl.go:433-452).
 * Synchronous. */
int bcw_index_apply(bcw_index* ix, uint64_t n, const uint8_t* h_keys, const uint64_t* h_key_off,
                    const uint8_t* h_ops, const uint64_t* h_fid, const uint64_t* h_off, const uint64_t* h_size);
/* bcw_index_apply plus the WriteStat of every op (index.go:100-165), for DBImpl.writeIndex's freed-bytes map
 * (db_impl.go:433-452, manifest.Apply db_impl.go:402): h_found[i] = 1 when op i replaced or removed a value
 * (the key was present before it: a previous op of the same batch counts), h_free_fid[i] / h_free_bytes[i] =
 * that value's fid / valueSize (0, 0 when h_found[i] = 0). The Go shim sums writeStats[free_fid] += free_bytes
 * exactly as writeIndex does. A Put of a new key reports nothing; evictions by bcw_index_set_limit's bound are
 * counted in bcw_index_info instead -- with a bounded Go index (IndexLimited below the key count) the reference
 * reports the evicted entry on the Put: keep the Go index authoritative then ("bounded index").
 * Synchronous. */
int bcw_index_apply_stat(bcw_index* ix, uint64_t n, const uint8_t* h_keys, const uint64_t* h_key_off,
                         const uint8_t* h_ops, const uint64_t* h_fid, const uint64_t* h_off, const uint64_t* h_size,
                         uint8_t* h_found, uint64_t* h_free_fid, uint64_t* h_free_bytes);
/* Remove every key (capacity kept). With bcw_index_apply of the Go index's live entries this loads a snapshot
 * of a bounded (evicting) Go index for the device compaction filter ("bounded index"). */
int bcw_index_clear(bcw_index* ix);
/* Index.Get of n merged keys (host arrays): status BCW_IDX_* and the value per key. Synchronous. */
int bcw_index_get(bcw_index* ix, uint64_t n, const uint8_t* h_keys, const uint64_t* h_key_off, uint64_t* h_fid,
                  uint64_t* h_off, uint64_t* h_size, uint8_t* h_status);
/* The Put loops that rebuild the index from a decoded WAL (async, on the context stream, after
 * bcw_decode_segment_async of d_seg on this index's context), for every delivered row in order:
 *   BCW_MODE_RECORD  recoverFromWal  db_impl.go:305-313  Put(ns, key, fid, foff - 7, size)
 *   BCW_MODE_HINT    recoverFromWal  db_impl.go:290-299  Put(ns, key, fid, hint.off, hint.size)
 *                    use_record_fid: onePhase compaction.go:248-251  Put(ns, key, hint.fid, ...)
 * Callers apply files in ascending fid order (db_impl.go:274-281): later calls override. d_out (device,
 * may be NULL) receives the outcome. */
int bcw_index_put_decoded_async(bcw_index* ix, const uint8_t* d_seg, const bcw_decode_params* p,
                                const bcw_record_table* d_table, const bcw_decode_result* d_result, uint64_t fid,
                                int use_record_fid, bcw_index_result* d_out);
/* compactOneWal's doFilter (compaction.go:329-348) on the device, for every delivered row of a decoded
 * data WAL: d_keep[i] = 1 when Index.Get(ns, key) succeeds and still points at (src_fid, foff - 7)
 * (compaction.go:302), else 0 (rows not delivered: 0). The user CompactionFilter, when configured, stays a
 * host callback over the kept rows. d_keep has the table's capacity; it feeds bcw_encode_segment_async
 * directly (decode -> filter -> encode without leaving HBM). */
int bcw_compact_filter_async(bcw_index* ix, const uint8_t* d_seg, const bcw_decode_params* p,
                             const bcw_record_table* d_table, const bcw_decode_result* d_result, uint64_t src_fid,
                             uint8_t* d_keep, bcw_index_result* d_out);
/* Every live entry (merged key, fid, off, size), in no particular order, into host arrays (h_key_off has
 * entries_cap + 1 entries). Returns BCW_E_CAPACITY when too small (*n_out / *key_bytes tell the sizes). */
int bcw_index_export(bcw_index* ix, uint8_t* h_keys, uint64_t keys_cap, uint64_t* h_key_off, uint64_t* h_fid,
                     uint64_t* h_off, uint64_t* h_size, uint64_t entries_cap, uint64_t* n_out, uint64_t* key_bytes);
/* bcw_index_export restricted to the live entries whose value fid is one of h_fids[0, n_fids) (n_fids 0: all):
 * the slice of the index that points into a set of WAL files (the compaction fan-out's filter snapshot). */
int bcw_index_export_fids(bcw_index* ix, const uint64_t* h_fids, uint64_t n_fids, uint8_t* h_keys, uint64_t keys_cap,
                          uint64_t* h_key_off, uint64_t* h_fid, uint64_t* h_off, uint64_t* h_size,
                          uint64_t entries_cap, uint64_t* n_out, uint64_t* key_bytes);
/* Synchronous compaction of one source WAL with the device filter: decode -> doFilter against the index
 * -> Record.Encode + WriteRecord + hint append (compaction.go:294-327 with doFilter compaction.go:329-348
 * and no user CompactionFilter), host in / host out like bcw_encode_segment. h_filter (may be NULL)
 * receives the filter's outcome (n_done = rows kept). ix must belong to ctx (BCW_E_INVAL otherwise). */
int bcw_compact_segment(bcw_ctx* ctx, bcw_index* ix, const uint8_t* h_src, const bcw_encode_params* p,
                        uint64_t src_fid, const bcw_encode_out* h_out, bcw_encode_result* h_result,
                        bcw_index_result* h_filter);
/* Synchronous recoverFromWal step (db_impl.go:286-313) for one file: decode h_seg (p->mode: BCW_MODE_HINT for a
 * hint file, BCW_MODE_RECORD for a data WAL) and put every delivered row into the index. h_dres (may be
 * NULL) receives the decode result: a hint file whose iteration failed is followed, as in the reference,
 * by the data WAL of the same fid. ix must belong to ctx (BCW_E_INVAL otherwise). */
int bcw_index_recover_segment(bcw_ctx* ctx, bcw_index* ix, const uint8_t* h_seg, const bcw_decode_params* p,
                              uint64_t fid, int use_record_fid, bcw_decode_result* h_dres, bcw_index_result* h_out);
/* ---- one process, several devices: the fan-outs of a Go caller that drives several GPUs -------------------------
 * Each takes n_ctx contexts (any devices, one host thread each) and the index; INTEGRATION.md shows the cgo loop.
 * The puts into the index and the appends to the dst files keep the reference's order; only the decodes (and
 * their uploads) run concurrently. Every context is named once (BCW_E_INVAL otherwise: each worker thread owns its
 * context's decode scratch). The index's own context may be one of ctxs: the index calls the caller's thread makes
 * meanwhile (the ordered puts, the filter snapshot) use only that context's device and stream, their staging
 * buffers are the index's own, and HIP orders the two threads' work on the one stream. */
typedef struct bcw_recover_file {
  uint64_t fid;
  const uint8_t* wal;       /* the data WAL file */
  bcw_decode_params wal_p;  /* BCW_MODE_RECORD */
  const uint8_t* hint;      /* the hint WAL file, NULL when LoadWal of the hint failed (db_impl.go:288-291) */
  bcw_decode_params hint_p; /* BCW_MODE_HINT */
} bcw_recover_file;

#define BCW_RECOVER_NOT_RUN 0
#define BCW_RECOVER_HINT 1      /* the hint's puts (its iteration succeeded, or it stopped recovery) */
#define BCW_RECOVER_HINT_WAL 2  /* the hint's puts, then the data WAL's (the hint iteration failed) */
#define BCW_RECOVER_WAL 3       /* the data WAL's puts (no hint file) */
typedef struct bcw_recover_status {
  int32_t used; /* BCW_RECOVER_* */
  int32_t rc;   /* BCW_OK or the error of this file's calls */
  bcw_decode_result hint_dres, wal_dres;
  bcw_index_result hint_ires, wal_ires;
} bcw_recover_status;

/* recoverFromWals (db_impl.go:268-314). Files (any order) are taken in ascending fid; the k-th goes to
 * ctxs[k % n_ctx], whose thread decodes its hint (and its data WAL when the hint iteration fails) into a staging
 * index of its own, concurrently with the other contexts. The staging index holds the file's last put per key:
 * the index receives those, file by file, in ascending fid -- the state the reference's serial Put loop leaves.
 * Recovery stops at the first file whose data WAL iteration fails (rejected row or fragment error), whose put
 * failed (hint/wal_ires.err_class), whose hint decode gave up (BCW_ERR_INTERNAL) or whose calls failed (rc):
 * that file's puts are applied (the reference returns its error after them), later files' are not. A failed put
 * (a staging or index capacity error, hint_ires / wal_ires.err_class) has no counterpart in the reference, whose
 * Index.Put does not fail: it stops recovery here as in the serial path (parity unpinned for that case).
 * st (n_files entries, in files[] order) receives each file's outcome; *stop_file the files[] index of the
 * stopping file, -1 when every file was applied. Returns BCW_OK, or an error of the index's own calls. */
int bcw_recover_wals(bcw_index* ix, bcw_ctx* const* ctxs, uint32_t n_ctx, const bcw_recover_file* files,
                     uint64_t n_files, bcw_recover_status* st, int64_t* stop_file);

typedef struct bcw_compact_src {
  uint64_t fid;          /* the source WAL's fid (doFilter's srcFid) */
  const uint8_t* data;   /* the source WAL file */
  uint64_t len;
  uint32_t start_off;    /* its super block startOff */
  uint32_t _pad;
  bcw_encode_out out;    /* this source's appended dst WAL bytes, hint bytes and offsets per row */
} bcw_compact_src;

/* doCompactionWork's loop (compaction.go:201-211) of compactOneWal with doFilter (compaction.go:294-348, no user
 * CompactionFilter): the sources, in the given order, append to one dst WAL and one hint WAL. Source k goes to
 * ctxs[k % n_ctx], whose thread uploads, decodes and filters it concurrently with the other contexts; the encodes
 * run in source order, each starting where the previous one ended. The filter reads a snapshot of the index's
 * entries that point into the sources' fids, taken when the call starts (bcw_index_export_fids): the same
 * keep mask as a lookup in the index when no write lands in between (the reference's compaction races writes
 * in the same window, compaction.go:181-200). dst: dst_base_time, fid, wal_pos, hint_pos, ns_size, etag_size
 * (src_len, src_start_off and mode are per source / BCW_ENC_COMPACT). res / filt (n_src entries): each source's
 * bcw_compact_segment outcome. *n_done: sources whose output is final -- the last one may carry an error
 * (res.err_class != 0: the caller raises it, as doCompactionWork returns it after its appends). Returns
 * BCW_E_CAPACITY when source *n_done's output did not fit its bcw_encode_out (res[*n_done] tells the sizes:
 * resume from it with wal_pos = res[*n_done - 1].wal_end), else BCW_OK or an error of the calls. */
int bcw_compact_wals(bcw_index* ix, bcw_ctx* const* ctxs, uint32_t n_ctx, const bcw_compact_src* srcs,
                     uint64_t n_src, const bcw_encode_params* dst, bcw_encode_result* res, bcw_index_result* filt,
                     uint64_t* n_done);

/* IndexOperator.Hash (index.go:15-19): murmur3 (spaolacci/murmur3 v1.1.0) New64().Sum64() on the host */
uint64_t bcw_murmur3_sum64(const uint8_t* p, uint64_t n);

/* ---- batched point reads (Get / GetV2's record fetch, db_impl.go:567-631) -----------------------------
 * For each request (offset, size) -- an index value -- Wal.ReadRecord (wal.go:556-573: WalRecordSize,
 * one read of the record's physical span) + WalParseRecord (wal.go:121-173) + RecordFromBytes
 * (record.go:140-239) against a WAL image resident in HBM. rd_status per request: */
#define BCW_RD_OK 0
#define BCW_RD_BEYOND 1     /* errors.New("read beyond file size") (wal.go:562-564) */
#define BCW_RD_CORRUPTED 2  /* ErrWalCorruptedData: a fragment length beyond the buffer */
#define BCW_RD_CRC 3        /* ErrWalMismatchCRC (verifyChecksum) */
#define BCW_RD_SIZE 4       /* ErrWalMismatchSize */
#define BCW_RD_TYPE 5       /* ErrWalUnknownRecordType */
#define BCW_RD_INCOMPLETE 6 /* ErrWalIncompleteRecord */
#define BCW_RD_PANIC 7      /* the reference panics (size 0: the header slice of an empty buffer) */

typedef struct bcw_read_params {
  uint64_t seg_len;   /* the WAL image's size (Wal.size) */
  uint64_t base_time; /* wal.BaseTime() for RecordFromBytes */
  uint32_t ns_size;
  uint32_t etag_size;
  uint32_t verify;    /* ReadOptions.VerifyChecksum */
  uint32_t _pad;
} bcw_read_params;

/* Async, device-resident: request i reads d_size[i] payload bytes into d_payload + d_pay_off[i]; d_table
 * (may be NULL) receives RecordFromBytes' fields and status (foff = offset + 7) when rd_status == OK. */
int bcw_read_records_async(bcw_ctx* ctx, const uint8_t* d_seg, const bcw_read_params* p, uint64_t n,
                           const uint64_t* d_off, const uint64_t* d_size, const uint64_t* d_pay_off,
                           uint8_t* d_payload, uint8_t* d_rd_status, const bcw_record_table* d_table);
/* Synchronous, host in / host out: payloads concatenated in request order into h_payload (sum of sizes). */
int bcw_read_records(bcw_ctx* ctx, const uint8_t* h_seg, const bcw_read_params* p, uint64_t n,
                     const uint64_t* h_off, const uint64_t* h_size, uint8_t* h_payload, uint8_t* h_rd_status,
                     const bcw_record_table* h_table);

/* ---- host I/O staging: WAL files <-> HBM through pinned slices ---------------------------------------
 * The reference reads a segment with PreadFull per 32 KiB block (utils.go:32-48, wal_iterator.go:55)
 * and writes the rewritten WAL through a buffer flushed every >= 1 MiB (WalRewriter
 * wal_rewriter.go:37-49 -> Wal.Flush wal.go:451-465). A stage owns `nslices` pinned host buffers of
 * `slice_bytes`; reads pread whole slices (up to `threads` reader threads) while earlier slices are
 * already copied to the device, writes copy slices back and pwrite them on writer threads while the next copies are in flight.
 * Copies are queued on hip_stream (a hipStream_t; NULL: the context's stream), so a decode launched on
 * that stream after bcw_stage_read returns sees the whole segment. */
typedef struct bcw_stage bcw_stage;
int bcw_stage_create(bcw_ctx* ctx, uint64_t slice_bytes, uint32_t nslices, bcw_stage** out);
int bcw_stage_destroy(bcw_stage* st);
/* len bytes of fd at file_off -> d_dst (device). Returns BCW_E_IO on a read error or a short file. A descriptor
 * opened with O_DIRECT is read past the page cache (the reference's io_uring block reader, block_reader/
 * iouring.go:47-76): file_off and slice_bytes must then be multiples of 4096 (else BCW_E_INVAL). */
int bcw_stage_read(bcw_stage* st, int fd, uint64_t file_off, uint64_t len, uint8_t* d_dst, void* hip_stream,
                   uint32_t threads);
/* len bytes of d_src (device) -> fd at file_off: each slice is copied back after the work queued on
 * hip_stream and pwritten by one of up to `threads` writer threads while the others' copies proceed.
 * Synchronous: returns once every byte is written. */
int bcw_stage_write(bcw_stage* st, int fd, uint64_t file_off, const uint8_t* d_src, uint64_t len,
                    void* hip_stream, uint32_t threads);

/* Segments already resident in another GPU's HBM (several GPUs in one process; SURVEY.md north_star: segment buffers
 * scattered and gathered over xGMI). bcw_peer_enable lets each of the two devices map the other's memory (both
 * directions; BCW_OK when already enabled or a == b, BCW_E_HIP when the pair cannot). bcw_stage_peer copies len bytes
 * of d_src, in the HBM of device src_device, to d_dst on the context's device, device to device (over xGMI between
 * linked MI355Xs once peer access is enabled; never through host memory), queued on hip_stream (NULL: the context's
 * stream) so that a decode queued after it on that stream sees the bytes. Asynchronous. */
int bcw_peer_enable(int device_a, int device_b);
int bcw_stage_peer(bcw_ctx* ctx, uint8_t* d_dst, const uint8_t* d_src, int src_device, uint64_t len, void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif
