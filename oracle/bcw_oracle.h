/*
 * bcw_oracle.h -- CPU restatement of bitcaskDB's WAL record codec (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the MI355X codec in bitcaskdb_amd/. It restates, in plain C,
 * the reference Go code of wenzhang-dev/bitcaskDB (snapshot mounted at /root/reference):
 *   utils.go:24-29   ComputeCRC32 (CRC-32C, rotr15, +0xa282ead8)
 *   utils.go:51-57   DecodeUvarint (Go encoding/binary.Uvarint, errors -> (0,0))
 *   wal.go:29-58     super block / framing constants
 *   wal.go:332-398   writeSuperBlock / loadSuperBlock
 *   wal.go:482-553   writeOffset / WriteRecord
 *   wal_iterator.go:40-100  WalIterator.Next
 *   record.go:57-138 Record.Encode, record.go:140-239 RecordFromBytes, record.go:242-266 IterateRecord
 *   hint.go:32-84    HintRecord.Encode/Decode, hint.go:123-161 NewHintByWal, hint.go:163-188 IterateHint
 *   compaction.go:294-327 compactOneWal (re-encode of kept records into a dst WAL + hint WAL)
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 * The product path (bitcaskdb_amd/) never links or calls it.
 *
 * Parity pinning: the reference Go toolchain is absent from this image (no `go` binary), so the
 * reference cannot be compiled or run here. This oracle is pinned by (i) public known answers
 * (CRC-32C("123456789") = 0xE3069283), (ii) the reference tests' round-trip scenarios restated in
 * tests/, and (iii) golden fixtures cross-checked against an independent pure-Python restatement
 * (tests/golden/pyref.py). msgpack app-meta is treated as opaque bytes: parity unpinned there.
 */
#ifndef BCW_ORACLE_H
#define BCW_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OC_BLOCK_SIZE 32768u
#define OC_HEADER_SIZE 7u
#define OC_SUPER_SIZE 40u
#define OC_MAGIC 0x77616C64ull

enum { OC_FULL = 1, OC_FIRST = 2, OC_MIDDLE = 3, OC_LAST = 4 };

/* per-record parse status (record.go:140-239 / hint.go:50-84) */
enum {
  OC_ST_OK = 0,
  OC_ST_INVALID = 1,     /* errors.New("invalid data") or ErrCorruptedHintRecord */
  OC_ST_PANIC = 2,       /* the reference would panic (slice bounds) */
  OC_ST_UNSUPPORTED = 3  /* a length >= 2^32: not representable in the device table */
};
/* segment-level error class (first failing fragment) */
enum { OC_ERR_NONE = 0, OC_ERR_CRC = 1, OC_ERR_TYPE = 2, OC_ERR_PANIC = 3 };
/* super block load errors (wal.go:362-398) */
enum { OC_SB_OK = 0, OC_SB_SHORT = 1, OC_SB_CRC = 2, OC_SB_MAGIC = 3, OC_SB_BLOCKSIZE = 4 };

typedef struct oc_frag {
  uint64_t data_off;   /* file offset of the fragment data (header + 7) */
  uint32_t len;        /* length after the clamp of wal_iterator.go:75 */
  uint32_t stored_crc; /* header bytes [0,4) */
  uint8_t type;        /* header byte 6 */
  uint8_t crc_ok;
  uint8_t pad[6];
} oc_frag; /* 24 B */

typedef struct oc_rec {
  uint64_t foff;      /* iterator offset: data start of the record (wal_iterator.go:70-72) */
  uint64_t size;      /* len(recordBytes) */
  uint64_t expire;    /* decoded expire incl. baseTime (record.go:184-188); hint: fid */
  uint64_t key_len;   /* record: keyLen; hint: keyLen */
  uint64_t val_len;   /* record: valLen; hint: off */
  uint64_t meta_len;  /* record: metaLen; hint: size */
  uint32_t first_frag;/* first fragment whose data is part of the record */
  uint32_t emit_frag; /* fragment that completed the record (Full or Last) */
  uint8_t hdr_size;   /* record: data[0]; hint: key offset mod 256 */
  uint8_t flags;      /* record: flag byte; hint: 0 */
  uint8_t etag_off;   /* record: offset of etag/expire fields; hint: 0 */
  uint8_t status;     /* OC_ST_* */
  uint8_t pad[4];
} oc_rec; /* 64 B */

typedef struct oc_super {
  uint64_t magic, block_size;
  uint32_t start_off;
  uint64_t create_time, base_time;
  uint32_t crc;
} oc_super;

/* ---- arithmetic core ---- */
uint32_t oc_crc32c_update(uint32_t crc, const uint8_t* p, size_t n); /* raw reflected update */
uint32_t oc_crc32c(const uint8_t* p, size_t n);                       /* standard CRC-32C */
uint32_t oc_compute_crc32(const uint8_t* p, size_t n);                /* utils.go:24-29 */
uint32_t oc_crc32c_hw(const uint8_t* p, size_t n);                    /* SSE4.2 3-way (baseline) */
int oc_uvarint(const uint8_t* p, size_t n, uint64_t* v);              /* Go binary.Uvarint */
int oc_put_uvarint(uint8_t* out, uint64_t v);                         /* Go binary.PutUvarint */

/* ---- super block ---- */
void oc_super_encode(uint8_t out[40], uint64_t create_time, uint64_t base_time);
int oc_super_load(const uint8_t* p, size_t n, oc_super* out);

/* ---- writer (wal.go:490-553), growable in-memory file image ---- */
typedef struct oc_writer oc_writer;
oc_writer* oc_writer_new(uint64_t create_time, uint64_t base_time);
/* a writer whose file already holds `size` bytes, none of them materialized: data() starts at file offset base() */
oc_writer* oc_writer_new_at(uint64_t size);
uint64_t oc_writer_base(const oc_writer* w);
uint64_t oc_writer_write(oc_writer* w, const uint8_t* rec, size_t n); /* returns record offset */
uint64_t oc_writer_size(const oc_writer* w);
const uint8_t* oc_writer_data(const oc_writer* w);
void oc_writer_free(oc_writer* w);

/* ---- record / hint payload codecs ---- */
/* Record.Encode (record.go:57-138); returns payload length, -1 on "invalid expire", -2 where the reference
 * panics (expire delta needs > 5 varint bytes). */
int64_t oc_record_encode(uint8_t* out, const uint8_t* ns, size_t ns_len, const uint8_t* key, size_t key_len,
                         const uint8_t* val, size_t val_len, const uint8_t* etag, size_t etag_len,
                         uint64_t expire, int tombstone, const uint8_t* meta, size_t meta_len,
                         uint64_t base_time);
/* RecordFromBytes (record.go:140-239) into r (fields + status) */
void oc_record_parse(const uint8_t* data, size_t len, size_t cap, uint64_t base_time, uint32_t ns_size,
                     uint32_t etag_size, oc_rec* r);
/* HintRecord.Encode (hint.go:32-48) */
size_t oc_hint_encode(uint8_t* out, const uint8_t* ns, size_t ns_len, const uint8_t* key, size_t key_len,
                      uint64_t fid, uint64_t off, uint64_t size);
/* HintRecord.Decode (hint.go:50-84) into r */
void oc_hint_parse(const uint8_t* data, size_t len, uint32_t ns_size, oc_rec* r);

/* ---- segment decode: WalIterator.Next + RecordFromBytes / HintRecord.Decode ---- */
typedef struct oc_decode oc_decode;
/* mode 0: data WAL (records), 1: hint WAL. Iterates from start_off to EOF or the first fragment
 * error; every emitted record is parsed (parse errors do not stop this raw iteration). */
oc_decode* oc_decode_segment(const uint8_t* seg, uint64_t len, uint32_t start_off, uint64_t base_time,
                             uint32_t ns_size, uint32_t etag_size, int mode);
void oc_decode_counts(const oc_decode* d, uint64_t* n_frags, uint64_t* n_recs, uint64_t* err_frag,
                      int32_t* err_class, uint64_t* rec_bytes);
void oc_decode_frags(const oc_decode* d, oc_frag* dst);
void oc_decode_recs(const oc_decode* d, oc_rec* dst);
void oc_decode_bytes(const oc_decode* d, uint8_t* dst, uint64_t* offs); /* payloads, concatenated */
void oc_decode_free(oc_decode* d);

/* fast restated decode loop used as the CPU baseline (hardware CRC, no allocation per record):
 * returns records delivered; *err_class gets OC_ERR_*. */
uint64_t oc_decode_fast(const uint8_t* seg, uint64_t len, uint32_t start_off, uint64_t base_time,
                        uint32_t ns_size, uint32_t etag_size, int32_t* err_class, uint64_t* checksum);
/* the same loop reading each 32 KiB block from a file descriptor with pread (wal_iterator.go:55, PreadFull) */
uint64_t oc_decode_fast_pread(int fd, uint64_t len, uint32_t start_off, uint64_t base_time, uint32_t ns_size,
                              uint32_t etag_size, int32_t* err_class, uint64_t* checksum);

/* ---- compaction re-encode (compactOneWal) and hint rebuild (NewHintByWal) ----
 * err_class: OC_ENC_OK, OC_ENC_SRC (the source iteration failed at row *err_rec, or a fragment error when
 * *err_rec == -1), OC_ENC_EXPIRE (Record.Encode "invalid expire" at row *err_rec), OC_ENC_PANIC (Record.Encode
 * panics: expire delta >= 2^35). Records before the error are written. offs[i] = dst offset of row i or
 * UINT64_MAX (dropped / not reached); *n_in = rows visited. */
enum { OC_ENC_OK = 0, OC_ENC_SRC = 1, OC_ENC_EXPIRE = 2, OC_ENC_PANIC = 3 };
int oc_meta_app_size_zero(const uint8_t* meta, size_t n);
void oc_compact_append(oc_writer* dst, oc_writer* hint, uint64_t dst_fid, const uint8_t* seg, uint64_t len,
                       uint32_t start_off, uint64_t src_base, uint64_t dst_base, uint32_t ns_size,
                       uint32_t etag_size, const uint8_t* keep, uint64_t n_keep, uint64_t* offs,
                       int32_t* err_class, int64_t* err_rec, uint64_t* n_in);
void oc_hint_by_wal(oc_writer* hint, uint64_t fid, const uint8_t* seg, uint64_t len, uint32_t start_off,
                    uint64_t base_time, uint32_t ns_size, uint32_t etag_size, int32_t* err_class, int64_t* err_rec,
                    uint64_t* n_in);

/* ---- synthetic segments for configs A-E (deterministic, seeded) ---- */
/* value_mode 0: fixed value_len; 1: 128*k, k ~ Zipf(s=1.1) on [1,512] */
oc_writer* oc_synth_segment(uint64_t target_bytes, uint64_t max_records, uint64_t seed, uint32_t ns_size,
                            uint32_t key_len, uint32_t value_len, int value_mode, uint64_t base_time);

/* ---- framing size maths (wal.go:61-97) ---- */
uint64_t oc_wal_record_size(uint64_t offset, uint64_t size);
void oc_wal_block_index_range(uint64_t offset, uint64_t size, uint64_t* first_idx, uint64_t* first_off,
                              uint64_t* blk_num);

/* ---- payload hashes for full-size parity checks ---- */
void oc_decode_payload_hashes(const oc_decode* d, uint64_t* out);
void oc_gather_payload_hashes(const uint8_t* seg, uint64_t seg_len, const uint64_t* data_off, const uint32_t* flen,
                              uint64_t n_frags, const uint32_t* first, const uint32_t* emit, const uint64_t* size,
                              uint64_t n_recs, uint64_t* out);

/* ---- index (index.go:15-19, 81-165; compaction.go:329-348) ---- */
void oc_murmur3_128(const uint8_t* p, size_t n, uint64_t seed, uint64_t* h1, uint64_t* h2);
uint64_t oc_murmur3_sum64(const uint8_t* p, size_t n); /* spaolacci/murmur3 v1.1.0 New64().Sum64() */
typedef struct oc_index oc_index;
oc_index* oc_index_new(void);
void oc_index_free(oc_index* x);
/* op 0: Put, 1: Delete, 2: SoftDelete */
void oc_index_set(oc_index* x, const uint8_t* ns, size_t nsl, const uint8_t* key, size_t kl, int op, uint64_t fid,
                  uint64_t off, uint64_t size);
/* 0: found, 1: ErrKeyNotFound, 2: ErrKeySoftDeleted (value still returned) */
int oc_index_get(oc_index* x, const uint8_t* ns, size_t nsl, const uint8_t* key, size_t kl, uint64_t* fid,
                 uint64_t* off, uint64_t* size);
uint64_t oc_index_live(const oc_index* x);
int oc_do_filter(oc_index* x, const uint8_t* ns, size_t nsl, const uint8_t* key, size_t kl, uint64_t src_fid,
                 uint64_t src_off);
int oc_index_put_segment(oc_index* x, const uint8_t* seg, uint64_t len, uint32_t start_off, uint64_t base_time,
                         uint32_t ns_size, uint32_t etag_size, int mode, uint64_t fid, int use_rec_fid,
                         uint64_t* n_put);
uint64_t oc_compact_filter(oc_index* x, const uint8_t* seg, uint64_t len, uint32_t start_off, uint64_t base_time,
                           uint32_t ns_size, uint32_t etag_size, uint64_t src_fid, uint8_t* keep, uint64_t n_keep);

/* ---- bounded index: map.go SimpleMap (nshards 1) / ShardMap (nshards 16) with eviction ----
 * hash_mode 0: murmur3 Sum64 (IndexOperator.Hash); 1: the key's first 8 bytes little-endian (map_test.go's
 * mockSimpleMapOperator, Hash(k) = k). Rand: rand_vals cycled (v[i] % n) or, with n_rand 0, splitmix64(seed).
 * NULL when NewMap's validate fails (ErrMapOptions). Values are 3 x u64 (IndexValue{fid, off, size}). */
typedef struct oc_smap oc_smap;
oc_smap* oc_smap_new(uint32_t nshards, uint64_t capacity, uint64_t limited, uint64_t pool_cap, uint64_t sample_keys,
                     int hash_mode, const uint64_t* rand_vals, uint64_t n_rand, uint64_t seed);
void oc_smap_free(oc_smap* m);
void oc_smap_set_now(oc_smap* m, uint64_t seconds);
uint64_t oc_smap_size(const oc_smap* m);
int oc_smap_set(oc_smap* m, const uint8_t* k, size_t kl, const uint64_t val[3], uint64_t old[3]); /* 0 new, 1 replaced, 2 evicted */
int oc_smap_get(oc_smap* m, const uint8_t* k, size_t kl, uint64_t val[3]);                        /* 0 found, 1 not found */
int oc_smap_delete(oc_smap* m, const uint8_t* k, size_t kl, uint64_t old[3]);                     /* 0 deleted, 1 not found */
uint64_t oc_smap_export(const oc_smap* m, uint8_t* keys, uint64_t keys_cap, uint64_t* koff, uint64_t* vals,
                        uint64_t cap, uint64_t* key_bytes);
void oc_bindex_op(oc_smap* m, const uint8_t* ns, size_t nsl, const uint8_t* key, size_t kl, int op, uint64_t fid,
                  uint64_t off, uint64_t size, uint64_t* free_fid, uint64_t* free_bytes);
int oc_bindex_get(oc_smap* m, const uint8_t* ns, size_t nsl, const uint8_t* key, size_t kl, uint64_t* fid,
                  uint64_t* off, uint64_t* size);
int oc_bindex_put_segment(oc_smap* m, const uint8_t* seg, uint64_t len, uint32_t start_off, uint64_t base_time,
                          uint32_t ns_size, uint32_t etag_size, int mode, uint64_t fid, int use_rec_fid,
                          uint64_t* n_put);
uint64_t oc_bindex_compact_filter(oc_smap* m, const uint8_t* seg, uint64_t len, uint32_t start_off,
                                  uint64_t base_time, uint32_t ns_size, uint32_t etag_size, uint64_t src_fid,
                                  uint8_t* keep, uint64_t n_keep);

/* ---- point reads: Wal.ReadRecord + WalParseRecord (wal.go:556-573, 121-173) ---- */
enum { OC_RD_OK = 0, OC_RD_BEYOND = 1, OC_RD_CORRUPTED = 2, OC_RD_CRC = 3, OC_RD_SIZE = 4, OC_RD_TYPE = 5,
       OC_RD_INCOMPLETE = 6, OC_RD_PANIC = 7 };
int oc_read_record(const uint8_t* seg, uint64_t seg_len, uint64_t offset, uint64_t size, int verify, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif
