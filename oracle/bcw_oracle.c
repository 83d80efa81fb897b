/*
 * bcw_oracle.c -- CPU restatement of bitcaskDB's WAL record codec. TEST INFRASTRUCTURE ONLY:
 * the parity checker for bitcaskdb_amd/ (see bcw_oracle.h for the reference map and pinning).
 * Every function cites the reference file:line it restates (paths relative to /root/reference).
 */
#define _GNU_SOURCE  /* pread */
#include "bcw_oracle.h"

#include <nmmintrin.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* memcpy of n bytes; n == 0 with a NULL pointer (an empty Go slice) is allowed */
static inline void oc_memcpy(void* d, const void* s, size_t n) {
  if (n) memcpy(d, s, n);
}

/* ------------------------------------------------------------------------------------------ */
/* CRC-32C (Castagnoli), reflected poly 0x82F63B78 == Go crc32.MakeTable(crc32.Castagnoli)      */
/* ------------------------------------------------------------------------------------------ */
static uint32_t g_tab[256];
static int g_tab_init = 0;

static void crc_init(void) {
  if (g_tab_init) return;
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    g_tab[b] = c;
  }
  g_tab_init = 1;
}

uint32_t oc_crc32c_update(uint32_t crc, const uint8_t* p, size_t n) {
  crc_init();
  for (size_t i = 0; i < n; ++i) crc = (crc >> 8) ^ g_tab[(crc ^ p[i]) & 0xffu];
  return crc;
}

uint32_t oc_crc32c(const uint8_t* p, size_t n) { return ~oc_crc32c_update(0xffffffffu, p, n); }

/* utils.go:24-29: checksum>>15 | checksum<<17, plus 0xa282ead8 (uint32 wraparound) */
uint32_t oc_compute_crc32(const uint8_t* p, size_t n) {
  uint32_t c = oc_crc32c(p, n);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

/* Hardware CRC-32C with a 3-way interleave (the shape of Go's amd64 castagnoliSSE42Triple).
 * The three partial CRCs are merged with a GF(2) shift operator built once per stripe length. */
static uint32_t gf2_times(const uint32_t* mat, uint32_t vec) {
  uint32_t s = 0;
  for (int i = 0; vec; ++i, vec >>= 1)
    if (vec & 1u) s ^= mat[i];
  return s;
}
static void gf2_square(uint32_t* sq, const uint32_t* mat) {
  for (int n = 0; n < 32; ++n) sq[n] = gf2_times(mat, mat[n]);
}
/* advance a raw reflected CRC state over `len` zero bytes (the zlib crc32_combine squaring) */
static uint32_t zeros_apply(uint32_t v, size_t len) {
  uint32_t odd[32], even[32];
  odd[0] = 0x82F63B78u;
  uint32_t row = 1;
  for (int n = 1; n < 32; ++n) { odd[n] = row; row <<= 1; }
  gf2_square(even, odd); /* 2 zero bits */
  gf2_square(odd, even); /* 4 zero bits */
  do {
    gf2_square(even, odd);
    if (len & 1) v = gf2_times(even, v);
    len >>= 1;
    if (!len) break;
    gf2_square(odd, even);
    if (len & 1) v = gf2_times(odd, v);
    len >>= 1;
  } while (len);
  return v;
}
static void shift_op(uint32_t* op, size_t len) {
  for (int n = 0; n < 32; ++n) op[n] = zeros_apply(1u << n, len);
}

#define HW_STRIPE 4096u
static uint32_t g_shift_stripe[32];
static uint32_t g_shift_2stripe[32];
static int g_shift_init = 0;

static uint32_t hw_run(uint32_t c, const uint8_t* p, size_t n) {
  while (n >= 8) { uint64_t w; oc_memcpy(&w, p, 8); c = (uint32_t)_mm_crc32_u64(c, w); p += 8; n -= 8; }
  while (n) { c = _mm_crc32_u8(c, *p++); --n; }
  return c;
}

uint32_t oc_crc32c_hw(const uint8_t* p, size_t n) {
  if (!g_shift_init) {
    shift_op(g_shift_stripe, HW_STRIPE);
    shift_op(g_shift_2stripe, 2 * HW_STRIPE);
    g_shift_init = 1;
  }
  uint32_t c = 0xffffffffu;
  while (n >= 3 * HW_STRIPE) {
    uint32_t a = c, b = 0, d = 0;
    const uint8_t* q = p;
    for (size_t i = 0; i < HW_STRIPE; i += 8) {
      uint64_t w0, w1, w2;
      oc_memcpy(&w0, q + i, 8); oc_memcpy(&w1, q + HW_STRIPE + i, 8); oc_memcpy(&w2, q + 2 * HW_STRIPE + i, 8);
      a = (uint32_t)_mm_crc32_u64(a, w0);
      b = (uint32_t)_mm_crc32_u64(b, w1);
      d = (uint32_t)_mm_crc32_u64(d, w2);
    }
    c = gf2_times(g_shift_2stripe, a) ^ gf2_times(g_shift_stripe, b) ^ d;
    p += 3 * HW_STRIPE; n -= 3 * HW_STRIPE;
  }
  c = hw_run(c, p, n);
  return ~c;
}

static inline uint32_t compute_crc32_hw(const uint8_t* p, size_t n) {
  uint32_t c = oc_crc32c_hw(p, n);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

/* ------------------------------------------------------------------------------------------ */
/* varints: Go encoding/binary (go1.24) Uvarint / PutUvarint; utils.go:51-57 DecodeUvarint       */
/* ------------------------------------------------------------------------------------------ */
int oc_uvarint(const uint8_t* p, size_t n, uint64_t* v) {
  uint64_t x = 0;
  unsigned s = 0;
  for (size_t i = 0; i < n; ++i) {
    if (i == 10) { *v = 0; return -(int)(i + 1); }
    uint8_t b = p[i];
    if (b < 0x80) {
      if (i == 9 && b > 1) { *v = 0; return -(int)(i + 1); }
      *v = x | ((uint64_t)b << s);
      return (int)(i + 1);
    }
    x |= (uint64_t)(b & 0x7f) << s;
    s += 7;
  }
  *v = 0;
  return 0;
}

/* DecodeUvarint: every failure maps to (0, 0) */
static inline uint64_t decode_uvarint(const uint8_t* p, size_t n, size_t* used) {
  uint64_t v;
  int k = oc_uvarint(p, n, &v);
  if (k <= 0) { *used = 0; return 0; }
  *used = (size_t)k;
  return v;
}

int oc_put_uvarint(uint8_t* out, uint64_t v) {
  int i = 0;
  while (v >= 0x80) { out[i++] = (uint8_t)(v | 0x80); v >>= 7; }
  out[i++] = (uint8_t)v;
  return i;
}

static inline void put_u32(uint8_t* p, uint32_t v) { oc_memcpy(p, &v, 4); }
static inline void put_u64(uint8_t* p, uint64_t v) { oc_memcpy(p, &v, 8); }
static inline uint32_t get_u32(const uint8_t* p) { uint32_t v; oc_memcpy(&v, p, 4); return v; }
static inline uint64_t get_u64(const uint8_t* p) { uint64_t v; oc_memcpy(&v, p, 8); return v; }

/* ------------------------------------------------------------------------------------------ */
/* super block: wal.go:332-360 (write), wal.go:362-398 (load: crc -> magic -> blockSize)        */
/* ------------------------------------------------------------------------------------------ */
void oc_super_encode(uint8_t out[40], uint64_t create_time, uint64_t base_time) {
  memset(out, 0, 40);
  put_u64(out + 0, OC_MAGIC);
  put_u64(out + 8, OC_BLOCK_SIZE);
  put_u32(out + 16, OC_SUPER_SIZE);
  put_u64(out + 20, create_time);
  put_u64(out + 28, base_time);
  put_u32(out + 36, oc_compute_crc32(out, 36));
}

int oc_super_load(const uint8_t* p, size_t n, oc_super* o) {
  if (n < OC_SUPER_SIZE) return OC_SB_SHORT; /* ReadAt returns io.EOF */
  uint32_t crc = oc_compute_crc32(p, 36);
  if (crc != get_u32(p + 36)) return OC_SB_CRC;
  o->magic = get_u64(p);
  if (o->magic != OC_MAGIC) return OC_SB_MAGIC;
  o->block_size = get_u64(p + 8);
  o->start_off = get_u32(p + 16);
  if (o->block_size != OC_BLOCK_SIZE) return OC_SB_BLOCKSIZE;
  o->create_time = get_u64(p + 20);
  o->base_time = get_u64(p + 28);
  o->crc = crc;
  return OC_SB_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* writer: wal.go:482-553. The in-memory image holds the whole file (super block included), so  */
/* writeOffset(true) = len - 40 and writeOffset(false) = len.                                   */
/* ------------------------------------------------------------------------------------------ */
/* len: the logical file size; vbase: bytes before buf[0] that are only counted (a writer opened at a position far into
 * a large file, oc_writer_new_at: WriteRecord's layout depends on the position only through its phase in the block
 * grid, the returned offsets on the position itself) */
struct oc_writer { uint8_t* buf; uint64_t len, cap, vbase; };

static void w_append(oc_writer* w, const void* p, uint64_t n) {
  const uint64_t used = w->len - w->vbase;
  if (used + n > w->cap) {
    uint64_t nc = w->cap ? w->cap : 1u << 16;
    while (nc < used + n) nc *= 2;
    w->buf = (uint8_t*)realloc(w->buf, nc);
    w->cap = nc;
  }
  oc_memcpy(w->buf + used, p, n);
  w->len += n;
}

oc_writer* oc_writer_new(uint64_t create_time, uint64_t base_time) {
  oc_writer* w = (oc_writer*)calloc(1, sizeof *w);
  uint8_t sb[40];
  oc_super_encode(sb, create_time, base_time);
  w_append(w, sb, 40);
  return w;
}

/* a writer whose file already holds `size` bytes (>= 40: the super block and earlier records), none of them kept */
oc_writer* oc_writer_new_at(uint64_t size) {
  oc_writer* w = (oc_writer*)calloc(1, sizeof *w);
  w->len = w->vbase = size < OC_SUPER_SIZE ? OC_SUPER_SIZE : size;
  return w;
}

uint64_t oc_writer_write(oc_writer* w, const uint8_t* rec, size_t n) {
  static const uint8_t padding[6] = {0, 0, 0, 0, 0, 0};
  uint64_t offset = 0;
  int begin = 1;
  uint64_t left = n;
  while (left > 0) {
    uint64_t leftover = OC_BLOCK_SIZE - ((w->len - OC_SUPER_SIZE) % OC_BLOCK_SIZE);
    if (leftover < OC_HEADER_SIZE) {
      w_append(w, padding, leftover);
      leftover = OC_BLOCK_SIZE;
    }
    if (begin) offset = w->len;
    uint64_t avail = leftover - OC_HEADER_SIZE;
    uint64_t frag = left < avail ? left : avail;
    int end = (left == frag);
    uint8_t type = (begin && end) ? OC_FULL : begin ? OC_FIRST : end ? OC_LAST : OC_MIDDLE;
    uint8_t hdr[7];
    put_u32(hdr, oc_compute_crc32(rec, frag));
    uint16_t l16 = (uint16_t)frag;
    oc_memcpy(hdr + 4, &l16, 2);
    hdr[6] = type;
    w_append(w, hdr, 7);
    w_append(w, rec, frag);
    rec += frag;
    left -= frag;
    begin = 0;
  }
  return offset;
}

uint64_t oc_writer_size(const oc_writer* w) { return w->len; }
/* the materialized bytes: file offsets [oc_writer_base(w), oc_writer_size(w)) */
const uint8_t* oc_writer_data(const oc_writer* w) { return w->buf; }
uint64_t oc_writer_base(const oc_writer* w) { return w->vbase; }
void oc_writer_free(oc_writer* w) { if (w) { free(w->buf); free(w); } }

/* ------------------------------------------------------------------------------------------ */
/* Record.Encode: record.go:57-138                                                              */
/* ------------------------------------------------------------------------------------------ */
int64_t oc_record_encode(uint8_t* out, const uint8_t* ns, size_t ns_len, const uint8_t* key, size_t key_len,
                         const uint8_t* val, size_t val_len, const uint8_t* etag, size_t etag_len,
                         uint64_t expire, int tombstone, const uint8_t* meta, size_t meta_len,
                         uint64_t base_time) {
  uint8_t flag = 0;
  if (etag_len == 0) flag |= 1u << 0;
  if (tombstone) flag |= 1u << 2;
  uint8_t expb[10];
  int expire_size = 0;
  if (expire == 0) flag |= 1u << 1;
  else if (expire < base_time) return -1; /* "invalid expire" */
  /* binary.PutUvarint into `var expireBytes [binary.MaxVarintLen32]byte` (record.go:67,78): a delta that
   * needs more than 5 varint bytes (>= 2^35) indexes past the array and panics */
  else if (expire - base_time >= (1ull << 35)) return -2;
  else expire_size = oc_put_uvarint(expb, expire - base_time);
  uint8_t tmp[30];
  int t = 0;
  t += oc_put_uvarint(tmp + t, key_len);
  t += oc_put_uvarint(tmp + t, val_len);
  t += oc_put_uvarint(tmp + t, meta_len);
  size_t header = (size_t)t + expire_size + ns_len + etag_len + 2;
  size_t o = 0;
  out[o++] = (uint8_t)header; /* byte(headerSize): truncates above 255 (record.go:109) */
  oc_memcpy(out + o, ns, ns_len); o += ns_len;
  out[o++] = flag;
  oc_memcpy(out + o, tmp, t); o += t;
  oc_memcpy(out + o, etag, etag_len); o += etag_len;
  oc_memcpy(out + o, expb, expire_size); o += expire_size;
  oc_memcpy(out + o, key, key_len); o += key_len;
  oc_memcpy(out + o, val, val_len); o += val_len;
  oc_memcpy(out + o, meta, meta_len); o += meta_len;
  return (int64_t)o;
}

/* ------------------------------------------------------------------------------------------ */
/* RecordFromBytes: record.go:140-239, with Go slice-bound panics made explicit.                */
/* `cap` is cap(data): a Full record aliases the 32 KiB iterator buffer (wal_iterator.go:76,87). */
/* ------------------------------------------------------------------------------------------ */
void oc_record_parse(const uint8_t* data, size_t len, size_t cap, uint64_t base_time, uint32_t ns_size,
                     uint32_t etag_size, oc_rec* r) {
  (void)cap;
  r->hdr_size = 0; r->flags = 0; r->etag_off = 0;
  r->key_len = r->val_len = r->meta_len = 0; r->expire = 0;
  size_t min_hdr = 1 + (size_t)ns_size + 1 + 3;
  if (len < min_hdr) { r->status = OC_ST_INVALID; return; }
  size_t off = 0;
  uint64_t header = data[0];
  off++;
  off += ns_size;
  uint8_t flag = data[off];
  off++;
  size_t used;
  uint64_t key_len = decode_uvarint(data + off, len - off, &used); off += used;
  uint64_t val_len = decode_uvarint(data + off, len - off, &used); off += used;
  uint64_t meta_len = decode_uvarint(data + off, len - off, &used); off += used;
  uint64_t etag_len = (flag & 1u) ? 0 : etag_size;
  uint64_t expire_size = 0, expire = 0;
  r->hdr_size = (uint8_t)header; r->flags = flag; r->etag_off = (uint8_t)off;
  r->key_len = key_len; r->val_len = val_len; r->meta_len = meta_len;
  if ((flag & 2u) == 0) {
    /* data[offset+etagLen:] panics when offset+etagLen > len(data) (record.go:186) */
    if ((uint64_t)off + etag_len > (uint64_t)len) { r->status = OC_ST_PANIC; return; }
    size_t p = off + (size_t)etag_len;
    expire = decode_uvarint(data + p, len - p, &used);
    expire_size = used;
    expire += base_time; /* uint64 wraparound */
  }
  r->expire = expire;
  /* currentTotalSize := currentHeaderSize + int(keyLen+valLen+metaLen): int64 arithmetic */
  int64_t cur_hdr = (int64_t)off + (int64_t)etag_len + (int64_t)expire_size;
  int64_t cur_total = cur_hdr + (int64_t)(key_len + val_len + meta_len);
  if ((uint64_t)cur_hdr != header || cur_total != (int64_t)len) { r->status = OC_ST_INVALID; return; }
  /* slicing after validation (record.go:197-212): data[o : o+int(n)] panics when int(n) < 0 or when
   * the cumulative end passes cap(data); after a passed validation the latter happens exactly when
   * keyLen+valLen+metaLen wrapped around 2^64 (then one length is > 2^62, far beyond any cap). */
  {
    uint64_t s1 = key_len + val_len;
    int wrapped = s1 < key_len;
    uint64_t s2 = s1 + meta_len;
    wrapped |= s2 < s1;
    if ((int64_t)key_len < 0 || (int64_t)val_len < 0 || (int64_t)meta_len < 0 || wrapped) {
      r->status = OC_ST_PANIC;
      return;
    }
  }
  if (key_len > 0xffffffffull || val_len > 0xffffffffull || meta_len > 0xffffffffull || len > 0xffffffffull) {
    r->status = OC_ST_UNSUPPORTED;
    return;
  }
  /* meta > 0 would be msgpack.Unmarshal'ed (record.go:217-223): opaque here (parity unpinned) */
  r->status = OC_ST_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* hint codec: hint.go:32-48 (Encode), hint.go:50-84 (Decode)                                   */
/* ------------------------------------------------------------------------------------------ */
size_t oc_hint_encode(uint8_t* out, const uint8_t* ns, size_t ns_len, const uint8_t* key, size_t key_len,
                      uint64_t fid, uint64_t off, uint64_t size) {
  size_t o = 0;
  oc_memcpy(out, ns, ns_len); o += ns_len;
  o += oc_put_uvarint(out + o, key_len);
  oc_memcpy(out + o, key, key_len); o += key_len;
  o += oc_put_uvarint(out + o, fid);
  o += oc_put_uvarint(out + o, off);
  o += oc_put_uvarint(out + o, size);
  return o;
}

void oc_hint_parse(const uint8_t* data, size_t len, uint32_t ns_size, oc_rec* r) {
  r->hdr_size = 0; r->flags = 0; r->etag_off = 0;
  r->key_len = r->val_len = r->meta_len = 0; r->expire = 0;
  size_t min_sz = (size_t)ns_size + 1 + 1 + 3;
  if (len < min_sz) { r->status = OC_ST_INVALID; return; }
  int64_t off = ns_size;
  size_t used;
  uint64_t key_len = decode_uvarint(data + off, len - (size_t)off, &used);
  off += (int64_t)used;
  int64_t key_off = off;
  off = (int64_t)((uint64_t)off + key_len); /* offset += int(keyLen): Go int64 wraparound */
  r->key_len = key_len;
  r->hdr_size = (uint8_t)key_off;
  if (off < 0 || off > (int64_t)len) { r->status = OC_ST_PANIC; return; } /* data[offset:] */
  uint64_t fid = decode_uvarint(data + off, len - (size_t)off, &used); off += (int64_t)used;
  uint64_t hoff = decode_uvarint(data + off, len - (size_t)off, &used); off += (int64_t)used;
  uint64_t hsize = decode_uvarint(data + off, len - (size_t)off, &used); off += (int64_t)used;
  r->expire = fid; r->val_len = hoff; r->meta_len = hsize;
  if (off != (int64_t)len) { r->status = OC_ST_INVALID; return; }
  /* r.key = data[keyOffset : keyOffset+int(keyLen)] -- panics when int(keyLen) < 0 */
  if ((int64_t)key_len < 0) { r->status = OC_ST_PANIC; return; }
  r->status = OC_ST_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* segment iteration: wal_iterator.go:40-100 (Next) driven as record.go:242-266 / hint.go:163  */
/* ------------------------------------------------------------------------------------------ */
struct oc_decode {
  oc_frag* frags; uint64_t n_frags, cap_frags;
  oc_rec* recs; uint64_t n_recs, cap_recs;
  uint8_t* bytes; uint64_t n_bytes, cap_bytes;
  uint64_t* byte_offs;
  uint64_t err_frag;
  int32_t err_class;
};

static void push_frag(oc_decode* d, const oc_frag* f) {
  if (d->n_frags == d->cap_frags) {
    d->cap_frags = d->cap_frags ? d->cap_frags * 2 : 1024;
    d->frags = (oc_frag*)realloc(d->frags, d->cap_frags * sizeof(oc_frag));
  }
  d->frags[d->n_frags++] = *f;
}

static void push_rec(oc_decode* d, const oc_rec* r, const uint8_t* bytes, uint64_t n) {
  if (d->n_recs == d->cap_recs) {
    d->cap_recs = d->cap_recs ? d->cap_recs * 2 : 1024;
    d->recs = (oc_rec*)realloc(d->recs, d->cap_recs * sizeof(oc_rec));
    d->byte_offs = (uint64_t*)realloc(d->byte_offs, (d->cap_recs + 1) * sizeof(uint64_t));
  }
  if (d->n_bytes + n > d->cap_bytes) {
    uint64_t nc = d->cap_bytes ? d->cap_bytes : 1u << 16;
    while (nc < d->n_bytes + n) nc *= 2;
    d->bytes = (uint8_t*)realloc(d->bytes, nc);
    d->cap_bytes = nc;
  }
  d->byte_offs[d->n_recs] = d->n_bytes;
  oc_memcpy(d->bytes + d->n_bytes, bytes, n);
  d->n_bytes += n;
  d->recs[d->n_recs++] = *r;
  d->byte_offs[d->n_recs] = d->n_bytes;
}

oc_decode* oc_decode_segment(const uint8_t* seg, uint64_t len, uint32_t start_off, uint64_t base_time,
                             uint32_t ns_size, uint32_t etag_size, int mode) {
  oc_decode* d = (oc_decode*)calloc(1, sizeof *d);
  d->err_frag = UINT64_MAX;
  d->err_class = OC_ERR_NONE;
  d->byte_offs = (uint64_t*)calloc(1, sizeof(uint64_t));
  /* NewWalIterator: fileOff = wal.offset (super.startOff), bufOff = bufSize = 0 */
  int64_t file_off = start_off;
  int64_t buf_off = 0, buf_size = 0;
  /* the Next() loop state carried across calls: record (acc) and off */
  uint8_t* acc = NULL; uint64_t acc_len = 0, acc_cap = 0;
  uint64_t off = 0;
  uint32_t rec_first = 0; /* first fragment index contributing bytes to acc */
  for (;;) {
    if (buf_off + (int64_t)OC_HEADER_SIZE > buf_size) {
      file_off += buf_size;
      int64_t rem = (int64_t)len - file_off;
      buf_size = rem < (int64_t)OC_BLOCK_SIZE ? rem : (int64_t)OC_BLOCK_SIZE;
      if (buf_size == 0) break; /* ErrWalIteratorEOF; a pending partial record is dropped */
      if (buf_size < 0) { d->err_class = OC_ERR_PANIC; d->err_frag = d->n_frags; break; } /* i.buf[:neg] */
      buf_off = 0;
      /* wal_iterator.go:62-76: after a refill the header is sliced without re-checking bufSize
       * (cap(i.buf) is 32 KiB, so buf[0:7] is legal), then length = min(len, bufSize-7) < 0 and
       * i.buf[7:7+length] panics: a last block of 1..6 bytes always panics. */
      if (buf_size < (int64_t)OC_HEADER_SIZE) { d->err_class = OC_ERR_PANIC; d->err_frag = d->n_frags; break; }
    }
    const uint8_t* buf = seg + file_off;
    const uint8_t* header = buf + buf_off;
    buf_off += OC_HEADER_SIZE;
    uint32_t crc = get_u32(header);
    uint16_t l16; oc_memcpy(&l16, header + 4, 2);
    int64_t length = l16;
    uint8_t type = header[6];
    if (acc_len == 0) { off = (uint64_t)(file_off + buf_off); rec_first = (uint32_t)d->n_frags; }
    if (length > buf_size - buf_off) length = buf_size - buf_off; /* wal_iterator.go:75 */
    const uint8_t* data = buf + buf_off;
    buf_off += length;
    oc_frag f;
    memset(&f, 0, sizeof f);
    f.data_off = (uint64_t)(file_off + (buf_off - length));
    f.len = (uint32_t)length;
    f.stored_crc = crc;
    f.type = type;
    f.crc_ok = oc_compute_crc32(data, (size_t)length) == crc;
    uint32_t fidx = (uint32_t)d->n_frags;
    push_frag(d, &f);
    if (!f.crc_ok) { d->err_class = OC_ERR_CRC; d->err_frag = fidx; break; }
    const uint8_t* rec_bytes = NULL;
    uint64_t rec_len = 0, rec_cap = 0;
    uint32_t first = rec_first;
    if (type == OC_FULL) {
      rec_bytes = data; rec_len = (uint64_t)length;
      rec_cap = (uint64_t)(buf_size - (buf_off - length)); /* cap of i.buf[bufOff:...] */
      first = fidx;
    } else if (type == OC_FIRST || type == OC_MIDDLE || type == OC_LAST) {
      if (acc_len + (uint64_t)length > acc_cap) {
        acc_cap = (acc_len + (uint64_t)length) * 2 + 64;
        acc = (uint8_t*)realloc(acc, acc_cap);
      }
      oc_memcpy(acc + acc_len, data, (size_t)length);
      acc_len += (uint64_t)length;
      if (type != OC_LAST) continue;
      rec_bytes = acc; rec_len = acc_len; rec_cap = acc_len;
    } else {
      d->err_class = OC_ERR_TYPE; d->err_frag = fidx; break;
    }
    oc_rec r;
    memset(&r, 0, sizeof r);
    r.foff = off;
    r.size = rec_len;
    r.first_frag = first;
    r.emit_frag = fidx;
    if (mode == 0) oc_record_parse(rec_bytes, (size_t)rec_len, (size_t)rec_cap, base_time, ns_size, etag_size, &r);
    else oc_hint_parse(rec_bytes, (size_t)rec_len, ns_size, &r);
    push_rec(d, &r, rec_bytes, rec_len);
    acc_len = 0; /* Next() returns: the next call starts with record == nil */
  }
  free(acc);
  return d;
}

void oc_decode_counts(const oc_decode* d, uint64_t* n_frags, uint64_t* n_recs, uint64_t* err_frag,
                      int32_t* err_class, uint64_t* rec_bytes) {
  *n_frags = d->n_frags; *n_recs = d->n_recs; *err_frag = d->err_frag; *err_class = d->err_class;
  *rec_bytes = d->n_bytes;
}
void oc_decode_frags(const oc_decode* d, oc_frag* dst) { oc_memcpy(dst, d->frags, d->n_frags * sizeof(oc_frag)); }
void oc_decode_recs(const oc_decode* d, oc_rec* dst) { oc_memcpy(dst, d->recs, d->n_recs * sizeof(oc_rec)); }
void oc_decode_bytes(const oc_decode* d, uint8_t* dst, uint64_t* offs) {
  oc_memcpy(dst, d->bytes, d->n_bytes);
  oc_memcpy(offs, d->byte_offs, (d->n_recs + 1) * sizeof(uint64_t));
}
void oc_decode_free(oc_decode* d) {
  if (!d) return;
  free(d->frags); free(d->recs); free(d->bytes); free(d->byte_offs); free(d);
}

/* ------------------------------------------------------------------------------------------ */
/* CPU baseline: the same Next() + RecordFromBytes loop with hardware CRC and no per-record      */
/* allocation (an upper bound on the Go path's speed).                             */
/* ------------------------------------------------------------------------------------------ */
static uint64_t decode_fast_impl(const uint8_t* seg, int fd, uint64_t len, uint32_t start_off, uint64_t base_time,
                                 uint32_t ns_size, uint32_t etag_size, int32_t* err_class, uint64_t* checksum) {
  int64_t file_off = start_off, buf_off = 0, buf_size = 0;
  uint64_t acc_len = 0, off = 0, n = 0, sum = 0;
  static __thread uint8_t* acc = NULL;
  static __thread uint64_t acc_cap = 0;
  uint8_t blk[OC_BLOCK_SIZE]; /* pread target: one 32 KiB block at a time (wal_iterator.go:55) */
  *err_class = OC_ERR_NONE;
  for (;;) {
    if (buf_off + (int64_t)OC_HEADER_SIZE > buf_size) {
      file_off += buf_size;
      int64_t rem = (int64_t)len - file_off;
      buf_size = rem < (int64_t)OC_BLOCK_SIZE ? rem : (int64_t)OC_BLOCK_SIZE;
      if (buf_size <= 0) { if (buf_size < 0) *err_class = OC_ERR_PANIC; break; }
      if (buf_size < (int64_t)OC_HEADER_SIZE) { *err_class = OC_ERR_PANIC; break; }
      if (seg) {
        oc_memcpy(blk, seg + file_off, (size_t)buf_size);
      } else { /* PreadFull (utils.go:32-48) */
        int64_t got = 0;
        while (got < buf_size) {
          ssize_t r = pread(fd, blk + got, (size_t)(buf_size - got), (off_t)(file_off + got));
          if (r <= 0) { *err_class = OC_ERR_PANIC; return n; }
          got += r;
        }
      }
      buf_off = 0;
    }
    const uint8_t* header = blk + buf_off;
    buf_off += OC_HEADER_SIZE;
    uint32_t crc = get_u32(header);
    uint16_t l16; oc_memcpy(&l16, header + 4, 2);
    int64_t length = l16;
    uint8_t type = header[6];
    if (acc_len == 0) off = (uint64_t)(file_off + buf_off);
    if (length > buf_size - buf_off) length = buf_size - buf_off;
    const uint8_t* data = blk + buf_off;
    buf_off += length;
    if (compute_crc32_hw(data, (size_t)length) != crc) { *err_class = OC_ERR_CRC; break; }
    const uint8_t* rb;
    uint64_t rl;
    if (type == OC_FULL) { rb = data; rl = (uint64_t)length; }
    else if (type >= OC_FIRST && type <= OC_LAST) {
      if (acc_len + (uint64_t)length > acc_cap) { acc_cap = (acc_len + length) * 2 + 64; acc = (uint8_t*)realloc(acc, acc_cap); }
      oc_memcpy(acc + acc_len, data, (size_t)length);
      acc_len += (uint64_t)length;
      if (type != OC_LAST) continue;
      rb = acc; rl = acc_len;
    } else { *err_class = OC_ERR_TYPE; break; }
    oc_rec r;
    oc_record_parse(rb, (size_t)rl, (size_t)rl, base_time, ns_size, etag_size, &r);
    acc_len = 0;
    if (r.status != OC_ST_OK) break; /* IterateRecord returns the parse error */
    sum += off + rl + r.key_len;
    ++n;
  }
  *checksum = sum;
  return n;
}

uint64_t oc_decode_fast(const uint8_t* seg, uint64_t len, uint32_t start_off, uint64_t base_time,
                        uint32_t ns_size, uint32_t etag_size, int32_t* err_class, uint64_t* checksum) {
  return decode_fast_impl(seg, -1, len, start_off, base_time, ns_size, etag_size, err_class, checksum);
}

uint64_t oc_decode_fast_pread(int fd, uint64_t len, uint32_t start_off, uint64_t base_time, uint32_t ns_size,
                              uint32_t etag_size, int32_t* err_class, uint64_t* checksum) {
  return decode_fast_impl(NULL, fd, len, start_off, base_time, ns_size, etag_size, err_class, checksum);
}

/* ------------------------------------------------------------------------------------------ */
/* compaction (compaction.go:294-327) and hint rebuild (hint.go:123-161)                        */
/* ------------------------------------------------------------------------------------------ */
/* Record.Meta.AppMetaSize == 0 after msgpack.Unmarshal(meta, &map[string]string) (record.go:213-220,
 * meta.go:38-49): Record.Encode then writes no meta (record.go:82). Recognised for the canonical msgpack
 * forms of an empty map: nil (0xc0), {} (0x80) and fixmaps whose keys and values are all empty
 * strings (0xa0) or nil. Any other meta is copied verbatim (msgpack re-encoding parity unpinned). */
int oc_meta_app_size_zero(const uint8_t* m, size_t n) {
  if (n == 1) return m[0] == 0xc0 || m[0] == 0x80;
  if (n < 3 || (m[0] & 0xf0) != 0x80) return 0;
  size_t e = m[0] & 0x0f;
  if (n != 1 + 2 * e) return 0;
  for (size_t i = 1; i < n; ++i)
    if (m[i] != 0xa0 && m[i] != 0xc0) return 0;
  return 1;
}

/* compactOneWal (compaction.go:294-327) over one source WAL: IterateRecord delivers records until the
 * first bad row or fragment error; every kept record is re-encoded (Record.Encode against the dst
 * baseTime) and appended to dst (WriteRecord), then its hint (ns, key, dst fid, dst offset, payload
 * size) is appended to `hint`. The callback's first error stops the iteration. */
void oc_compact_append(oc_writer* dst, oc_writer* hint, uint64_t dst_fid, const uint8_t* seg, uint64_t len,
                       uint32_t start_off, uint64_t src_base, uint64_t dst_base, uint32_t ns_size,
                       uint32_t etag_size, const uint8_t* keep, uint64_t n_keep, uint64_t* offs,
                       int32_t* err_class, int64_t* err_rec, uint64_t* n_in) {
  oc_decode* d = oc_decode_segment(seg, len, start_off, src_base, ns_size, etag_size, 0);
  uint8_t* buf = NULL;
  size_t buf_cap = 0;
  *err_class = OC_ENC_OK;
  *err_rec = -1;
  uint64_t i = 0;
  for (; i < d->n_recs; ++i) {
    const oc_rec* r = &d->recs[i];
    if (r->status != OC_ST_OK) { *err_class = OC_ENC_SRC; *err_rec = (int64_t)i; break; } /* RecordFromBytes error */
    if (offs) offs[i] = UINT64_MAX;
    if (i >= n_keep || !keep[i]) continue; /* doFilter dropped it */
    const uint8_t* p = d->bytes + d->byte_offs[i];
    const uint8_t* ns = p + 1;
    size_t etag_len = (r->flags & 1u) ? 0 : etag_size;
    const uint8_t* etag = p + r->etag_off;
    const uint8_t* key = p + r->hdr_size;
    const uint8_t* val = key + r->key_len;
    const uint8_t* meta = val + r->val_len;
    size_t meta_len = oc_meta_app_size_zero(meta, r->meta_len) ? 0 : r->meta_len;
    size_t need = 64 + ns_size + etag_len + r->key_len + r->val_len + meta_len;
    if (need > buf_cap) { buf_cap = need * 2; buf = (uint8_t*)realloc(buf, buf_cap); }
    int64_t n = oc_record_encode(buf, ns, ns_size, key, r->key_len, val, r->val_len, etag, etag_len, r->expire,
                                 (r->flags >> 2) & 1u, meta, meta_len, dst_base);
    if (n < 0) { *err_class = n == -1 ? OC_ENC_EXPIRE : OC_ENC_PANIC; *err_rec = (int64_t)i; break; }
    uint64_t o = oc_writer_write(dst, buf, (size_t)n);
    if (offs) offs[i] = o;
    size_t hneed = ns_size + r->key_len + 40;
    uint8_t* hp = (uint8_t*)malloc(hneed);
    size_t hn = oc_hint_encode(hp, ns, ns_size, key, r->key_len, dst_fid, o, (uint64_t)n);
    oc_writer_write(hint, hp, hn);
    free(hp);
  }
  if (*err_class == OC_ENC_OK && d->err_class != OC_ERR_NONE) *err_class = OC_ENC_SRC; /* iterator error */
  *n_in = i;
  free(buf);
  oc_decode_free(d);
}

/* NewHintByWal (hint.go:123-161): one hint per delivered record, off = foff - 7 (the iterator offset,
 * so a zero-length First shifts it), size = len(payload). */
void oc_hint_by_wal(oc_writer* hint, uint64_t fid, const uint8_t* seg, uint64_t len, uint32_t start_off,
                    uint64_t base_time, uint32_t ns_size, uint32_t etag_size, int32_t* err_class, int64_t* err_rec,
                    uint64_t* n_in) {
  oc_decode* d = oc_decode_segment(seg, len, start_off, base_time, ns_size, etag_size, 0);
  *err_class = OC_ENC_OK;
  *err_rec = -1;
  uint64_t i = 0;
  for (; i < d->n_recs; ++i) {
    const oc_rec* r = &d->recs[i];
    if (r->status != OC_ST_OK) { *err_class = OC_ENC_SRC; *err_rec = (int64_t)i; break; }
    const uint8_t* p = d->bytes + d->byte_offs[i];
    size_t hneed = ns_size + r->key_len + 40;
    uint8_t* hb = (uint8_t*)malloc(hneed);
    size_t hn = oc_hint_encode(hb, p + 1, ns_size, p + r->hdr_size, r->key_len, fid, r->foff - OC_HEADER_SIZE, r->size);
    oc_writer_write(hint, hb, hn);
    free(hb);
  }
  if (*err_class == OC_ENC_OK && d->err_class != OC_ERR_NONE) *err_class = OC_ENC_SRC;
  *n_in = i;
  oc_decode_free(d);
}

/* ------------------------------------------------------------------------------------------ */
/* synthetic segments: splitmix64 stream; ns = 'A'+i%26; key = index(8 B LE) +    */
/* PRNG bytes; value = PRNG bytes; no etag / expire / meta; createTime = baseTime.              */
/* ------------------------------------------------------------------------------------------ */
static inline uint64_t splitmix64(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static void fill_rand(uint64_t* s, uint8_t* p, size_t n) {
  size_t i = 0;
  for (; i + 8 <= n; i += 8) { uint64_t v = splitmix64(s); oc_memcpy(p + i, &v, 8); }
  if (i < n) { uint64_t v = splitmix64(s); oc_memcpy(p + i, &v, n - i); }
}

oc_writer* oc_synth_segment(uint64_t target_bytes, uint64_t max_records, uint64_t seed, uint32_t ns_size,
                            uint32_t key_len, uint32_t value_len, int value_mode, uint64_t base_time) {
  oc_writer* w = oc_writer_new(base_time, base_time);
  uint64_t s = seed;
  double cdf[512];
  if (value_mode == 1) {
    double acc = 0;
    for (int k = 1; k <= 512; ++k) { acc += pow((double)k, -1.1); cdf[k - 1] = acc; }
    for (int k = 0; k < 512; ++k) cdf[k] /= acc;
  }
  uint8_t* ns = (uint8_t*)malloc(ns_size + 1);
  for (uint32_t i = 0; i < ns_size; ++i) ns[i] = (uint8_t)('A' + i % 26);
  size_t vmax = value_mode == 1 ? 128 * 512 : value_mode == 2 ? 1400 : value_len;
  uint8_t etag[20];
  uint8_t* key = (uint8_t*)malloc(key_len + 8);
  uint8_t* val = (uint8_t*)malloc(vmax + 8);
  uint8_t* rec = (uint8_t*)malloc(vmax + key_len + ns_size + 64);
  for (uint64_t i = 0; (max_records == 0 || i < max_records) && w->len < target_bytes; ++i) {
    size_t vl = value_len;
    if (value_mode == 1) {
      double u = (double)(splitmix64(&s) >> 11) * (1.0 / 9007199254740992.0);
      int lo = 0, hi = 511;
      while (lo < hi) { int mid = (lo + hi) / 2; if (cdf[mid] < u) lo = mid + 1; else hi = mid; }
      vl = 128u * (size_t)(lo + 1);
    }
    if (value_mode == 2) {
      /* value_mode 2 (compaction tests): 200-1399 B values, every record with an expire (baseTime + 1 h + up to
       * ~2 days), a 20 B etag on every third, a tombstone on every 17th */
      vl = 200 + (size_t)(splitmix64(&s) % 1200);
      fill_rand(&s, key, key_len);
      if (key_len >= 8) oc_memcpy(key, &i, 8);
      fill_rand(&s, val, vl);
      fill_rand(&s, etag, sizeof etag);
      const uint64_t expire = base_time + 3600 + splitmix64(&s) % 170000;
      int64_t n = oc_record_encode(rec, ns, ns_size, key, key_len, val, vl, i % 3 == 0 ? etag : NULL,
                                   i % 3 == 0 ? sizeof etag : 0, expire, i % 17 == 0, NULL, 0, base_time);
      oc_writer_write(w, rec, (size_t)n);
      continue;
    }
    fill_rand(&s, key, key_len);
    if (key_len >= 8) oc_memcpy(key, &i, 8);
    fill_rand(&s, val, vl);
    int64_t n = oc_record_encode(rec, ns, ns_size, key, key_len, val, vl, NULL, 0, 0, 0, NULL, 0, base_time);
    oc_writer_write(w, rec, (size_t)n);
  }
  free(ns); free(key); free(val); free(rec);
  return w;
}

/* ------------------------------------------------------------------------------------------ */
/* framing size maths: wal.go:61-97                                                            */
/* ------------------------------------------------------------------------------------------ */
uint64_t oc_wal_record_size(uint64_t offset, uint64_t size) {
  /* WalRecordSize (wal.go:61-86): uint64 arithmetic, `offset -= SuperBlockSize` wraps below 40 */
  uint64_t left = size, phy = 0;
  offset -= OC_SUPER_SIZE;
  while (left > 0) {
    uint64_t leftover = OC_BLOCK_SIZE - (offset % OC_BLOCK_SIZE);
    if (leftover < OC_HEADER_SIZE) {
      phy += leftover;
      offset += leftover;
      leftover = OC_BLOCK_SIZE;
    }
    uint64_t avail = leftover - OC_HEADER_SIZE;
    uint64_t frag = left < avail ? left : avail;
    phy += OC_HEADER_SIZE + frag;
    offset += OC_HEADER_SIZE + frag;
    left -= frag;
  }
  return phy;
}

void oc_wal_block_index_range(uint64_t offset, uint64_t size, uint64_t* first_idx, uint64_t* first_off,
                              uint64_t* blk_num) {
  /* WalBlockIndexRange (wal.go:88-97) */
  uint64_t rs = oc_wal_record_size(offset, size);
  *first_idx = (offset - OC_SUPER_SIZE) / OC_BLOCK_SIZE;
  *first_off = *first_idx * OC_BLOCK_SIZE + OC_SUPER_SIZE;
  uint64_t last = (offset - OC_SUPER_SIZE + rs) / OC_BLOCK_SIZE;
  *blk_num = last - *first_idx + 1;
}

/* ------------------------------------------------------------------------------------------ */
/* payload hashes for full-size parity checks (test infrastructure)                            */
/* ------------------------------------------------------------------------------------------ */
static uint64_t oc_hash_bytes(uint64_t h, const uint8_t* p, uint64_t n) {
  /* 64-bit multiply-rotate over 8-byte words; the length is mixed in by the caller */
  uint64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    oc_memcpy(&w, p + i, 8);
    h = (h ^ w) * 0x9E3779B97F4A7C15ull;
    h = (h << 27) | (h >> 37);
  }
  if (i < n) {
    uint64_t w = 0;
    oc_memcpy(&w, p + i, (size_t)(n - i));
    h = (h ^ w ^ ((n - i) << 56)) * 0xC2B2AE3D27D4EB4Full;
    h = (h << 31) | (h >> 33);
  }
  return h;
}

/* hash of every record payload of an oracle decode */
void oc_decode_payload_hashes(const oc_decode* d, uint64_t* out) {
  for (uint64_t r = 0; r < d->n_recs; ++r) {
    uint64_t n = d->byte_offs[r + 1] - d->byte_offs[r];
    out[r] = oc_hash_bytes(0x5EEDull ^ n, d->bytes + d->byte_offs[r], n);
  }
}

/* the same hash over payloads gathered from a (device-produced) fragment table: record r's bytes are
 * the data of fragments [first[r], emit[r]] (data_off / flen per fragment); the words are streamed
 * across fragment boundaries exactly as over the concatenation */
void oc_gather_payload_hashes(const uint8_t* seg, uint64_t seg_len, const uint64_t* data_off, const uint32_t* flen,
                              uint64_t n_frags, const uint32_t* first, const uint32_t* emit, const uint64_t* size,
                              uint64_t n_recs, uint64_t* out) {
  uint8_t* tmp = NULL;
  uint64_t cap = 0;
  for (uint64_t r = 0; r < n_recs; ++r) {
    uint64_t f0 = first[r], f1 = emit[r];
    if (f1 >= n_frags || f0 > f1) { out[r] = 0; continue; }
    if (f0 == f1) {
      uint64_t o = data_off[f0], n = flen[f0];
      out[r] = (o + n <= seg_len) ? oc_hash_bytes(0x5EEDull ^ n, seg + o, n) : 0;
      continue;
    }
    uint64_t n = size[r];
    if (n > cap) { cap = n * 2 + 64; tmp = (uint8_t*)realloc(tmp, cap); }
    uint64_t w = 0;
    for (uint64_t g = f0; g <= f1 && w <= n; ++g) {
      uint64_t o = data_off[g], l = flen[g];
      if (o + l > seg_len || w + l > n) { w = n + 1; break; }
      oc_memcpy(tmp + w, seg + o, l);
      w += l;
    }
    out[r] = (w == n) ? oc_hash_bytes(0x5EEDull ^ n, tmp, n) : 0;
  }
  free(tmp);
}

/* ------------------------------------------------------------------------------------------ */
/* index: IndexOperator.Hash (index.go:15-19) = murmur3.New64().Write(key).Sum64() of          */
/* github.com/spaolacci/murmur3 v1.1.0 (go.mod:10; not vendored): MurmurHash3_x64_128 with     */
/* seed 0, Sum64 = h1 (Austin Appleby's published algorithm, restated here)                    */
/* ------------------------------------------------------------------------------------------ */
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

void oc_murmur3_128(const uint8_t* p, size_t n, uint64_t seed, uint64_t* o1, uint64_t* o2) {
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  uint64_t h1 = seed, h2 = seed;
  size_t nb = n / 16;
  for (size_t i = 0; i < nb; ++i) {
    uint64_t k1 = get_u64(p + 16 * i), k2 = get_u64(p + 16 * i + 8);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
  }
  const uint8_t* t = p + 16 * nb;
  uint64_t k1 = 0, k2 = 0;
  switch (n & 15) {
    case 15: k2 ^= (uint64_t)t[14] << 48; /* fallthrough */
    case 14: k2 ^= (uint64_t)t[13] << 40; /* fallthrough */
    case 13: k2 ^= (uint64_t)t[12] << 32; /* fallthrough */
    case 12: k2 ^= (uint64_t)t[11] << 24; /* fallthrough */
    case 11: k2 ^= (uint64_t)t[10] << 16; /* fallthrough */
    case 10: k2 ^= (uint64_t)t[9] << 8;   /* fallthrough */
    case 9:  k2 ^= (uint64_t)t[8];
             k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2; /* fallthrough */
    case 8:  k1 ^= (uint64_t)t[7] << 56;  /* fallthrough */
    case 7:  k1 ^= (uint64_t)t[6] << 48;  /* fallthrough */
    case 6:  k1 ^= (uint64_t)t[5] << 40;  /* fallthrough */
    case 5:  k1 ^= (uint64_t)t[4] << 32;  /* fallthrough */
    case 4:  k1 ^= (uint64_t)t[3] << 24;  /* fallthrough */
    case 3:  k1 ^= (uint64_t)t[2] << 16;  /* fallthrough */
    case 2:  k1 ^= (uint64_t)t[1] << 8;   /* fallthrough */
    case 1:  k1 ^= (uint64_t)t[0];
             k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
  }
  h1 ^= (uint64_t)n; h2 ^= (uint64_t)n;
  h1 += h2; h2 += h1;
  h1 = fmix64(h1); h2 = fmix64(h2);
  h1 += h2; h2 += h1;
  *o1 = h1; *o2 = h2;
}

uint64_t oc_murmur3_sum64(const uint8_t* p, size_t n) {
  uint64_t h1, h2;
  oc_murmur3_128(p, n, 0, &h1, &h2);
  return h1;
}

/* The index's observable semantics (index.go:81-165 over map.go's ShardMap): a map from
 * MergedKey(ns, key) = ns || key (utils.go:133-139) to IndexValue{fid, valueOff, valueSize}.
 *   Put        -> Set (insert or replace)                       index.go:144-165, map.go:160-207
 *   Delete     -> remove                                        index.go:107-124
 *   SoftDelete -> Set(IndexValue{valueOff: 0}) (fid 0, size 0)   index.go:126-142
 *   Get        -> value, ErrKeyNotFound, or ErrKeySoftDeleted when valueOff == 0  index.go:81-98
 * Bucket placement (hash % 16 shards, hash % (cap/16) chains) is unobservable; the sampled
 * approximate-LRU eviction (map.go:395-420, random slots) is not restated: this oracle and the
 * device index hold every key (the reference's deterministic regime: capacity >= keys). */
typedef struct oc_islot { uint8_t* key; uint32_t klen, live; uint64_t h, fid, off, size; } oc_islot;
struct oc_index { oc_islot* s; uint64_t cap, used, live; };

oc_index* oc_index_new(void) {
  oc_index* x = (oc_index*)calloc(1, sizeof *x);
  x->cap = 1024;
  x->s = (oc_islot*)calloc(x->cap, sizeof(oc_islot));
  return x;
}
void oc_index_free(oc_index* x) {
  if (!x) return;
  for (uint64_t i = 0; i < x->cap; ++i) free(x->s[i].key);
  free(x->s);
  free(x);
}
static oc_islot* oc_index_find(oc_index* x, const uint8_t* k, uint32_t kl, uint64_t h, int create) {
  if (create && (x->used + 1) * 2 > x->cap) {
    oc_islot* old = x->s;
    uint64_t oc = x->cap;
    x->cap *= 2;
    x->s = (oc_islot*)calloc(x->cap, sizeof(oc_islot));
    for (uint64_t i = 0; i < oc; ++i) {
      if (!old[i].key) continue;
      uint64_t j = old[i].h & (x->cap - 1);
      while (x->s[j].key) j = (j + 1) & (x->cap - 1);
      x->s[j] = old[i];
    }
    free(old);
  }
  uint64_t j = h & (x->cap - 1);
  for (;;) {
    oc_islot* e = &x->s[j];
    if (!e->key) {
      if (!create) return NULL;
      e->key = (uint8_t*)malloc(kl ? kl : 1);
      oc_memcpy(e->key, k, kl);
      e->klen = kl;
      e->h = h;
      e->live = 0;
      x->used++;
      return e;
    }
    if (e->h == h && e->klen == kl && memcmp(e->key, k, kl) == 0) return e;
    j = (j + 1) & (x->cap - 1);
  }
}
static uint8_t* merged_key(const uint8_t* ns, size_t nsl, const uint8_t* key, size_t kl) {
  uint8_t* m = (uint8_t*)malloc(nsl + kl + 1);
  if (nsl) oc_memcpy(m, ns, nsl);
  if (kl) oc_memcpy(m + nsl, key, kl);
  return m;
}
void oc_index_set(oc_index* x, const uint8_t* ns, size_t nsl, const uint8_t* key, size_t kl, int op, uint64_t fid,
                  uint64_t off, uint64_t size) {
  /* op 0: Put, 1: Delete, 2: SoftDelete */
  uint8_t* m = merged_key(ns, nsl, key, kl);
  uint64_t h = oc_murmur3_sum64(m, nsl + kl);
  oc_islot* e = oc_index_find(x, m, (uint32_t)(nsl + kl), h, op != 1);
  free(m);
  if (!e) return;
  if (op == 1) {
    if (e->live) { e->live = 0; x->live--; }
    return;
  }
  if (!e->live) { e->live = 1; x->live++; }
  e->fid = op == 0 ? fid : 0;
  e->off = op == 0 ? off : 0;
  e->size = op == 0 ? size : 0;
}
int oc_index_get(oc_index* x, const uint8_t* ns, size_t nsl, const uint8_t* key, size_t kl, uint64_t* fid,
                 uint64_t* off, uint64_t* size) {
  uint8_t* m = merged_key(ns, nsl, key, kl);
  uint64_t h = oc_murmur3_sum64(m, nsl + kl);
  oc_islot* e = oc_index_find(x, m, (uint32_t)(nsl + kl), h, 0);
  free(m);
  if (!e || !e->live) return 1; /* ErrKeyNotFound */
  *fid = e->fid; *off = e->off; *size = e->size;
  return e->off == 0 ? 2 : 0;   /* ErrKeySoftDeleted */
}
uint64_t oc_index_live(const oc_index* x) { return x->live; }

/* doFilter (compaction.go:329-348) without the user CompactionFilter: 1 = drop */
int oc_do_filter(oc_index* x, const uint8_t* ns, size_t nsl, const uint8_t* key, size_t kl, uint64_t src_fid,
                 uint64_t src_off) {
  uint64_t fid = 0, off = 0, size = 0;
  if (oc_index_get(x, ns, nsl, key, kl, &fid, &off, &size) != 0) return 1;
  return (fid != src_fid || off != src_off) ? 1 : 0;
}

/* the record's ns and key spans inside its payload (RecordFromBytes record.go:140-239 / HintRecord.Decode
 * hint.go:50-84 layouts) */
static void rec_ns_key(const oc_rec* r, const uint8_t* payload, uint32_t ns_size, int mode, const uint8_t** ns,
                       const uint8_t** key, uint64_t* kl) {
  *ns = payload + (mode == 0 ? 1 : 0);
  *key = payload + r->hdr_size;
  if (mode == 1) { /* hint key offset NsSize + len(uvarint keyLen) (hint.go:62-66): hdr_size holds it mod 256 */
    size_t u = 1;
    while (u < 10 && (payload[ns_size + u - 1] & 0x80)) ++u;
    *key = payload + ns_size + u;
  }
  *kl = r->key_len;
}

/* the callback loops of recovery / compaction that feed the index, over the oracle decode:
 *   mode 0 (data WAL)  recoverFromWal    db_impl.go:305-313: Put(ns, key, fid, foff - 7, size)
 *   mode 1 (hint WAL)  recoverFromWal    db_impl.go:290-299: Put(ns, key, fid, h.off, h.size)
 *                      (use_rec_fid: onePhase compaction.go:248-251: Put(ns, key, h.fid, h.off, h.size))
 * Rows are put in order up to the first row the iteration rejects; returns the iteration's error
 * (OC_ERR_* of the fragment, or 16 + OC_ST_* of the failing row), *n_put = rows put. */
int oc_index_put_segment(oc_index* x, const uint8_t* seg, uint64_t len, uint32_t start_off, uint64_t base_time,
                         uint32_t ns_size, uint32_t etag_size, int mode, uint64_t fid, int use_rec_fid,
                         uint64_t* n_put) {
  oc_decode* d = oc_decode_segment(seg, len, start_off, base_time, ns_size, etag_size, mode);
  int ret = d->err_class;
  uint64_t r = 0;
  for (; r < d->n_recs; ++r) {
    const oc_rec* rc = &d->recs[r];
    if (rc->status != OC_ST_OK) { ret = 16 + rc->status; break; }
    const uint8_t *ns, *key;
    uint64_t kl;
    rec_ns_key(rc, d->bytes + d->byte_offs[r], ns_size, mode, &ns, &key, &kl);
    if (mode == 0) oc_index_set(x, ns, ns_size, key, kl, 0, fid, rc->foff - OC_HEADER_SIZE, rc->size);
    else oc_index_set(x, ns, ns_size, key, kl, 0, use_rec_fid ? rc->expire : fid, rc->val_len, rc->meta_len);
  }
  *n_put = r;
  oc_decode_free(d);
  return ret;
}

/* compactOneWal's doFilter over every delivered row (compaction.go:299-303): keep[r] = 1 when the index
 * still points at (src_fid, foff - 7); rows from the first rejected row on are 0. Returns rows visited. */
uint64_t oc_compact_filter(oc_index* x, const uint8_t* seg, uint64_t len, uint32_t start_off, uint64_t base_time,
                           uint32_t ns_size, uint32_t etag_size, uint64_t src_fid, uint8_t* keep, uint64_t n_keep) {
  oc_decode* d = oc_decode_segment(seg, len, start_off, base_time, ns_size, etag_size, 0);
  uint64_t r = 0;
  for (uint64_t i = 0; i < n_keep; ++i) keep[i] = 0;
  for (; r < d->n_recs; ++r) {
    const oc_rec* rc = &d->recs[r];
    if (rc->status != OC_ST_OK) break;
    const uint8_t *ns, *key;
    uint64_t kl;
    rec_ns_key(rc, d->bytes + d->byte_offs[r], ns_size, 0, &ns, &key, &kl);
    if (r < n_keep) keep[r] = oc_do_filter(x, ns, ns_size, key, kl, src_fid, rc->foff - OC_HEADER_SIZE) ? 0 : 1;
  }
  oc_decode_free(d);
  return r;
}

/* ------------------------------------------------------------------------------------------ */
/* point reads: Wal.ReadRecord (wal.go:556-573) = WalRecordSize + one PreadFull of the record's */
/* physical span + WalParseRecord (wal.go:121-173) over that single buffer                     */
/* ------------------------------------------------------------------------------------------ */
/* returns OC_RD_*; payload (size bytes) into out when OC_RD_OK */
int oc_read_record(const uint8_t* seg, uint64_t seg_len, uint64_t offset, uint64_t size, int verify, uint8_t* out) {
  uint64_t rs = oc_wal_record_size(offset, size);
  if (offset + rs > seg_len) return OC_RD_BEYOND;   /* "read beyond file size" (wal.go:562-564) */
  const uint8_t* buf = seg + offset;                /* buffer := make([]byte, recordSize); PreadFull */
  uint64_t blk_size = rs, blk_off = 0, got = 0;     /* WalParseRecord(size, 0, [][]byte{buffer}, ...) */
  for (;;) {
    if (blk_off + OC_HEADER_SIZE > blk_size) return OC_RD_PANIC; /* header := blks[i][blkOff:blkOff+7] */
    const uint8_t* h = buf + blk_off;
    blk_off += OC_HEADER_SIZE;
    uint32_t crc = get_u32(h);
    uint16_t l16;
    oc_memcpy(&l16, h + 4, 2);
    uint64_t length = l16;
    uint8_t type = h[6];
    if (length > blk_size - blk_off) return OC_RD_CORRUPTED;  /* ErrWalCorruptedData */
    const uint8_t* data = buf + blk_off;
    blk_off += length;
    if (verify && oc_compute_crc32(data, (size_t)length) != crc) return OC_RD_CRC;
    /* record = append(record, data...): the capacity is `size`, appending beyond it just grows */
    if (got + length <= size) oc_memcpy(out + got, data, (size_t)length);
    got += length;
    if (type == OC_FULL || type == OC_LAST) return got != size ? OC_RD_SIZE : OC_RD_OK;
    if (type != OC_FIRST && type != OC_MIDDLE) return OC_RD_TYPE;
    if (blk_size - blk_off <= OC_HEADER_SIZE) return OC_RD_INCOMPLETE; /* break; i++ ends the block loop */
  }
}

/* ------------------------------------------------------------------------------------------ */
/* bounded index: map.go's SimpleMap / ShardMap with the sampled approximate-LRU eviction        */
/* ------------------------------------------------------------------------------------------ */
/* Restated operation by operation (map.go:122-428) so that an index whose Limited is below its key count
 * (IndexCapacity / IndexLimited / IndexEvictionPoolCapacity, db.go:70-72 -> db_impl.go:164-166) has an
 * oracle: Set evicts before inserting once used + 1 > limited (map.go:185-187) and returns the evicted
 * value as "old" (so WriteStat reports it, index.go:152-162); the eviction samples SampleKeys entries of
 * random buckets (Rand(capacity), chains walked from the bucket head, map.go:349-371) into a pool kept in
 * ascending expire order with upper-bound insertion (map.go:294-316), then deletes the first pool entry
 * that still exists and drops [0, pos] from the pool while the size shrinks by pos only
 * (map.go:319-342 -- the last survivor stays duplicated, as in the reference). Rand and WallTime are
 * the injected MapOperatorBase (map.go:23-29): a scripted value list cycled like map_test.go's
 * mockSimpleMapOperator (v[i] % n), or a seeded splitmix64 stream; WallTime is a seconds counter the
 * caller advances (genExpire = seconds since the map's initTime, map.go:149-156). */
typedef struct oc_bkt {
  uint8_t* key; /* NULL: empty bucket head */
  uint32_t klen;
  uint32_t expire;
  uint64_t val[3];
  struct oc_bkt* next;
} oc_bkt;
typedef struct oc_pent { uint64_t slot; const uint8_t* key; uint32_t klen, expire; } oc_pent;
typedef struct oc_shard {
  uint64_t cap, used, limited, pool_size, pool_cap, sample;
  oc_bkt* b;
  oc_pent* pool;
  uint64_t init;
} oc_shard;
struct oc_smap {
  uint32_t nsh;
  int hash_mode;
  oc_shard* sh;
  uint64_t now;
  uint64_t* rv;
  uint64_t nrv, ri, seed;
  uint8_t** arena; /* pool key copies (the pool may hold stale duplicates: never freed before the map) */
  uint64_t narena, carena;
};

static uint64_t sm_rand(oc_smap* m, uint64_t n) {
  if (m->nrv) {
    if (m->ri >= m->nrv) m->ri = 0;
    return m->rv[m->ri++] % n;
  }
  uint64_t z = (m->seed += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (z ^ (z >> 31)) % n;
}
static uint64_t sm_hash(const oc_smap* m, const uint8_t* k, size_t kl) {
  if (m->hash_mode == 1) { uint64_t v = 0; oc_memcpy(&v, k, kl < 8 ? kl : 8); return v; }
  return oc_murmur3_sum64(k, kl);
}
static uint32_t sm_expire(const oc_smap* m, const oc_shard* s) {
  return m->now < s->init ? 0u : (uint32_t)(m->now - s->init);
}
static const uint8_t* sm_keep_key(oc_smap* m, const uint8_t* k, uint32_t kl) {
  if (m->narena == m->carena) {
    m->carena = m->carena ? 2 * m->carena : 1024;
    m->arena = (uint8_t**)realloc(m->arena, m->carena * sizeof *m->arena);
  }
  uint8_t* c = (uint8_t*)malloc(kl ? kl : 1);
  oc_memcpy(c, k, kl);
  m->arena[m->narena++] = c;
  return c;
}
static int sm_eq(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
  return al == bl && (al == 0 || memcmp(a, b, al) == 0);
}

oc_smap* oc_smap_new(uint32_t nshards, uint64_t capacity, uint64_t limited, uint64_t pool_cap, uint64_t sample_keys,
                     int hash_mode, const uint64_t* rand_vals, uint64_t n_rand, uint64_t seed) {
  if (nshards == 0) return NULL;
  /* NewShardMap divides Capacity and Limited (map.go:385-390); validate per map (map.go:102-120) */
  const uint64_t cap = capacity / nshards, lim = limited / nshards;
  if (lim > cap || pool_cap > lim || sample_keys < 1 || pool_cap < 16 || cap == 0) return NULL;
  oc_smap* m = (oc_smap*)calloc(1, sizeof *m);
  m->nsh = nshards;
  m->hash_mode = hash_mode;
  m->seed = seed;
  if (n_rand) {
    m->rv = (uint64_t*)malloc(n_rand * sizeof(uint64_t));
    oc_memcpy(m->rv, rand_vals, n_rand * sizeof(uint64_t));
    m->nrv = n_rand;
  }
  m->sh = (oc_shard*)calloc(nshards, sizeof(oc_shard));
  for (uint32_t i = 0; i < nshards; ++i) {
    oc_shard* s = &m->sh[i];
    s->cap = cap; s->limited = lim; s->pool_cap = pool_cap; s->sample = sample_keys;
    s->b = (oc_bkt*)calloc(cap, sizeof(oc_bkt));
    s->pool = (oc_pent*)calloc(pool_cap, sizeof(oc_pent));
    s->init = m->now;
  }
  return m;
}
void oc_smap_free(oc_smap* m) {
  if (!m) return;
  for (uint32_t i = 0; i < m->nsh; ++i) {
    oc_shard* s = &m->sh[i];
    for (uint64_t j = 0; j < s->cap; ++j) {
      oc_bkt* e = s->b[j].next;
      while (e) { oc_bkt* n = e->next; free(e->key); free(e); e = n; }
      free(s->b[j].key);
    }
    free(s->b);
    free(s->pool);
  }
  for (uint64_t i = 0; i < m->narena; ++i) free(m->arena[i]);
  free(m->arena);
  free(m->rv);
  free(m->sh);
  free(m);
}
void oc_smap_set_now(oc_smap* m, uint64_t seconds) { m->now = seconds; }
uint64_t oc_smap_size(const oc_smap* m) {
  uint64_t n = 0;
  for (uint32_t i = 0; i < m->nsh; ++i) n += m->sh[i].used;
  return n;
}

/* getEntryWithSlot (map.go:229-245) */
static oc_bkt* sm_find(oc_shard* s, const uint8_t* k, uint32_t kl, uint64_t slot) {
  slot %= s->cap;
  if (!s->b[slot].key) return NULL;
  for (oc_bkt* e = &s->b[slot]; e; e = e->next)
    if (sm_eq(k, kl, e->key, e->klen)) return e;
  return NULL;
}
/* deleteWithSlotInternal (map.go:260-292): 0 deleted (old value out), 1 ErrKeyNotFound */
static int sm_delete(oc_shard* s, const uint8_t* k, uint32_t kl, uint64_t slot, uint64_t old[3]) {
  slot %= s->cap;
  oc_bkt* h = &s->b[slot];
  if (!h->key) return 1;
  if (sm_eq(h->key, h->klen, k, kl)) {
    if (old) oc_memcpy(old, h->val, sizeof h->val);
    free(h->key);
    if (h->next) {
      oc_bkt* n = h->next;
      *h = *n; /* m.buckets[slot] = *m.buckets[slot].next */
      free(n);
    } else {
      h->key = NULL;
      h->klen = 0;
      memset(h->val, 0, sizeof h->val);
    }
    s->used--;
    return 0;
  }
  for (oc_bkt* e = h; e->next; e = e->next) {
    if (sm_eq(e->next->key, e->next->klen, k, kl)) {
      oc_bkt* d = e->next;
      if (old) oc_memcpy(old, d->val, sizeof d->val);
      e->next = d->next;
      free(d->key);
      free(d);
      s->used--;
      return 0;
    }
  }
  return 1;
}
/* insertEvictionEntry (map.go:294-316) */
static void sm_pool_insert(oc_shard* s, oc_pent en) {
  uint64_t idx = 0;
  while (idx < s->pool_size && !(en.expire < s->pool[idx].expire)) ++idx; /* sort.Search upper bound */
  if (idx == s->pool_size) {
    idx = s->pool_size - 1; /* size 0 only when pool_cap > 0: then the next line makes it 0 */
    if (s->pool_size != s->pool_cap) idx = s->pool_size;
  }
  if (s->pool_size != s->pool_cap) s->pool_size++;
  if (s->pool_size - 1 > idx) memmove(&s->pool[idx + 1], &s->pool[idx], (s->pool_size - 1 - idx) * sizeof(oc_pent));
  s->pool[idx] = en;
}
/* evictMinExpireEntry (map.go:319-342); the reference's own argument guarantees a hit */
static void sm_evict_min(oc_shard* s, uint64_t old[3]) {
  uint64_t pos = 0;
  while (pos < s->pool_size) {
    if (sm_delete(s, s->pool[pos].key, s->pool[pos].klen, s->pool[pos].slot, old) == 0) break;
    pos++;
  }
  if (pos + 1 <= s->pool_size)
    memmove(&s->pool[0], &s->pool[pos + 1], (s->pool_size - pos - 1) * sizeof(oc_pent));
  s->pool_size -= pos;
}
/* evict (map.go:349-371) */
static void sm_evict(oc_smap* m, oc_shard* s, uint64_t old[3]) {
  uint64_t left = s->sample;
  while (left > 0) {
    const uint64_t slot = sm_rand(m, s->cap);
    oc_bkt* e = &s->b[slot];
    if (!e->key) continue;
    for (; left > 0 && e; e = e->next, --left) {
      oc_pent p;
      p.expire = e->expire;
      p.key = sm_keep_key(m, e->key, e->klen);
      p.klen = e->klen;
      p.slot = slot;
      sm_pool_insert(s, p);
    }
  }
  sm_evict_min(s, old);
}

/* Set (map.go:160-210 via ShardMap.Set map.go:414-418): 0 inserted (no old value), 1 replaced (old = the
 * previous value), 2 inserted after an eviction (old = the evicted value) */
int oc_smap_set(oc_smap* m, const uint8_t* k, size_t kl, const uint64_t val[3], uint64_t old[3]) {
  const uint64_t h = sm_hash(m, k, kl);
  oc_shard* s = &m->sh[h % m->nsh];
  const uint64_t slot = h % s->cap;
  oc_bkt* e = sm_find(s, k, (uint32_t)kl, slot);
  if (e) {
    if (old) oc_memcpy(old, e->val, sizeof e->val);
    oc_memcpy(e->val, val, sizeof e->val);
    e->expire = sm_expire(m, s);
    return 1;
  }
  int ret = 0;
  if (s->used + 1 > s->limited) { sm_evict(m, s, old); ret = 2; }
  s->used++;
  oc_bkt* hd = &s->b[slot];
  uint8_t* kc = (uint8_t*)malloc(kl ? kl : 1);
  oc_memcpy(kc, k, kl);
  if (!hd->key) {
    hd->key = kc; hd->klen = (uint32_t)kl;
    oc_memcpy(hd->val, val, sizeof hd->val);
    hd->expire = sm_expire(m, s);
    return ret;
  }
  oc_bkt* n = (oc_bkt*)calloc(1, sizeof *n);
  n->key = kc; n->klen = (uint32_t)kl;
  oc_memcpy(n->val, val, sizeof n->val);
  n->next = hd->next;
  n->expire = sm_expire(m, s);
  hd->next = n;
  return ret;
}
/* Get (map.go:212-227): 0 found, 1 ErrKeyNotFound */
int oc_smap_get(oc_smap* m, const uint8_t* k, size_t kl, uint64_t val[3]) {
  const uint64_t h = sm_hash(m, k, kl);
  oc_shard* s = &m->sh[h % m->nsh];
  oc_bkt* e = sm_find(s, k, (uint32_t)kl, h);
  if (!e) return 1;
  oc_memcpy(val, e->val, sizeof e->val);
  return 0;
}
/* Delete (map.go:248-258): 0 deleted (old out), 1 ErrKeyNotFound */
int oc_smap_delete(oc_smap* m, const uint8_t* k, size_t kl, uint64_t old[3]) {
  const uint64_t h = sm_hash(m, k, kl);
  oc_shard* s = &m->sh[h % m->nsh];
  return sm_delete(s, k, (uint32_t)kl, h, old);
}
/* every live entry, in bucket order: keys concatenated (koff has n + 1 entries), values 3 per entry;
 * returns the entry count (outputs written only while they fit) */
uint64_t oc_smap_export(const oc_smap* m, uint8_t* keys, uint64_t keys_cap, uint64_t* koff, uint64_t* vals,
                        uint64_t cap, uint64_t* key_bytes) {
  uint64_t n = 0, kb = 0;
  if (koff && cap) koff[0] = 0;
  for (uint32_t i = 0; i < m->nsh; ++i)
    for (uint64_t j = 0; j < m->sh[i].cap; ++j) {
      if (!m->sh[i].b[j].key) continue;
      for (const oc_bkt* e = &m->sh[i].b[j]; e; e = e->next) {
        if (n < cap && kb + e->klen <= keys_cap) {
          if (e->klen) oc_memcpy(keys + kb, e->key, e->klen);
          oc_memcpy(vals + 3 * n, e->val, sizeof e->val);
          koff[n + 1] = kb + e->klen;
        }
        kb += e->klen;
        n++;
      }
    }
  if (key_bytes) *key_bytes = kb;
  return n;
}

/* Index over the bounded map (index.go:81-165): op 0 Put, 1 Delete, 2 SoftDelete. Returns the WriteStat
 * the reference fills (index.go:115-118,134-137,157-160): *free_bytes = old.valueSize and *free_fid =
 * old.fid when an old value came back (a replaced key, a deleted key, or the entry evicted to make room),
 * else 0, 0. */
void oc_bindex_op(oc_smap* m, const uint8_t* ns, size_t nsl, const uint8_t* key, size_t kl, int op, uint64_t fid,
                  uint64_t off, uint64_t size, uint64_t* free_fid, uint64_t* free_bytes) {
  uint8_t* mk = merged_key(ns, nsl, key, kl);
  uint64_t old[3] = {0, 0, 0};
  int has_old = 0;
  if (op == 1) {
    has_old = oc_smap_delete(m, mk, nsl + kl, old) == 0;
  } else {
    const uint64_t v[3] = {op == 0 ? fid : 0, op == 0 ? off : 0, op == 0 ? size : 0};
    has_old = oc_smap_set(m, mk, nsl + kl, v, old) != 0;
  }
  free(mk);
  if (free_fid) *free_fid = has_old ? old[0] : 0;
  if (free_bytes) *free_bytes = has_old ? old[2] : 0;
}
/* Index.Get over the bounded map: 0 found, 1 ErrKeyNotFound, 2 ErrKeySoftDeleted */
int oc_bindex_get(oc_smap* m, const uint8_t* ns, size_t nsl, const uint8_t* key, size_t kl, uint64_t* fid,
                  uint64_t* off, uint64_t* size) {
  uint8_t* mk = merged_key(ns, nsl, key, kl);
  uint64_t v[3];
  const int r = oc_smap_get(m, mk, nsl + kl, v);
  free(mk);
  if (r) return 1;
  *fid = v[0]; *off = v[1]; *size = v[2];
  return v[1] == 0 ? 2 : 0;
}
/* recoverFromWal's Put loop (db_impl.go:290-313) into the bounded index, as oc_index_put_segment */
int oc_bindex_put_segment(oc_smap* m, const uint8_t* seg, uint64_t len, uint32_t start_off, uint64_t base_time,
                          uint32_t ns_size, uint32_t etag_size, int mode, uint64_t fid, int use_rec_fid,
                          uint64_t* n_put) {
  oc_decode* d = oc_decode_segment(seg, len, start_off, base_time, ns_size, etag_size, mode);
  int ret = d->err_class;
  uint64_t r = 0;
  for (; r < d->n_recs; ++r) {
    const oc_rec* rc = &d->recs[r];
    if (rc->status != OC_ST_OK) { ret = 16 + rc->status; break; }
    const uint8_t *ns, *key;
    uint64_t kl;
    rec_ns_key(rc, d->bytes + d->byte_offs[r], ns_size, mode, &ns, &key, &kl);
    if (mode == 0) oc_bindex_op(m, ns, ns_size, key, kl, 0, fid, rc->foff - OC_HEADER_SIZE, rc->size, NULL, NULL);
    else oc_bindex_op(m, ns, ns_size, key, kl, 0, use_rec_fid ? rc->expire : fid, rc->val_len, rc->meta_len, NULL, NULL);
  }
  *n_put = r;
  oc_decode_free(d);
  return ret;
}
/* doFilter over every delivered row against the bounded index (compaction.go:329-348: a key evicted from
 * the index is dropped like a deleted one) */
uint64_t oc_bindex_compact_filter(oc_smap* m, const uint8_t* seg, uint64_t len, uint32_t start_off,
                                  uint64_t base_time, uint32_t ns_size, uint32_t etag_size, uint64_t src_fid,
                                  uint8_t* keep, uint64_t n_keep) {
  oc_decode* d = oc_decode_segment(seg, len, start_off, base_time, ns_size, etag_size, 0);
  uint64_t r = 0;
  for (uint64_t i = 0; i < n_keep; ++i) keep[i] = 0;
  for (; r < d->n_recs; ++r) {
    const oc_rec* rc = &d->recs[r];
    if (rc->status != OC_ST_OK) break;
    const uint8_t *ns, *key;
    uint64_t kl, fid = 0, off = 0, size = 0;
    rec_ns_key(rc, d->bytes + d->byte_offs[r], ns_size, 0, &ns, &key, &kl);
    const int g = oc_bindex_get(m, ns, ns_size, key, kl, &fid, &off, &size);
    if (r < n_keep) keep[r] = (g == 0 && fid == src_fid && off == rc->foff - OC_HEADER_SIZE) ? 1 : 0;
  }
  oc_decode_free(d);
  return r;
}
