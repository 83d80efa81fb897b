// bcw_api.cpp -- host side of libbcw.so: contexts, constant tables, super block, host WAL writer
// and the launch orchestration of the decode pipeline (kernels in bcw_decode.hip).
#include <hip/hip_runtime.h>
#include <nmmintrin.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "bcw.h"
#include "bcw_internal.h"

namespace bcw {

// ---- CRC-32C constant tables (reflected polynomial 0x82F63B78, Go crc32.Castagnoli) ----
static void byte_table(uint32_t* t0) {
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    t0[b] = c;
  }
}

static inline uint32_t zero_step(const uint32_t* t0, uint32_t s) { return (s >> 8) ^ t0[s & 0xffu]; }

// images of the 32 basis vectors under "advance over n zero bytes"
static void shift_basis(const uint32_t* t0, uint64_t n, uint32_t* img) {
  for (int i = 0; i < 32; ++i) {
    uint32_t v = 1u << i;
    for (uint64_t k = 0; k < n; ++k) v = zero_step(t0, v);
    img[i] = v;
  }
}
static inline uint32_t apply_basis(const uint32_t* img, uint32_t x) {
  uint32_t r = 0;
  for (int i = 0; x; ++i, x >>= 1)
    if (x & 1u) r ^= img[i];
  return r;
}

// basis images of the inverse of a (bijective) GF(2)-linear map given by its basis images
static void invert_basis(const uint32_t* img, uint32_t* inv) {
  uint32_t out[32], in[32];
  for (int i = 0; i < 32; ++i) { out[i] = img[i]; in[i] = 1u << i; }
  for (int bit = 0; bit < 32; ++bit) {
    int p = bit;
    while (p < 32 && !((out[p] >> bit) & 1u)) ++p;  // x^8n mod P is invertible: a pivot always exists
    std::swap(out[bit], out[p]);
    std::swap(in[bit], in[p]);
    for (int r = 0; r < 32; ++r)
      if (r != bit && ((out[r] >> bit) & 1u)) { out[r] ^= out[bit]; in[r] ^= in[bit]; }
  }
  for (int bit = 0; bit < 32; ++bit) inv[bit] = in[bit];
}

static void nibble_image(const uint32_t* img, uint32_t* t) {
  for (int i = 0; i < 8; ++i)
    for (uint32_t n = 0; n < 16; ++n) t[i * 16 + n] = apply_basis(img, n << (4 * i));
}

// encode shift operators (nibble images, 128 words each; layout in bcw_internal.h): A_{8*16*n},
// A_{8*256*n}, A_{8*4096*n} (k_write's lane chains), A_{8t}^-1 (t < 16), and A_{8*2^k} / A_{8*2^k}^-1 for
// shifts by arbitrary distances (the CRC combine of re-encoded records)
static void build_enc_ops(uint32_t* ops) {
  uint32_t t0[256];
  byte_table(t0);
  uint32_t img[32], inv[32], sq[32];
  for (int n = 0; n < 16; ++n) { shift_basis(t0, 16ull * n, img); nibble_image(img, ops + n * 128); }
  for (int n = 0; n < 16; ++n) { shift_basis(t0, 256ull * n, img); nibble_image(img, ops + (16 + n) * 128); }
  for (int n = 0; n < 8; ++n) { shift_basis(t0, 4096ull * n, img); nibble_image(img, ops + (32 + n) * 128); }
  for (int t = 0; t < 16; ++t) {
    shift_basis(t0, (uint64_t)t, img);
    invert_basis(img, inv);
    nibble_image(inv, ops + (kOpInv + t) * 128);
  }
  shift_basis(t0, 1, img);  // A_8, then repeated squaring
  for (int k = 0; k < 32; ++k) {
    nibble_image(img, ops + (kOpPow2 + k) * 128);
    if (k < 15) {
      invert_basis(img, inv);
      nibble_image(inv, ops + (kOpPow2Inv + k) * 128);
    }
    for (int i = 0; i < 32; ++i) sq[i] = apply_basis(img, img[i]);
    memcpy(img, sq, sizeof img);
  }
}

// initc[L] = A_{8L}(0xFFFFFFFF): the contribution of the CRC init value after L data bytes
void build_initc(uint32_t* initc) {
  uint32_t t0[256];
  byte_table(t0);
  uint32_t v = 0xffffffffu;
  for (uint32_t L = 0; L <= kBlock; ++L) {
    initc[L] = v;
    v = zero_step(t0, v);
  }
}

// ---- host CRC-32C (SSE4.2) for the writer and bcw_crc32c_masked ----
static uint32_t crc32c_hw(const uint8_t* p, size_t n) {
  uint64_t c = 0xffffffffu;
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    c = _mm_crc32_u64(c, w);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return ~c32;
}
static inline uint32_t mask_crc(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

}  // namespace bcw

using namespace bcw;


#define HIPCHK(x)                          \
  do {                                     \
    if ((x) != hipSuccess) return BCW_E_HIP; \
  } while (0)

namespace {
std::atomic<uint64_t> g_ctx_ids{1};
}  // namespace

extern "C" {

int bcw_abi_version(void) { return BCW_ABI_VERSION; }

const char* bcw_strerror(int code) {
  switch (code) {
    case BCW_OK: return "ok";
    case BCW_E_INVAL: return "invalid argument";
    case BCW_E_HIP: return "HIP runtime error";
    case BCW_E_NOMEM: return "out of memory";
    case BCW_E_CAPACITY: return "output capacity too small";
    case BCW_E_NODEVICE: return "no HIP device";
    case BCW_E_IO: return "file read / write failed";
    default: return "unknown error";
  }
}

int bcw_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

uint32_t bcw_crc32c_masked(const uint8_t* p, uint64_t n) { return mask_crc(crc32c_hw(p, (size_t)n)); }

void bcw_write_super_block(uint8_t out[40], uint64_t create_time, uint64_t base_time) {
  // wal.go:332-360: magic @0, blockSize @8, startOff @16, createTime @20, baseTime @28, crc @36
  memset(out, 0, 40);
  const uint64_t magic = BCW_MAGIC, bs = BCW_BLOCK_SIZE;
  const uint32_t so = BCW_SUPER_BLOCK_SIZE;
  memcpy(out + 0, &magic, 8);
  memcpy(out + 8, &bs, 8);
  memcpy(out + 16, &so, 4);
  memcpy(out + 20, &create_time, 8);
  memcpy(out + 28, &base_time, 8);
  const uint32_t crc = bcw_crc32c_masked(out, 36);
  memcpy(out + 36, &crc, 4);
}

int bcw_load_super_block(const uint8_t* p, uint64_t n, bcw_super_block* out) {
  // wal.go:362-398: CRC first, then magic, then blockSize (startOff is not validated)
  if (!p || !out) return BCW_E_INVAL;
  if (n < BCW_SUPER_BLOCK_SIZE) return BCW_SB_SHORT;
  uint32_t want;
  memcpy(&want, p + 36, 4);
  const uint32_t crc = bcw_crc32c_masked(p, 36);
  if (crc != want) return BCW_SB_CRC;
  memcpy(&out->magic, p, 8);
  if (out->magic != BCW_MAGIC) return BCW_SB_MAGIC;
  memcpy(&out->block_size, p + 8, 8);
  memcpy(&out->start_off, p + 16, 4);
  if (out->block_size != BCW_BLOCK_SIZE) return BCW_SB_BLOCKSIZE;
  memcpy(&out->create_time, p + 20, 8);
  memcpy(&out->base_time, p + 28, 8);
  out->crc = crc;
  return BCW_SB_OK;
}

// WalRecordSize (wal.go:61-86), same uint64 arithmetic (offset below 40 wraps as in Go)
uint64_t bcw_wal_record_size(uint64_t offset, uint64_t size) {
  uint64_t left = size, phy = 0;
  offset -= BCW_SUPER_BLOCK_SIZE;
  while (left > 0) {
    uint64_t leftover = BCW_BLOCK_SIZE - (offset % BCW_BLOCK_SIZE);
    if (leftover < BCW_HEADER_SIZE) {
      phy += leftover;
      offset += leftover;
      leftover = BCW_BLOCK_SIZE;
    }
    const uint64_t frag = std::min(left, leftover - BCW_HEADER_SIZE);
    phy += BCW_HEADER_SIZE + frag;
    offset += BCW_HEADER_SIZE + frag;
    left -= frag;
  }
  return phy;
}

// WalBlockIndexRange (wal.go:88-97)
void bcw_wal_block_index_range(uint64_t offset, uint64_t size, uint64_t* first_blk_idx, uint64_t* first_blk_off,
                               uint64_t* blk_num) {
  const uint64_t rs = bcw_wal_record_size(offset, size);
  const uint64_t first = (offset - BCW_SUPER_BLOCK_SIZE) / BCW_BLOCK_SIZE;
  const uint64_t last = (offset - BCW_SUPER_BLOCK_SIZE + rs) / BCW_BLOCK_SIZE;
  if (first_blk_idx) *first_blk_idx = first;
  if (first_blk_off) *first_blk_off = first * BCW_BLOCK_SIZE + BCW_SUPER_BLOCK_SIZE;
  if (blk_num) *blk_num = last - first + 1;
}

uint64_t bcw_max_fragments(uint64_t seg_len, uint32_t start_off) {
  if (seg_len <= start_off) return 0;
  return (seg_len - start_off) / BCW_HEADER_SIZE + 1;
}

int bcw_ctx_create(int device, bcw_ctx** out) {
  if (!out) return BCW_E_INVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return BCW_E_NODEVICE;
  if (device < 0 || device >= n) return BCW_E_INVAL;
  bcw_ctx* c = new (std::nothrow) bcw_ctx();
  if (!c) return BCW_E_NOMEM;
  c->device = device;
  c->id = g_ctx_ids.fetch_add(1);
  DeviceGuard dg(device);
  if (!dg.ok) { delete c; return BCW_E_HIP; }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    c->num_cus = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) { delete c; return BCW_E_HIP; }
  c->cur = c->own;
  std::vector<uint32_t> initc(kBlock + 1);
  build_initc(initc.data());
  std::vector<uint32_t> enc_ops(kEncOpsWords);
  build_enc_ops(enc_ops.data());
  std::vector<uint32_t> pow2(kPow2Ops * 128);
  {
    uint32_t t0[256], img[32], sq[32];
    byte_table(t0);
    shift_basis(t0, 1, img);  // A_8, then repeated squaring: A_{8*2^(k+1)} = A_{8*2^k} o A_{8*2^k}
    for (int k = 0; k < kPow2Ops; ++k) {
      nibble_image(img, pow2.data() + k * 128);
      for (int i = 0; i < 32; ++i) sq[i] = apply_basis(img, img[i]);
      memcpy(img, sq, sizeof img);
    }
  }
  std::vector<uint32_t> image2(kS2Image);
  {  // stream verify (bcw_internal.h kS2*): slice rows with the shifted tables, lane operators, split operators
    uint32_t tk[4][256], t0[256], img[32], nib[128], step[32], m[32];
    byte_table(t0);
    memcpy(tk[0], t0, sizeof t0);
    for (int k = 1; k < 4; ++k)
      for (int e = 0; e < 256; ++e) tk[k][e] = (tk[k - 1][e] >> 8) ^ t0[tk[k - 1][e] & 0xffu];
    uint32_t sh[32];
    shift_basis(t0, kSChunk - kSPiece, sh);
    for (int e = 0; e < 256; ++e)
      for (int s = 0; s < 4; ++s)
        for (int cp = 0; cp < 8; ++cp) {
          image2[kS2SliceOff + e * 64 + s * 8 + cp] = tk[3 - s][e];
          image2[kS2SliceOff + e * 64 + 32 + s * 8 + cp] = apply_basis(sh, tk[3 - s][e]);
        }
    shift_basis(t0, kSPiece, step);
    for (int i = 0; i < 32; ++i) m[i] = 1u << i;  // identity for lane 63
    for (int l = 63; l >= 0; --l) {
      nibble_image(m, nib);
      for (int k = 0; k < 128; ++k) image2[kS2LopOff + k * 64 + l] = nib[k];
      for (int i = 0; i < 32; ++i) m[i] = apply_basis(step, m[i]);
    }
    for (int k = 0; k < kSPW; ++k) {  // split operators as byte tables: [k][t][e] = A(e << 8t)
      shift_basis(t0, 4u * (kSPW - k) + (kSChunk - kSPiece), img);
      for (int t = 0; t < 4; ++t)
        for (uint32_t e = 0; e < 256; ++e)
          image2[kS2KopOff + (k * 4 + t) * 256 + e] = apply_basis(img, e << (8 * t));
    }
    auto put_bytes = [&](int at, const uint8_t (&b)[16]) {
      for (int w = 0; w < 4; ++w)
        image2[at + w] = b[4 * w] | b[4 * w + 1] << 8 | b[4 * w + 2] << 16 | (uint32_t)b[4 * w + 3] << 24;
    };
    for (int n = 0; n < kS2GeN; ++n) {  // GE[n]: bytes q >= n
      uint8_t b[16];
      for (int q = 0; q < 16; ++q) b[q] = q >= n ? 0xff : 0x00;
      put_bytes(kS2Ge + 4 * n, b);
    }
    for (int m = 0; m < kS2JselN; ++m) {  // JSEL[m]: perm selectors, J byte q - o at q in [o, o + 4) (o = m - 3), else 0
      uint8_t b[16];
      for (int q = 0; q < 16; ++q) {
        const int p = q - (m - 3);
        b[q] = (m < kS2JselN - 1 && p >= 0 && p < 4) ? (uint8_t)(4 + p) : 0x0c;
      }
      put_bytes(kS2Jsel + 4 * m, b);
    }
    for (int g = 0; g < kS2GapN; ++g) {  // GAP[g]: J at [o, o + 4) (o = g - 6), zeros at [o + 4, o + 7), else the byte
      uint8_t b[16];
      for (int q = 0; q < 16; ++q) {
        const int p = q - (g - 6);
        b[q] = g == kS2GapN - 1 ? (uint8_t)(q & 3) : (p >= 0 && p < 4) ? (uint8_t)(4 + p) : (p >= 4 && p < 7) ? 0x0c
                                                                                            : (uint8_t)(q & 3);
      }
      put_bytes(kS2Gap + 4 * g, b);
    }
  }
  bool ok = hipMalloc(&c->tabs.lds_image2, image2.size() * 4) == hipSuccess &&
            hipMemcpy(c->tabs.lds_image2, image2.data(), image2.size() * 4, hipMemcpyHostToDevice) == hipSuccess;
  ok = ok && hipMalloc(&c->tabs.initc, initc.size() * 4) == hipSuccess &&
            hipMalloc(&c->tabs.enc_ops, enc_ops.size() * 4) == hipSuccess &&
            hipMalloc(&c->tabs.pow2, pow2.size() * 4) == hipSuccess &&
            hipMalloc(&c->d_eres, sizeof(bcw_encode_result)) == hipSuccess &&
            hipMalloc(&c->d_result, sizeof(bcw_decode_result)) == hipSuccess &&
            hipMalloc(&c->d_ires, sizeof(bcw_index_result)) == hipSuccess;
  ok = ok && hipMemcpy(c->tabs.initc, initc.data(), initc.size() * 4, hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(c->tabs.enc_ops, enc_ops.data(), enc_ops.size() * 4, hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(c->tabs.pow2, pow2.data(), pow2.size() * 4, hipMemcpyHostToDevice) == hipSuccess;
  if (!ok) { bcw_ctx_destroy(c); return BCW_E_NOMEM; }
  *out = c;
  return BCW_OK;
}

static void free_scratch(Scratch& s) {
  (void)hipFree(s.fbase);
  (void)hipFree(s.rbase);
  (void)hipFree(s.bsum);
  (void)hipFree(s.lb);
  (void)hipFree(s.lbe);
  (void)hipFree(s.frags);
  (void)hipFree(s.srec);
  (void)hipFree(s.fok);
  (void)hipFree(s.wstart);
  (void)hipFree(s.xbal);
  (void)hipFree(s.misc);
  s = Scratch{};
}

static void free_enc_scratch(EncScratch& e) {
  void* ptrs[] = {e.sz,    e.mflag, e.dsrc, e.da,      e.hda,       e.hsz,  e.dpos,
                  e.hpos,  e.tiles, e.ev,   e.evb,     e.recdesc,   e.emisc, e.evt,
                  e.hnl,   e.evw,   e.wl};
  for (void* q : ptrs) (void)hipFree(q);
  hipStream_t aux = e.aux;
  hipEvent_t evs[3] = {e.ev_scan, e.ev_hscan, e.ev_desc};
  e = EncScratch{};
  e.aux = aux;  // the auxiliary stream and its events live as long as the context
  e.ev_scan = evs[0];
  e.ev_hscan = evs[1];
  e.ev_desc = evs[2];
}

int bcw_ctx_destroy(bcw_ctx* c) {
  if (!c) return BCW_E_INVAL;
  DeviceGuard dg(c->device);
  if (c->cur) (void)hipStreamSynchronize(c->cur);
  free_scratch(c->s);
  free_enc_scratch(c->es);
  if (c->es.aux) (void)hipStreamSynchronize(c->es.aux);
  if (c->es.ev_scan) (void)hipEventDestroy(c->es.ev_scan);
  if (c->es.ev_hscan) (void)hipEventDestroy(c->es.ev_hscan);
  if (c->es.ev_desc) (void)hipEventDestroy(c->es.ev_desc);
  if (c->es.aux) (void)hipStreamDestroy(c->es.aux);
  (void)hipFree(c->tabs.enc_ops);
  (void)hipFree(c->tabs.pow2);
  (void)hipFree(c->d_keep);
  (void)hipFree(c->d_eout);
  (void)hipFree(c->d_eres);
  (void)hipFree(c->tabs.initc);
  (void)hipFree(c->tabs.lds_image2);
  (void)hipFree(c->d_seg);
  (void)hipFree(c->d_tab_mem);
  (void)hipFree(c->d_result);
  (void)hipFree(c->d_ires);
  for (auto& m : c->prof.marks) { (void)hipEventDestroy(m.a); (void)hipEventDestroy(m.b); }
  for (auto e : c->prof.pool) (void)hipEventDestroy(e);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
  return BCW_OK;
}

int bcw_ctx_set_stream(bcw_ctx* c, void* stream) {
  if (!c) return BCW_E_INVAL;
  c->cur = stream ? (hipStream_t)stream : c->own;
  return BCW_OK;
}
void* bcw_ctx_stream(bcw_ctx* c) { return c ? (void*)c->cur : nullptr; }
int bcw_ctx_device(bcw_ctx* c) { return c ? c->device : -1; }
int bcw_ctx_sync(bcw_ctx* c) {
  if (!c) return BCW_E_INVAL;
  return hipStreamSynchronize(c->cur) == hipSuccess ? BCW_OK : BCW_E_HIP;
}

static int ensure_scratch(bcw_ctx* c, uint64_t nblocks, uint64_t frag_cap) {
  Scratch& s = c->s;
  if (nblocks <= s.nblocks_cap && frag_cap <= s.frag_cap && s.misc) return BCW_OK;
  (void)hipStreamSynchronize(c->cur);
  const uint64_t nb = std::max(nblocks, s.nblocks_cap);
  const uint64_t fc = std::max(frag_cap, s.frag_cap);
  free_scratch(s);
  // look-back words: one per 64-block k_chase workgroup. The stream records have 4 entries of slack: k_crc's stream
  // loads the record after a wave's current fragment unconditionally (bcw_decode.hip, stream_verify)
  const uint64_t nwg = std::max<uint64_t>(nb / 64 + 2, (uint64_t)c->num_cus + 2);
  bool ok = hipMalloc(&s.fbase, (nb + 1) * 4) == hipSuccess && hipMalloc(&s.rbase, (nb + 1) * 4) == hipSuccess &&
            hipMalloc(&s.bsum, (nb + 1) * sizeof(uint2)) == hipSuccess && hipMalloc(&s.lb, nwg * 8) == hipSuccess &&
            hipMalloc(&s.lbe, nwg * 8) == hipSuccess && hipMalloc(&s.frags, fc * sizeof(Frag)) == hipSuccess &&
            hipMalloc(&s.srec, (fc + 4) * sizeof(uint4)) == hipSuccess &&
            hipMalloc(&s.fok, fc) == hipSuccess &&
            hipMalloc(&s.wstart, ((size_t)c->num_cus * kCrcWaves + 1) * 4) == hipSuccess &&
            hipMalloc(&s.xbal, sizeof(XBal)) == hipSuccess &&
            hipMalloc(&s.misc, 16 * sizeof(uint64_t)) == hipSuccess;
  if (!ok) { free_scratch(s); return BCW_E_NOMEM; }
  s.nblocks_cap = nb;
  s.frag_cap = fc;
  s.nlb = nwg;
  s.epoch = 1;
  s.chase_direct = c->chase_direct;
  // on the codec's stream: a null-stream hipMemset is not ordered before kernels on a non-blocking
  // stream, and a look-back word zeroed after k_chase published it would never be seen again
  // misc[15] (the first unknown-type fragment, an atomicMin in k_chase) starts at UINT64_MAX; every decode's
  // finalizer resets it for the next one
  // misc[0] (first bad record) and misc[14] (first CRC failure) start at UINT64_MAX too
  XBal xb{};  // equal weights to begin with; k_crc's finalize adapts them decode by decode
  for (uint32_t y = 0; y < 8; ++y) xb.w[y] = 65536u;
  if (hipMemcpyHtoDAsync(s.xbal, &xb, sizeof xb, c->cur) != hipSuccess || hipStreamSynchronize(c->cur) != hipSuccess ||
      hipMemsetAsync(s.lb, 0, nwg * 8, c->cur) != hipSuccess || hipMemsetAsync(s.lbe, 0, nwg * 8, c->cur) != hipSuccess ||
      hipMemsetAsync(s.misc, 0, 16 * sizeof(uint64_t), c->cur) != hipSuccess ||
      hipMemsetAsync(s.misc + 14, 0xff, 2 * sizeof(uint64_t), c->cur) != hipSuccess ||
      hipMemsetAsync(s.misc, 0xff, sizeof(uint64_t), c->cur) != hipSuccess) {
    free_scratch(s);
    return BCW_E_HIP;
  }
  return BCW_OK;
}

int bcw_decode_segment_async(bcw_ctx* c, const uint8_t* d_seg, const bcw_decode_params* p,
                             const bcw_record_table* t, bcw_decode_result* d_result) {
  if (!c || !p || !t || !d_result) return BCW_E_INVAL;
  if (p->mode != BCW_MODE_RECORD && p->mode != BCW_MODE_HINT) return BCW_E_INVAL;
  if (!t->foff || !t->size || !t->expire || !t->key_len || !t->val_len || !t->meta_len || !t->first_frag ||
      !t->emit_frag || !t->hdr_size || !t->flags || !t->etag_off || !t->status)
    return BCW_E_INVAL;
  if (p->mode == BCW_MODE_HINT && (!t->aux0 || !t->aux1)) return BCW_E_INVAL;
  if (p->seg_len > BCW_MAX_SEGMENT) return BCW_E_INVAL;  // k_crc's item arithmetic is 32-bit (< 2^24 blocks)
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  c->last_start_off = p->start_off;
  const uint64_t gen = (c->id << 32) | (++c->gen_seq & 0xffffffffull);
  c->frag_gen = gen;  // from here on the fragment scratch belongs to this decode
  bcw_decode_result r{};
  r.err_frag = ~0ull;
  r.first_bad_record = -1;
  r.generation = gen;
  if ((uint64_t)p->start_off > p->seg_len) {
    // wal_iterator.go:49,55: bufSize < 0 -> i.buf[:bufSize] panics before any fragment
    r.err_class = BCW_ERR_PANIC;
    HIPCHK(hipMemcpyAsync(d_result, &r, sizeof r, hipMemcpyHostToDevice, c->cur));
    return BCW_OK;
  }
  const uint64_t nblocks = (p->seg_len - p->start_off + kBlock - 1) / kBlock;
  if (nblocks == 0 || !d_seg) {
    if (nblocks != 0) return BCW_E_INVAL;
    HIPCHK(hipMemcpyAsync(d_result, &r, sizeof r, hipMemcpyHostToDevice, c->cur));
    return BCW_OK;
  }
  // fragment ids are u32: segments may be any size as long as they hold < 2^32 - 16 fragments
  // (bcw_ctx_reserve_fragments refuses more)
  // first guess of the fragment count (a retry sizes it exactly): 4 KiB-class records average ~4 KiB
  // per fragment; hint WALs hold ~130 B records
  const uint64_t per = p->mode == BCW_MODE_HINT ? 96 : 256;
  uint64_t want = std::max<uint64_t>(65536, (p->seg_len - p->start_off) / per + nblocks * 2);
  want = std::max(want, c->frag_hint);
  want = std::min(want, bcw_max_fragments(p->seg_len, p->start_off) + 64);
  want = std::min<uint64_t>(want, 0xfffffff0ull);
  int rc = ensure_scratch(c, nblocks, want);
  if (rc != BCW_OK) return rc;
  c->s.test_abort_wg = c->test_abort_wg;  // one-shot (launch_decode clears the scratch copy)
  c->test_abort_wg = 0;
  if (launch_decode(d_seg, *p, *t, d_result, c->tabs, c->s, nblocks, gen, c->cur, c->num_cus, &c->prof) !=
      hipSuccess)
    return BCW_E_HIP;
  return BCW_OK;
}

int bcw_decode_fragments_async(bcw_ctx* c, const bcw_frag_table* d_frags) {
  if (!c || !d_frags) return BCW_E_INVAL;
  if (!c->s.misc) return BCW_OK;
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  const uint64_t n = std::min(c->s.frag_cap, d_frags->capacity);
  return launch_export_frags(c->s, *d_frags, c->last_start_off, c->cur, n, c->tabs.initc) == hipSuccess ? BCW_OK
                                                                                                  : BCW_E_HIP;
}

static const char* kKernelNames[K_NUM] = {"k_chase", "k_crc", "(retired)", "k_enc_prep", "k_enc_scan", "k_events",
                                          "k_write", "k_hint_layout", "k_events_hint"};

int bcw_ctx_reserve_fragments(bcw_ctx* c, uint64_t n) {
  if (!c || n >= 0xfffffff0ull) return BCW_E_INVAL;
  c->frag_hint = std::max(c->frag_hint, n);
  return BCW_OK;
}

int bcw_ctx_set_option(bcw_ctx* c, int option, uint64_t value) {
  if (!c) return BCW_E_INVAL;
  switch (option) {
    case BCW_OPT_CHASE_DIRECT:
      if (value > BCW_CHASE_DIRECT_MAX) return BCW_E_INVAL;
      c->s.chase_direct = (uint32_t)value;
      c->chase_direct = (uint32_t)value;
      return BCW_OK;
    case BCW_OPT_DECODE_PATH:    // retired options (bcw.h): only their one remaining value is accepted
    case BCW_OPT_DECODE_CHUNKS:
      return value == 1 ? BCW_OK : BCW_E_INVAL;
    case BCW_OPT_XCD_BALANCE:
      if (value > 1) return BCW_E_INVAL;
      c->s.xbal_on = (uint32_t)value;
      return BCW_OK;
    case BCW_OPT_FILTER_SNAPSHOT:
      if (value > 1) return BCW_E_INVAL;
      c->filter_snapshot = value != 0;
      return BCW_OK;
    case BCW_OPT_TEST_ABORT_WAIT: {  // fault injection: refused unless the process opted in (BCW_TEST_HOOKS=1)
      const char* hooks = getenv("BCW_TEST_HOOKS");
      if (!hooks || strcmp(hooks, "1") != 0 || value > 0xffffffffull) return BCW_E_INVAL;
      c->test_abort_wg = value;
      return BCW_OK;
    }
    default:
      return BCW_E_INVAL;
  }
}

int bcw_ctx_set_profiling(bcw_ctx* c, int mask) {
  if (!c) return BCW_E_INVAL;
  c->prof.mask = (uint32_t)mask;
  return BCW_OK;
}

int bcw_ctx_set_profiling_sample(bcw_ctx* c, int every) {
  if (!c || every < 1) return BCW_E_INVAL;
  c->prof.every = (uint32_t)every;
  for (uint32_t& q : c->prof.seq) q = 0;
  return BCW_OK;
}

int bcw_ctx_kernel_times(bcw_ctx* c, double* total_ms, uint64_t* launches, int n) {
  if (!c || n < 0) return BCW_E_INVAL;
  if (hipStreamSynchronize(c->cur) != hipSuccess) return BCW_E_HIP;
  for (int k = 0; k < n; ++k) { if (total_ms) total_ms[k] = 0; if (launches) launches[k] = 0; }
  for (const auto& m : c->prof.marks) {
    float ms = 0;
    if (m.kid < n && hipEventElapsedTime(&ms, m.a, m.b) == hipSuccess) {
      if (total_ms) total_ms[m.kid] += ms;
      if (launches) launches[m.kid] += 1;
    }
    c->prof.pool.push_back(m.a);
    c->prof.pool.push_back(m.b);
  }
  c->prof.marks.clear();
  return K_NUM;
}

const char* bcw_kernel_name(int kid) { return (kid >= 0 && kid < K_NUM) ? kKernelNames[kid] : nullptr; }

int bcw_decode_fragments(bcw_ctx* c, const bcw_frag_table* h, uint64_t* n_total) {
  if (!c || !h) return BCW_E_INVAL;
  if (n_total) *n_total = 0;
  if (!c->s.misc) return BCW_OK;
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  uint64_t misc[16];
  HIPCHK(hipMemcpyAsync(misc, c->s.misc, sizeof misc, hipMemcpyDeviceToHost, c->cur));
  HIPCHK(hipStreamSynchronize(c->cur));
  const uint64_t total = std::min(misc[4], c->s.frag_cap);
  if (n_total) *n_total = total;
  const uint64_t n = std::min(total, h->capacity);
  if (n == 0) return BCW_OK;
  void* mem = nullptr;
  if (hipMalloc(&mem, n * 19) != hipSuccess) return BCW_E_NOMEM;
  uint8_t* m = (uint8_t*)mem;
  bcw_frag_table d;
  d.capacity = n;
  d.data_off = (uint64_t*)m; m += n * 8;
  d.len = (uint32_t*)m; m += n * 4;
  d.stored_crc = (uint32_t*)m; m += n * 4;
  d.type = m; m += n;
  d.crc_ok = m;
  bool ok = launch_export_frags(c->s, d, c->last_start_off, c->cur, n, c->tabs.initc) == hipSuccess;
  auto cp = [&](void* dst, const void* src, size_t esz) {
    return !dst || hipMemcpyAsync(dst, src, n * esz, hipMemcpyDeviceToHost, c->cur) == hipSuccess;
  };
  ok = ok && cp(h->data_off, d.data_off, 8) && cp(h->len, d.len, 4) && cp(h->stored_crc, d.stored_crc, 4) &&
       cp(h->type, d.type, 1) && cp(h->crc_ok, d.crc_ok, 1);
  ok = ok && hipStreamSynchronize(c->cur) == hipSuccess;
  (void)hipFree(mem);
  return ok ? BCW_OK : BCW_E_HIP;
}

static int ensure_dev_table(bcw_ctx* c, uint64_t cap, bool hint) {
  if (cap <= c->d_tab_cap && c->d_tab_mem) return BCW_OK;
  (void)hipStreamSynchronize(c->cur);
  (void)hipFree(c->d_tab_mem);
  c->d_tab_mem = nullptr;
  const uint64_t n = std::max<uint64_t>(cap, 1);
  const size_t bytes = n * (8 * 5 + 4 * 5 + 4);
  if (hipMalloc(&c->d_tab_mem, bytes) != hipSuccess) { c->d_tab_cap = 0; return BCW_E_NOMEM; }
  uint8_t* m = (uint8_t*)c->d_tab_mem;
  bcw_record_table& t = c->d_tab;
  t.capacity = n;
  t.foff = (uint64_t*)m; m += n * 8;
  t.size = (uint64_t*)m; m += n * 8;
  t.expire = (uint64_t*)m; m += n * 8;
  t.aux0 = (uint64_t*)m; m += n * 8;
  t.aux1 = (uint64_t*)m; m += n * 8;
  t.key_len = (uint32_t*)m; m += n * 4;
  t.val_len = (uint32_t*)m; m += n * 4;
  t.meta_len = (uint32_t*)m; m += n * 4;
  t.first_frag = (uint32_t*)m; m += n * 4;
  t.emit_frag = (uint32_t*)m; m += n * 4;
  t.hdr_size = m; m += n;
  t.flags = m; m += n;
  t.etag_off = m; m += n;
  t.status = m;
  c->d_tab_cap = n;
  (void)hint;
  return BCW_OK;
}

int bcw_decode_segment(bcw_ctx* c, const uint8_t* h_seg, const bcw_decode_params* p,
                       const bcw_record_table* h, bcw_decode_result* h_result) {
  if (!c || !p || !h || !h_result) return BCW_E_INVAL;
  if (p->seg_len && !h_seg) return BCW_E_INVAL;
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  if (p->seg_len > c->d_seg_cap) {
    (void)hipStreamSynchronize(c->cur);
    (void)hipFree(c->d_seg);
    c->d_seg = nullptr;
    c->d_seg_cap = 0;
    if (hipMalloc(&c->d_seg, p->seg_len) != hipSuccess) return BCW_E_NOMEM;
    c->d_seg_cap = p->seg_len;
  }
  if (p->seg_len) HIPCHK(hipMemcpyAsync(c->d_seg, h_seg, p->seg_len, hipMemcpyHostToDevice, c->cur));
  int rc = ensure_dev_table(c, h->capacity, p->mode == BCW_MODE_HINT);
  if (rc != BCW_OK) return rc;
  for (int attempt = 0; attempt < 3; ++attempt) {
    rc = bcw_decode_segment_async(c, c->d_seg, p, &c->d_tab, c->d_result);
    if (rc != BCW_OK) return rc;
    HIPCHK(hipMemcpyAsync(h_result, c->d_result, sizeof *h_result, hipMemcpyDeviceToHost, c->cur));
    HIPCHK(hipStreamSynchronize(c->cur));
    if (!h_result->retry_frag_capacity) break;
    if (bcw_ctx_reserve_fragments(c, h_result->retry_frag_capacity + 64) != BCW_OK) return BCW_E_CAPACITY;
  }
  if (h_result->retry_frag_capacity) return BCW_E_NOMEM;
  const uint64_t n = std::min(h_result->n_records, h->capacity);
  const bcw_record_table& d = c->d_tab;
  auto cp = [&](void* dst, const void* src, size_t esz) -> bool {
    if (!dst || n == 0) return true;
    return hipMemcpyAsync(dst, src, n * esz, hipMemcpyDeviceToHost, c->cur) == hipSuccess;
  };
  bool ok = cp(h->foff, d.foff, 8) && cp(h->size, d.size, 8) && cp(h->expire, d.expire, 8) &&
            cp(h->aux0, d.aux0, 8) && cp(h->aux1, d.aux1, 8) && cp(h->key_len, d.key_len, 4) &&
            cp(h->val_len, d.val_len, 4) && cp(h->meta_len, d.meta_len, 4) && cp(h->first_frag, d.first_frag, 4) &&
            cp(h->emit_frag, d.emit_frag, 4) && cp(h->hdr_size, d.hdr_size, 1) && cp(h->flags, d.flags, 1) &&
            cp(h->etag_off, d.etag_off, 1) && cp(h->status, d.status, 1);
  if (!ok) return BCW_E_HIP;
  HIPCHK(hipStreamSynchronize(c->cur));
  return h_result->n_records > h->capacity ? BCW_E_CAPACITY : BCW_OK;
}


// ---- encode (bcw_encode.hip) ----
static int ensure_enc_scratch(bcw_ctx* c, uint64_t rows) {
  EncScratch& e = c->es;
  if (rows <= e.rows_cap && e.emisc) return BCW_OK;
  (void)hipStreamSynchronize(c->cur);
  const uint64_t r = std::max(std::max(rows, e.rows_cap), (uint64_t)1);
  free_enc_scratch(e);
  const uint64_t ntiles = r / enc_tile_items() + 2;
  const uint64_t nwin = r / enc_ev_win() + 2;
  bool ok = hipMalloc(&e.sz, r * 4) == hipSuccess && hipMalloc(&e.mflag, r) == hipSuccess &&
            hipMalloc(&e.dsrc, r * 4) == hipSuccess && hipMalloc(&e.da, (r + 1) * 8) == hipSuccess &&
            hipMalloc(&e.hda, (r + 1) * 8) == hipSuccess && hipMalloc(&e.hsz, r * 4) == hipSuccess &&
            hipMalloc(&e.dpos, r * 8) == hipSuccess && hipMalloc(&e.hpos, r * 8) == hipSuccess &&
            hipMalloc(&e.tiles, ntiles * enc_sizeof_tile()) == hipSuccess &&
            hipMalloc(&e.ev, (r + 2) * enc_sizeof_ev()) == hipSuccess && hipMalloc(&e.evb, nwin * 4) == hipSuccess &&
            hipMalloc(&e.evt, nwin * 32768 * 8) == hipSuccess && hipMalloc(&e.hnl, r * 2) == hipSuccess &&
            hipMalloc(&e.evw, nwin * 12) == hipSuccess &&
            hipMalloc(&e.recdesc, r * enc_sizeof_recdesc()) == hipSuccess && hipMalloc(&e.wl, r * 4) == hipSuccess &&
            hipMalloc(&e.emisc, 64 * sizeof(uint64_t)) == hipSuccess;
  if (!ok) { free_enc_scratch(e); return BCW_E_NOMEM; }
  if (!e.aux && (hipStreamCreateWithFlags(&e.aux, hipStreamNonBlocking) != hipSuccess ||
                 hipEventCreateWithFlags(&e.ev_scan, hipEventDisableTiming) != hipSuccess ||
                 hipEventCreateWithFlags(&e.ev_hscan, hipEventDisableTiming) != hipSuccess ||
                 hipEventCreateWithFlags(&e.ev_desc, hipEventDisableTiming) != hipSuccess))
    return BCW_E_HIP;
  (void)hipMemsetAsync(e.mflag, 0, r, c->cur);
  e.rows_cap = r;
  return BCW_OK;
}

int bcw_encode_segment_async(bcw_ctx* c, const uint8_t* d_src, const bcw_encode_params* p,
                             const bcw_record_table* t, const bcw_decode_result* d_src_result, const uint8_t* d_keep,
                             const bcw_encode_out* o, bcw_encode_result* d_result) {
  if (!c || !p || !t || !d_src_result || !o || !d_result) return BCW_E_INVAL;
  if (p->mode != BCW_ENC_COMPACT && p->mode != BCW_ENC_HINT) return BCW_E_INVAL;
  if (p->hint_pos < BCW_SUPER_BLOCK_SIZE || !o->hint) return BCW_E_INVAL;
  if (p->mode == BCW_ENC_COMPACT && (p->wal_pos < BCW_SUPER_BLOCK_SIZE || !o->wal || !d_keep)) return BCW_E_INVAL;
  if (!t->foff || !t->size || !t->expire || !t->key_len || !t->val_len || !t->meta_len || !t->first_frag ||
      !t->emit_frag || !t->hdr_size || !t->flags || !t->etag_off || !t->status)
    return BCW_E_INVAL;
  if (!c->s.frags) return BCW_E_INVAL;  // no decode on this context yet
  if (t->capacity >= 0xffffff00ull) return BCW_E_INVAL;  // u32 dense record ids
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  int rc = ensure_enc_scratch(c, t->capacity);
  if (rc != BCW_OK) return rc;
  EncLaunch L{};
  L.d_src = d_src;
  L.p = *p;
  L.table = *t;
  L.rows = t->capacity;
  L.d_src_result = d_src_result;
  L.d_keep = d_keep;
  L.out = *o;
  L.d_result = d_result;
  L.frags = c->s.frags;
  L.crc_ops = c->tabs.enc_ops;
  L.initc = c->tabs.initc;
  L.num_cus = c->num_cus;
  L.gen = c->frag_gen;
  return launch_encode(L, c->es, c->cur, &c->prof) == hipSuccess ? BCW_OK : BCW_E_HIP;
}

}  // extern "C"

namespace bcw {
// Sync-API staging: the source segment into the context's device buffer, decoded into the context's
// device table (grown until it holds every record), the fragment scratch retried until it fits.
int sync_decode(bcw_ctx* c, const uint8_t* h_src, const bcw_decode_params& dp, bcw_decode_result& dres) {
  uint64_t cap = std::max<uint64_t>(16, dp.seg_len / 64 + 16);
  if (dp.seg_len > c->d_seg_cap) {
    (void)hipStreamSynchronize(c->cur);
    (void)hipFree(c->d_seg);
    c->d_seg = nullptr;
    c->d_seg_cap = 0;
    if (hipMalloc(&c->d_seg, dp.seg_len) != hipSuccess) return BCW_E_NOMEM;
    c->d_seg_cap = dp.seg_len;
  }
  if (dp.seg_len) HIPCHK(hipMemcpyAsync(c->d_seg, h_src, dp.seg_len, hipMemcpyHostToDevice, c->cur));
  for (;;) {
    int rc = ensure_dev_table(c, cap, dp.mode == BCW_MODE_HINT);
    if (rc != BCW_OK) return rc;
    for (int attempt = 0; attempt < 3; ++attempt) {
      rc = bcw_decode_segment_async(c, c->d_seg, &dp, &c->d_tab, c->d_result);
      if (rc != BCW_OK) return rc;
      HIPCHK(hipMemcpyAsync(&dres, c->d_result, sizeof dres, hipMemcpyDeviceToHost, c->cur));
      HIPCHK(hipStreamSynchronize(c->cur));
      if (!dres.retry_frag_capacity) break;
      if (bcw_ctx_reserve_fragments(c, dres.retry_frag_capacity + 64) != BCW_OK) return BCW_E_CAPACITY;
    }
    if (dres.retry_frag_capacity) return BCW_E_NOMEM;
    if (dres.n_records <= c->d_tab.capacity) return BCW_OK;
    cap = dres.n_records + 16;
  }
}

int ensure_keep(bcw_ctx* c, uint64_t rows) {
  if (rows <= c->d_keep_cap && c->d_keep) return BCW_OK;
  (void)hipStreamSynchronize(c->cur);
  (void)hipFree(c->d_keep);
  c->d_keep = nullptr;
  c->d_keep_cap = 0;
  if (hipMalloc(&c->d_keep, std::max<uint64_t>(rows, 1)) != hipSuccess) return BCW_E_NOMEM;
  c->d_keep_cap = std::max<uint64_t>(rows, 1);
  return BCW_OK;
}

bcw_decode_params src_params(const uint8_t* h_src, const bcw_encode_params* p) {
  bcw_super_block sb{};
  bcw_decode_params dp{};
  dp.seg_len = p->src_len;
  dp.start_off = p->src_start_off;
  dp.ns_size = p->ns_size;
  dp.etag_size = p->etag_size;
  dp.mode = BCW_MODE_RECORD;
  dp.base_time = (bcw_load_super_block(h_src, p->src_len, &sb) == BCW_SB_OK) ? sb.base_time : 0;
  return dp;
}

// the encode of the context's decoded source with the context's keep mask, outputs copied to the host
int encode_run(bcw_ctx* c, const bcw_encode_params* p, const bcw_encode_out* h, bcw_encode_result* h_result,
               bcw_encode_out* d_out) {
  const uint64_t rows = c->d_tab.capacity;
  const uint64_t need = h->wal_cap + h->hint_cap + rows * 8;
  if (need > c->d_eout_cap) {
    (void)hipStreamSynchronize(c->cur);
    (void)hipFree(c->d_eout);
    c->d_eout = nullptr;
    c->d_eout_cap = 0;
    if (hipMalloc(&c->d_eout, need + 64) != hipSuccess) return BCW_E_NOMEM;
    c->d_eout_cap = need;
  }
  uint8_t* m = (uint8_t*)c->d_eout;
  bcw_encode_out& d = *d_out;
  d = bcw_encode_out{};
  d.rec_off = (uint64_t*)m;
  d.rec_off_cap = rows;
  m += rows * 8;
  d.wal = m;
  d.wal_cap = h->wal_cap;
  m += (h->wal_cap + 15) & ~15ull;
  d.hint = (uint8_t*)(((uintptr_t)m + 15) & ~(uintptr_t)15);
  d.hint_cap = h->hint_cap;
  if (p->mode == BCW_ENC_HINT && !d.wal) d.wal = d.hint;
  int rc = bcw_encode_segment_async(c, c->d_seg, p, &c->d_tab, c->d_result, c->d_keep, &d, c->d_eres);
  if (rc != BCW_OK) return rc;
  HIPCHK(hipMemcpyAsync(h_result, c->d_eres, sizeof *h_result, hipMemcpyDeviceToHost, c->cur));
  HIPCHK(hipStreamSynchronize(c->cur));
  if (!h_result->fits) return BCW_E_CAPACITY;
  if (h->rec_off && h->rec_off_cap < h_result->n_in) return BCW_E_CAPACITY;
  return BCW_OK;
}

int encode_copy_out(bcw_ctx* c, const bcw_encode_params* p, const bcw_encode_out* h, const bcw_encode_result& r,
                    const bcw_encode_out& d, const bcw_decode_result& dres) {
  if (h->wal && r.wal_need && p->mode == BCW_ENC_COMPACT)
    HIPCHK(hipMemcpyAsync(h->wal, d.wal, r.wal_need, hipMemcpyDeviceToHost, c->cur));
  if (h->hint && r.hint_need) HIPCHK(hipMemcpyAsync(h->hint, d.hint, r.hint_need, hipMemcpyDeviceToHost, c->cur));
  // rows >= n_in are never written (UINT64_MAX): copy only rows the encode can have written
  const uint64_t nr = std::min(r.n_in, d.rec_off_cap);
  if (h->rec_off && nr) HIPCHK(hipMemcpyAsync(h->rec_off, d.rec_off, nr * 8, hipMemcpyDeviceToHost, c->cur));
  HIPCHK(hipStreamSynchronize(c->cur));
  if (h->rec_off)
    for (uint64_t i = nr; i < h->rec_off_cap && i < dres.n_records; ++i) h->rec_off[i] = ~0ull;
  return BCW_OK;
}

int encode_to_host(bcw_ctx* c, const bcw_encode_params* p, const bcw_encode_out* h, bcw_encode_result* h_result,
                   const bcw_decode_result& dres) {
  bcw_encode_out d{};
  const int rc = encode_run(c, p, h, h_result, &d);
  return rc != BCW_OK ? rc : encode_copy_out(c, p, h, *h_result, d, dres);
}
}  // namespace bcw

extern "C" {

int bcw_encode_segment(bcw_ctx* c, const uint8_t* h_src, const bcw_encode_params* p, const uint8_t* h_keep,
                       uint64_t n_keep, const bcw_encode_out* h, bcw_encode_result* h_result) {
  if (!c || !p || !h || !h_result) return BCW_E_INVAL;
  if (p->src_len && !h_src) return BCW_E_INVAL;
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  const bcw_decode_params dp = src_params(h_src, p);
  bcw_decode_result dres{};
  int rc = sync_decode(c, h_src, dp, dres);
  if (rc != BCW_OK) return rc;
  const uint64_t rows = c->d_tab.capacity;
  rc = ensure_keep(c, rows);  // keep mask (missing entries: dropped)
  if (rc != BCW_OK) return rc;
  HIPCHK(hipMemsetAsync(c->d_keep, 0, rows, c->cur));
  const uint64_t nk = std::min(n_keep, rows);
  if (h_keep && nk) HIPCHK(hipMemcpyAsync(c->d_keep, h_keep, nk, hipMemcpyHostToDevice, c->cur));
  return encode_to_host(c, p, h, h_result, dres);
}

int bcw_compact_segment(bcw_ctx* c, bcw_index* ix, const uint8_t* h_src, const bcw_encode_params* p, uint64_t src_fid,
                        const bcw_encode_out* h, bcw_encode_result* h_result, bcw_index_result* h_filter) {
  if (!c || !ix || !p || !h || !h_result || p->mode != BCW_ENC_COMPACT) return BCW_E_INVAL;
  if (index_ctx(ix) != c) return BCW_E_INVAL;  // the filter runs on the index's context (stream, fragment table)
  if (p->src_len && !h_src) return BCW_E_INVAL;
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  const bcw_decode_params dp = src_params(h_src, p);
  bcw_decode_result dres{};
  int rc = sync_decode(c, h_src, dp, dres);
  if (rc != BCW_OK) return rc;
  rc = ensure_keep(c, c->d_tab.capacity);
  if (rc != BCW_OK) return rc;
  rc = bcw_compact_filter_async(ix, c->d_seg, &dp, &c->d_tab, c->d_result, src_fid, c->d_keep,
                                h_filter ? c->d_ires : nullptr);
  if (rc != BCW_OK) return rc;
  if (h_filter) HIPCHK(hipMemcpyAsync(h_filter, c->d_ires, sizeof *h_filter, hipMemcpyDeviceToHost, c->cur));
  return encode_to_host(c, p, h, h_result, dres);
}

int bcw_index_recover_segment(bcw_ctx* c, bcw_index* ix, const uint8_t* h_seg, const bcw_decode_params* p,
                              uint64_t fid, int use_record_fid, bcw_decode_result* h_dres,
                              bcw_index_result* h_out) {
  if (!c || !ix || !p || !h_out) return BCW_E_INVAL;
  if (index_ctx(ix) != c) return BCW_E_INVAL;  // the puts run on the index's context (stream, fragment table)
  if (p->seg_len && !h_seg) return BCW_E_INVAL;
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  bcw_decode_result dres{};
  int rc = sync_decode(c, h_seg, *p, dres);
  if (rc != BCW_OK) return rc;
  if (h_dres) *h_dres = dres;
  rc = bcw_index_put_decoded_async(ix, c->d_seg, p, &c->d_tab, c->d_result, fid, use_record_fid, c->d_ires);
  if (rc != BCW_OK) return rc;
  HIPCHK(hipMemcpyAsync(h_out, c->d_ires, sizeof *h_out, hipMemcpyDeviceToHost, c->cur));
  HIPCHK(hipStreamSynchronize(c->cur));
  return BCW_OK;
}

// ---- host WAL writer: Record.Encode (record.go:57-138) at synthetic shapes + WriteRecord ----
namespace {
struct Writer {
  uint8_t* out;
  uint64_t cap;
  uint64_t len;
  void put(const void* p, uint64_t n) {
    if (out && len + n <= cap) memcpy(out + len, p, n);
    len += n;
  }
  // wal.go:490-553 (writeOffset(true) = len - 40); returns the record offset
  uint64_t write_record(const uint8_t* rec, uint64_t n, bool compute_crc) {
    static const uint8_t pad[6] = {0, 0, 0, 0, 0, 0};
    uint64_t offset = 0, left = n;
    bool begin = true;
    while (left > 0) {
      uint64_t leftover = BCW_BLOCK_SIZE - ((len - BCW_SUPER_BLOCK_SIZE) % BCW_BLOCK_SIZE);
      if (leftover < BCW_HEADER_SIZE) {
        put(pad, leftover);
        leftover = BCW_BLOCK_SIZE;
      }
      if (begin) offset = len;
      const uint64_t avail = leftover - BCW_HEADER_SIZE;
      const uint64_t frag = std::min(left, avail);
      const bool end = left == frag;
      const uint8_t type = (begin && end) ? BCW_RECORD_FULL : begin ? BCW_RECORD_FIRST : end ? BCW_RECORD_LAST
                                                                                          : BCW_RECORD_MIDDLE;
      uint8_t hdr[7];
      const uint32_t crc = compute_crc ? mask_crc(crc32c_hw(rec, frag)) : 0;
      const uint16_t l16 = (uint16_t)frag;
      memcpy(hdr, &crc, 4);
      memcpy(hdr + 4, &l16, 2);
      hdr[6] = type;
      put(hdr, 7);
      put(rec, frag);
      rec += frag;
      left -= frag;
      begin = false;
    }
    return offset;
  }
};

inline uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline void fill_rand(uint64_t& s, uint8_t* p, size_t n) {
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    const uint64_t v = splitmix64(s);
    memcpy(p + i, &v, 8);
  }
  if (i < n) {
    const uint64_t v = splitmix64(s);
    memcpy(p + i, &v, n - i);
  }
}
inline int put_uvarint(uint8_t* o, uint64_t v) {
  int i = 0;
  while (v >= 0x80) { o[i++] = (uint8_t)(v | 0x80); v >>= 7; }
  o[i++] = (uint8_t)v;
  return i;
}
}  // namespace

int bcw_synth_segment(uint64_t target_bytes, uint64_t max_records, uint64_t seed, uint32_t ns_size,
                      uint32_t key_len, uint32_t value_len, int value_mode, uint64_t base_time, uint8_t* h_out,
                      uint64_t out_cap, uint64_t* out_len, uint64_t* out_records) {
  if (value_mode != 0 && value_mode != 1) return BCW_E_INVAL;
  if (ns_size > 255 || key_len > (1u << 20) || value_len > (1u << 26)) return BCW_E_INVAL;
  Writer w0{h_out, out_cap, 0};
  uint8_t sb[40];
  bcw_write_super_block(sb, base_time, base_time);
  w0.put(sb, 40);
  std::vector<double> cdf;
  if (value_mode == 1) {
    cdf.resize(512);
    double acc = 0;
    for (int k = 1; k <= 512; ++k) { acc += std::pow((double)k, -1.1); cdf[k - 1] = acc; }
    for (auto& x : cdf) x /= acc;
  }
  const size_t vmax = value_mode == 1 ? 128 * 512 : value_len;
  std::vector<uint8_t> ns(ns_size);
  for (uint32_t i = 0; i < ns_size; ++i) ns[i] = (uint8_t)('A' + i % 26);
  struct Bufs {
    std::vector<uint8_t> key, val, rec;
  };
  // record i at the writer's position, with the random stream at s (advanced past the record)
  auto one = [&](uint64_t i, uint64_t& s, Writer& w, bool fill, Bufs& B) {
    size_t vl = value_len;
    if (value_mode == 1) {
      const double u = (double)(splitmix64(s) >> 11) * (1.0 / 9007199254740992.0);
      vl = 128u * (size_t)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin() + 1);
    }
    if (fill) {
      fill_rand(s, B.key.data(), key_len);
      if (key_len >= 8) memcpy(B.key.data(), &i, 8);
      fill_rand(s, B.val.data(), vl);
    } else {
      s += 0x9E3779B97F4A7C15ull * (uint64_t)(((key_len + 7) / 8) + ((vl + 7) / 8));
    }
    // Record.Encode with no etag, no expire, no meta (record.go:57-138)
    uint8_t tmp[30];
    int t = 0;
    t += put_uvarint(tmp + t, key_len);
    t += put_uvarint(tmp + t, vl);
    t += put_uvarint(tmp + t, 0);
    const size_t header = (size_t)t + ns_size + 2;
    const size_t n = header + key_len + vl;
    if (!fill) {  // the layout only (w has no output buffer: nothing is read from the record)
      w.write_record(B.rec.data(), n, false);
      return;
    }
    uint8_t* r = B.rec.data();
    size_t o = 0;
    r[o++] = (uint8_t)header;
    memcpy(r + o, ns.data(), ns_size); o += ns_size;
    r[o++] = (uint8_t)((1u << 0) | (1u << 1));  // noEtag | noExpire
    memcpy(r + o, tmp, t); o += t;
    memcpy(r + o, B.key.data(), key_len); o += key_len;
    memcpy(r + o, B.val.data(), vl); o += vl;
    w.write_record(r, o, true);
  };
  auto bufs = [&]() {
    Bufs B;
    B.key.resize(key_len + 8);
    B.val.resize(vmax + 8);
    B.rec.resize(vmax + key_len + ns_size + 64);
    return B;
  };
  // pass 1: the layout (and the random stream's state) at every kCk-th record; pass 2 fills the records in
  // parallel from those checkpoints -- the same bytes as one sequential pass (a 42 GB config-E segment: one
  // thread took about a minute)
  constexpr uint64_t kCk = 4096;
  struct Ck {
    uint64_t i, s, len;
  };
  std::vector<Ck> ck;
  Writer wl{nullptr, 0, w0.len};
  uint64_t s = seed, n = 0;
  Bufs B0 = bufs();
  for (uint64_t i = 0; (max_records == 0 || i < max_records) && wl.len < target_bytes; ++i) {
    if (i % kCk == 0) ck.push_back(Ck{i, s, wl.len});
    one(i, s, wl, false, B0);
    ++n;
  }
  if (out_len) *out_len = wl.len;
  if (out_records) *out_records = n;
  if (!h_out) return BCW_OK;
  if (wl.len > out_cap) return BCW_E_CAPACITY;
  const unsigned hw = std::thread::hardware_concurrency();
  const uint64_t nth = std::max<uint64_t>(1, std::min<uint64_t>({(uint64_t)(hw ? hw : 1), 16, ck.size()}));
  std::atomic<uint64_t> next{0};
  auto fill = [&]() {
    Bufs B = bufs();
    for (uint64_t c; (c = next.fetch_add(1)) < ck.size();) {
      Writer w{h_out, out_cap, ck[c].len};
      uint64_t st = ck[c].s;
      const uint64_t i1 = std::min<uint64_t>(ck[c].i + kCk, n);
      for (uint64_t i = ck[c].i; i < i1; ++i) one(i, st, w, true, B);
    }
  };
  std::vector<std::thread> pool;
  for (uint64_t t = 1; t < nth; ++t) pool.emplace_back(fill);
  fill();
  for (auto& t : pool) t.join();
  return BCW_OK;
}

}  // extern "C"
