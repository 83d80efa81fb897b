// bcw_decode.hip -- MI355X (gfx950) kernels for bitcaskDB WAL segment decode + CRC verify.
//
// Pipeline (one HIP stream, no host synchronisation inside; DESIGN.md "decode pipeline"):
//   k_chase(count)   one lane per 32 KiB block: header chase        wal_iterator.go:45-77
//   k_scan_u32       exclusive scan of fragments per block -> global fragment index
//   k_chase(write)   second chase (headers now cache-resident): compact fragment table
//   k_crc            per-fragment masked CRC-32C verify as a zero test  wal_iterator.go:79 /
//                    utils.go:24-29 (LDS slice-by-2 tables, 128 B window per lane, lane
//                    shift operators + segmented XOR scan across lanes)
//   k_blocksum       per-block transform of the iterator's record state machine wal_iterator.go:69-96
//   k_blockscan      composes the block transforms (one workgroup): record bases, first error
//   k_records        record emission + RecordFromBytes / HintRecord.Decode   record.go:140-239,
//                    hint.go:50-84, one wave per block
//   k_finalize       bcw_decode_result
#include <hip/hip_runtime.h>

#include <cstdint>

#include "bcw_internal.h"

namespace bcw {

// ------------------------------------------------------------------------------------------
// misc counters (Scratch::misc)
enum { M_FIRST_BAD = 0, M_NREC = 1, M_ERR_FRAG = 2, M_ERR_CLASS = 3, M_NFRAGS = 4 };

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// 7-byte fragment header at seg[off..off+7) (off + 7 <= seg_len guaranteed by the caller)
__device__ __forceinline__ void read_header(const uint8_t* __restrict__ seg, uint64_t seg_len, uint64_t off,
                                            uint32_t& crc, uint32_t& len, uint32_t& type) {
  const uint64_t a = off & ~3ull;
  uint32_t w0, w1, w2;
  if (a + 12 <= seg_len) {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(seg + a);
    w0 = q[0]; w1 = q[1]; w2 = q[2];
  } else {
    uint32_t b[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) b[i] = (a + i < seg_len) ? seg[a + i] : 0u;
    w0 = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
    w1 = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
    w2 = b[8] | b[9] << 8 | b[10] << 16 | b[11] << 24;
  }
  const uint32_t sh = (uint32_t)(off & 3);
  crc = __builtin_amdgcn_alignbyte(w1, w0, sh);
  const uint32_t t = __builtin_amdgcn_alignbyte(w2, w1, sh);
  len = t & 0xffffu;
  type = (t >> 16) & 0xffu;
}

// ------------------------------------------------------------------------------------------
// k_chase: WalIterator refill + header chase of one block (wal_iterator.go:45-77). The block's
// buffer is min(32768, Size - fileOff) bytes; a header is parsed while bufOff + 7 <= bufSize;
// the data length is clamped to the buffer. Pass 0 counts, pass 1 writes the compact table.
__global__ __launch_bounds__(256) void k_chase(const uint8_t* __restrict__ seg, uint64_t seg_len,
                                               uint32_t start_off, uint64_t nblocks, uint32_t* __restrict__ nfrag,
                                               const uint32_t* __restrict__ fbase, Frag* __restrict__ frags,
                                               uint64_t frag_cap, int write) {
  const uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const uint64_t boff = (uint64_t)start_off + b * kBlock;
  const uint32_t bufsize = (uint32_t)((seg_len - boff) < kBlock ? (seg_len - boff) : kBlock);
  uint32_t h = 0, n = 0;
  const uint64_t g0 = write ? fbase[b] : 0;
  while (h + kHdr <= bufsize) {
    uint32_t crc, len, type;
    read_header(seg, seg_len, boff + h, crc, len, type);
    const uint32_t start = h + kHdr;
    if (len > bufsize - start) len = bufsize - start;
    if (write && g0 + n < frag_cap) {
      Frag f;
      f.blk = (uint32_t)b;
      f.start = (uint16_t)start;
      f.len = (uint16_t)len;
      f.crc = crc;
      f.type = (uint8_t)type;
      f.ok = 0;
      f.pad = 0;
      frags[g0 + n] = f;
    }
    h = start + len;
    ++n;
  }
  if (!write) nfrag[b] = n;
}

// ------------------------------------------------------------------------------------------
// exclusive scan of a u32 array (one workgroup of 1024 threads); out[n] = total (saturated).
__global__ __launch_bounds__(1024) void k_scan_u32(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                   uint64_t n, uint64_t* __restrict__ total) {
  __shared__ uint64_t sm[1024];
  const uint32_t t = threadIdx.x;
  const uint64_t per = (n + 1023) / 1024;
  const uint64_t lo = t * per;
  const uint64_t hi = lo + per < n ? lo + per : n;
  uint64_t s = 0;
  for (uint64_t i = lo; i < hi; ++i) s += in[i];
  sm[t] = s;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    const uint64_t v = t >= d ? sm[t - d] : 0;
    __syncthreads();
    sm[t] += v;
    __syncthreads();
  }
  uint64_t run = sm[t] - s;
  for (uint64_t i = lo; i < hi; ++i) {
    out[i] = (uint32_t)(run < 0xffffffffull ? run : 0xffffffffull);
    run += in[i];
  }
  if (t == 1023) {
    const uint64_t tot = sm[1023];
    out[n] = (uint32_t)(tot < 0xffffffffull ? tot : 0xffffffffull);
    *total = tot;
  }
}

// ------------------------------------------------------------------------------------------
// k_crc: per-fragment CRC verify.
//
// For fragment f with data [s, e) (block-relative) let E = 4*ceil(e/4) + 4 and tile [E-128C, E)
// with C = ceil((E - s)/128) windows of 128 B. A raw (init 0) CRC-32C chain over the windows,
// with the bytes before s zeroed and the bytes [e, e+4) replaced by
//     J = ~unmask(stored) ^ A_{8L}(0xFFFFFFFF)          (L = e - s)
// and zeros after, ends in state 0 exactly when ComputeCRC32(data) == stored (linearity of CRC:
// the init 0xFFFFFFFF contributes A_{8L}(~0) at e, the XOR-out is folded into ~unmask). So the
// CRC check becomes a zero test of a linear functional, and windows can be computed by separate
// lanes and combined with fixed shift operators:
//   * head pass: lane i processes the first window of fragment i (prefix masking); if C == 1 it
//     also holds the J word and tests zero directly, otherwise its end state seeds the second
//     window's chain.
//   * body passes: the remaining windows of consecutive fragments, one per lane, consecutive
//     windows of a fragment on consecutive lanes. Lane l maps its end state into a common frame
//     with F_l = A_{8*128*(63-l)} (lane-replicated nibble tables), a segmented XOR scan combines
//     the fragment's windows, and the lane holding the last window tests the total for zero.
//     A fragment continuing past lane 63 carries its value to the next pass (shift A_{8*8192}).
constexpr int kCrcWaves = 16;
constexpr int kLdsSlice = 2 * 256 * 32;  // dwords, slice-by-2 tables replicated x32 (64 KiB)
constexpr int kLdsFwd = 8 * 16 * 64;     // dwords, lane operators (32 KiB)
constexpr int kLdsCarry = 8 * 16;        // dwords
constexpr int kSlots = 128;              // fragment slots per wave (two windows of 64)
constexpr int kSlotWords = 5;            // cpre, blk, se, J, V1
constexpr size_t kCrcLds = (size_t)(kLdsSlice + kLdsFwd + kLdsCarry + kCrcWaves * kSlots * kSlotWords) * 4;

__device__ __forceinline__ uint32_t lds_tab(const uint32_t* __restrict__ t, uint32_t idx) { return t[idx]; }

// slice-by-2 step on the low 16 bits of h: T0 = byte table, T1 = one byte further
__device__ __forceinline__ uint32_t step16(const uint32_t* __restrict__ tab, uint32_t lo, uint32_t s, uint32_t h) {
  const uint32_t x = s ^ h;
  const uint32_t a = tab[((256u + (x & 0xffu)) << 5) | lo];
  const uint32_t b = tab[((((x >> 8) & 0xffu)) << 5) | lo];
  return (s >> 16) ^ a ^ b;
}
__device__ __forceinline__ uint32_t step32(const uint32_t* __restrict__ tab, uint32_t lo, uint32_t s, uint32_t w) {
  s = step16(tab, lo, s, w & 0xffffu);
  return step16(tab, lo, s, w >> 16);
}
// advance by one byte
__device__ __forceinline__ uint32_t step8(const uint32_t* __restrict__ tab, uint32_t lo, uint32_t s, uint32_t b) {
  return (s >> 8) ^ tab[(((s ^ b) & 0xffu)) << 5 | lo];
}
// F_l(x): lane-replicated nibble images, lane l reads its own copy (bank = l % 32)
__device__ __forceinline__ uint32_t apply_fwd(const uint32_t* __restrict__ fwd, uint32_t lane, uint32_t x) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= fwd[((i * 16 + ((x >> (4 * i)) & 15u)) << 6) | lane];
  return r;
}
__device__ __forceinline__ uint32_t apply_carry(const uint32_t* __restrict__ c, uint32_t x) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= c[i * 16 + ((x >> (4 * i)) & 15u)];
  return r;
}

// 16 bytes at seg[o..o+16), zero outside [0, seg_len)
__device__ __forceinline__ uint4 load16(const uint8_t* __restrict__ seg, uint64_t seg_len, int64_t o) {
  if (o >= 0 && (uint64_t)o + 16 <= seg_len) return *reinterpret_cast<const uint4*>(seg + o);
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t p = o + 4 * k + i;
      const uint32_t byte = (p >= 0 && (uint64_t)p < seg_len) ? seg[p] : 0u;
      v |= byte << (8 * i);
    }
    w[k] = v;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void load_window(const uint8_t* __restrict__ seg, uint64_t seg_len, int64_t goff,
                                            uint32_t (&w)[32]) {
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const uint4 v = load16(seg, seg_len, goff + 16 * g);
    w[4 * g + 0] = v.x; w[4 * g + 1] = v.y; w[4 * g + 2] = v.z; w[4 * g + 3] = v.w;
  }
}

// last-window fix: keep bytes < hi of words 30/31, put J at [hi, hi+4), zero the rest.
__device__ __forceinline__ void fix_last(uint32_t (&w)[32], uint32_t hi, uint32_t J) {
  const uint32_t r = hi - 120u;  // 1..4
  uint64_t d = (uint64_t)w[30] | ((uint64_t)w[31] << 32);
  const uint64_t keep = (1ull << (8 * r)) - 1ull;
  d = (d & keep) | ((uint64_t)J << (8 * r));
  w[30] = (uint32_t)d;
  w[31] = (uint32_t)(d >> 32);
}

__device__ __forceinline__ uint32_t wave_incl_scan_add(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += t;
  }
  return v;
}

__global__ __launch_bounds__(1024) void k_crc(const uint8_t* __restrict__ seg, uint64_t seg_len, uint32_t start_off,
                                              uint64_t nblocks, const uint32_t* __restrict__ fbase,
                                              Frag* __restrict__ frags, uint64_t frag_cap, Tables tabs) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* s_slice = lds;
  uint32_t* s_fwd = lds + kLdsSlice;
  uint32_t* s_carry = s_fwd + kLdsFwd;
  uint32_t* s_slots_all = s_carry + kLdsCarry;
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < (uint32_t)kLdsSlice; i += 1024) s_slice[i] = tabs.slice[i >> 5];
  for (uint32_t i = tid; i < (uint32_t)kLdsFwd; i += 1024) s_fwd[i] = tabs.fwd[(i & 63u) * 128u + (i >> 6)];
  if (tid < (uint32_t)kLdsCarry) s_carry[tid] = tabs.carry[tid];
  __syncthreads();

  const uint32_t lane = tid & 63u;
  const uint32_t lo = lane & 31u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint32_t* s_cpre = s_slots_all + wave * kSlots * kSlotWords;
  uint32_t* s_blk = s_cpre + kSlots;
  uint32_t* s_se = s_blk + kSlots;
  uint32_t* s_J = s_se + kSlots;
  uint32_t* s_V1 = s_J + kSlots;

  const uint64_t nw = (uint64_t)gridDim.x * kCrcWaves;
  const uint64_t gw = (uint64_t)blockIdx.x * kCrcWaves + wave;
  const uint64_t b0 = nblocks * gw / nw, b1 = nblocks * (gw + 1) / nw;
  const uint64_t f0 = fbase[b0];
  uint64_t f1 = fbase[b1];
  if (f1 > frag_cap) f1 = frag_cap;
  if (f0 >= f1) return;
  const uint32_t nfr = (uint32_t)(f1 - f0);
  const uint32_t nwin = (nfr + 63u) / 64u;

  // load fragment window k (64 fragments) into slot half (k & 1); run its head pass.
  // returns the exclusive body-chunk prefix after the window.
  auto load_win = [&](uint32_t k, uint32_t cbase) -> uint32_t {
    const uint32_t half = (k & 1u) * 64u;
    const uint32_t fi = k * 64u + lane;
    uint32_t cb = 0, s = 0, e = 0, E = 0, J = 0, blk = 0, C = 1;
    const bool valid = fi < nfr;
    Frag f;
    if (valid) {
      f = frags[f0 + fi];
      s = f.start;
      e = (uint32_t)f.start + f.len;
      E = ((e + 3u) & ~3u) + 4u;
      C = (E - s + 127u) >> 7;
      cb = C - 1u;
      const uint32_t crc = rotl32(f.crc - 0xa282ead8u, 15);
      J = ~crc ^ tabs.initc[f.len];
      blk = f.blk;
    }
    const uint32_t incl = wave_incl_scan_add(cb, lane);
    const uint32_t tot = __shfl(incl, 63, 64);
    s_cpre[half + lane] = valid ? cbase + incl - cb : 0xffffffffu;
    s_blk[half + lane] = blk;
    s_se[half + lane] = s | (e << 16);
    s_J[half + lane] = J;
    // head pass: first window [E - 128C, E - 128C + 128)
    uint32_t V = 0;
    if (valid) {
      const int64_t wst = (int64_t)E - 128 * (int64_t)C;
      const int64_t goff = (int64_t)start_off + (int64_t)blk * kBlock + wst;
      uint32_t w[32];
      load_window(seg, seg_len, goff, w);
      const int32_t lo8 = 8 * (int32_t)((int64_t)s - wst);  // 8 * lo, lo in [0,128)
#pragma unroll
      for (int k2 = 0; k2 < 32; ++k2) {
        int32_t sh = lo8 - 32 * k2;
        sh = sh < 0 ? 0 : (sh > 32 ? 32 : sh);
        const uint32_t m = (uint32_t)(0xffffffffffffffffull << sh);
        w[k2] &= m;
      }
      if (C == 1u) fix_last(w, (uint32_t)((int64_t)e - wst), J);
      uint32_t S = 0;
#pragma unroll
      for (int k2 = 0; k2 < 32; ++k2) S = step32(s_slice, lo, S, w[k2]);
      V = S;
      if (C == 1u) frags[f0 + fi].ok = (S == 0u) ? 1 : 0;
    }
    s_V1[half + lane] = V;
    return cbase + tot;
  };

  uint32_t kA = 0;
  uint32_t cA_end = load_win(0, 0);
  uint32_t cB_end = nwin > 1 ? load_win(1, cA_end) : cA_end;
  if (nwin <= 1) {
    s_cpre[64 + lane] = 0xffffffffu;
  }
  uint32_t carry = 0;
  for (uint32_t pass = 0;; pass += 64u) {
    while (cA_end <= pass && kA + 1u < nwin) {
      ++kA;
      cA_end = cB_end;
      if (kA + 1u < nwin) cB_end = load_win(kA + 1u, cB_end);
      else s_cpre[((kA + 1u) & 1u) * 64u + lane] = 0xffffffffu;
    }
    if (pass >= cB_end) break;
    const uint32_t j = pass + lane;
    const bool active = j < cB_end;
    const uint32_t hA = (kA & 1u) * 64u, hB = 64u - hA;
    // largest virtual index i in [0,128) with cpre(i) <= j (window A first, then B)
    uint32_t i = 0;
#pragma unroll
    for (uint32_t st = 64; st >= 1; st >>= 1) {
      const uint32_t c = i + st;
      if (c < 128u) {
        const uint32_t slot = c < 64u ? hA + c : hB + (c - 64u);
        if (s_cpre[slot] <= j) i = c;
      }
    }
    const uint32_t slot = i < 64u ? hA + i : hB + (i - 64u);
    uint32_t v = 0, cfb = 0;
    bool is_last = false;
    if (active) {
      const uint32_t cpre = s_cpre[slot];
      const uint32_t se = s_se[slot];
      const uint32_t s = se & 0xffffu, e = se >> 16;
      const uint32_t E = ((e + 3u) & ~3u) + 4u;
      const uint32_t C = (E - s + 127u) >> 7;
      cfb = j - cpre;                 // index among body windows, from the first
      const uint32_t c = C - 2u - cfb; // windows from the end (0 = last)
      is_last = (c == 0u);
      const int64_t wst = (int64_t)E - 128 * (int64_t)(c + 1u);
      const int64_t goff = (int64_t)start_off + (int64_t)s_blk[slot] * kBlock + wst;
      uint32_t w[32];
      load_window(seg, seg_len, goff, w);
      if (is_last) fix_last(w, (uint32_t)((int64_t)e - wst), s_J[slot]);
      uint32_t S = cfb == 0u ? s_V1[slot] : 0u;
#pragma unroll
      for (int k2 = 0; k2 < 32; ++k2) S = step32(s_slice, lo, S, w[k2]);
      v = apply_fwd(s_fwd, lane, S);
      if (lane == 0 && cfb > 0u) v ^= apply_carry(s_carry, carry);
    }
    // segmented inclusive XOR scan: a lane's segment starts at lane - cfb (clamped to 0)
    const uint32_t seg_start = active ? (cfb > lane ? 0u : lane - cfb) : lane;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t t = __shfl_up(v, d, 64);
      if (lane >= (uint32_t)d && lane - (uint32_t)d >= seg_start) v ^= t;
    }
    if (active && is_last) frags[f0 + (uint64_t)kA * 64u + i].ok = (v == 0u) ? 1 : 0;
    carry = __shfl(v, 63, 64);
  }
}

// ------------------------------------------------------------------------------------------
// k_blocksum: the iterator's record state machine (wal_iterator.go:69-96) summarised per block.
__global__ __launch_bounds__(256) void k_blocksum(const Frag* __restrict__ frags, const uint32_t* __restrict__ fbase,
                                                  uint64_t nblocks, uint32_t start_off, uint64_t frag_cap,
                                                  BlockSum* __restrict__ sums) {
  const uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  uint64_t g0 = fbase[b], g1 = fbase[b + 1];
  if (g1 > frag_cap) g1 = frag_cap;
  if (g0 > g1) g0 = g1;
  BlockSum S{};
  S.err_frag = 0xffffffffu;
  bool in_pre = true;
  uint64_t acc = 0, off = 0;
  uint32_t first = 0;
  for (uint64_t g = g0; g < g1; ++g) {
    const Frag f = frags[g];
    if (!f.ok) { S.err_class = BCW_ERR_CRC; S.err_frag = (uint32_t)g; break; }        // wal_iterator.go:79-82
    if (f.type < 1 || f.type > 4) { S.err_class = BCW_ERR_TYPE; S.err_frag = (uint32_t)g; break; }  // :94-95
    const uint64_t doff = (uint64_t)start_off + (uint64_t)f.blk * kBlock + f.start;
    if (in_pre) {
      if (f.type == BCW_RECORD_FULL || f.type == BCW_RECORD_LAST) {
        in_pre = false;
        S.has_emit = 1;
        S.n_emit = 1;
        acc = 0;
        continue;
      }
      if (f.len > 0 && !S.pre_nz) { S.pre_nz = 1; S.pre_off = doff; S.pre_first = (uint32_t)g; }
      S.pre_len += f.len;
    } else {
      if (acc == 0) { off = doff; first = (uint32_t)g; }
      if (f.type == BCW_RECORD_FULL) { S.n_emit++; acc = 0; }
      else if (f.type == BCW_RECORD_LAST) { S.n_emit++; acc = 0; }
      else acc += f.len;
    }
  }
  S.out_acc = acc;
  S.out_off = off;
  S.out_first = first;
  sums[b] = S;
}

// ------------------------------------------------------------------------------------------
// k_blockscan: exclusive composition of block transforms (one workgroup).
struct Xf {
  uint64_t n_emit;
  uint64_t a;      // has_emit: out acc    else: pre len
  uint64_t off;    // has_emit: out off    else: pre off
  uint32_t first;
  uint32_t err_frag;
  uint8_t has_emit, nz, err, err_class;
};

__device__ __forceinline__ Xf xf_of(const BlockSum& s) {
  Xf x;
  x.n_emit = s.n_emit;
  x.has_emit = s.has_emit;
  x.err = s.err_class != 0;
  x.err_class = s.err_class;
  x.err_frag = s.err_frag;
  if (s.has_emit) { x.a = s.out_acc; x.off = s.out_off; x.first = s.out_first; x.nz = 0; }
  else { x.a = s.pre_len; x.off = s.pre_off; x.first = s.pre_first; x.nz = s.pre_nz; }
  return x;
}
__device__ __forceinline__ Xf xf_identity() {
  Xf x{};
  x.err_frag = 0xffffffffu;
  return x;
}
// A then B
__device__ __forceinline__ Xf xf_compose(const Xf& A, const Xf& B) {
  if (A.err) return A;
  Xf R;
  R.n_emit = A.n_emit + B.n_emit;
  R.err = B.err;
  R.err_class = B.err_class;
  R.err_frag = B.err_frag;
  if (B.has_emit) {
    R.has_emit = 1; R.a = B.a; R.off = B.off; R.first = B.first; R.nz = 0;
  } else if (A.has_emit) {
    R.has_emit = 1; R.nz = 0;
    R.a = A.a + B.a;
    if (A.a > 0 || !B.nz) { R.off = A.off; R.first = A.first; }
    else { R.off = B.off; R.first = B.first; }
  } else {
    R.has_emit = 0;
    R.a = A.a + B.a;
    R.nz = A.nz | B.nz;
    if (A.nz) { R.off = A.off; R.first = A.first; } else { R.off = B.off; R.first = B.first; }
  }
  return R;
}

__global__ __launch_bounds__(1024) void k_blockscan(const BlockSum* __restrict__ sums, uint64_t nblocks,
                                                    BlockIn* __restrict__ ins, uint64_t* __restrict__ misc) {
  __shared__ Xf sm[1024];
  const uint32_t t = threadIdx.x;
  const uint64_t per = (nblocks + 1023) / 1024;
  const uint64_t lo = t * per;
  const uint64_t hi = lo + per < nblocks ? lo + per : nblocks;
  Xf mine = xf_identity();
  for (uint64_t b = lo; b < hi; ++b) mine = xf_compose(mine, xf_of(sums[b]));
  sm[t] = mine;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    Xf left = t >= d ? sm[t - d] : xf_identity();
    __syncthreads();
    if (t >= d) sm[t] = xf_compose(left, sm[t]);
    __syncthreads();
  }
  Xf run = t > 0 ? sm[t - 1] : xf_identity();
  for (uint64_t b = lo; b < hi; ++b) {
    BlockIn in;
    in.rec_base = run.n_emit;
    in.live = run.err ? 0u : 1u;
    if (run.has_emit) { in.acc = run.a; in.off = run.off; in.first = run.first; }
    else { in.acc = run.a; in.off = run.off; in.first = run.first; }
    ins[b] = in;
    run = xf_compose(run, xf_of(sums[b]));
  }
  if (t == 1023) {
    const Xf tot = sm[1023];
    misc[M_NREC] = tot.n_emit;
    misc[M_ERR_FRAG] = tot.err ? tot.err_frag : ~0ull;
    misc[M_ERR_CLASS] = tot.err ? tot.err_class : 0;
    misc[M_FIRST_BAD] = ~0ull;
  }
}

// ------------------------------------------------------------------------------------------
// k_records: record emission per block (one wave per block) + RecordFromBytes / HintRecord.Decode.
struct Emit {
  uint64_t foff, size;
  uint32_t first, emit;
};

// Go encoding/binary.Uvarint over a byte accessor; DecodeUvarint maps errors to (0,0).
template <typename RD>
__device__ __forceinline__ uint64_t uvarint(RD& rd, uint64_t pos, uint64_t len, uint32_t& used) {
  uint64_t x = 0;
  uint32_t s = 0;
  for (uint32_t i = 0; pos + i < len; ++i) {
    if (i == 10) { used = 0; return 0; }
    const uint32_t b = rd(pos + i);
    if (b < 0x80u) {
      if (i == 9 && b > 1u) { used = 0; return 0; }
      used = i + 1;
      return x | ((uint64_t)b << s);
    }
    x |= (uint64_t)(b & 0x7fu) << s;
    s += 7;
  }
  used = 0;
  return 0;
}

constexpr int kRecWaves = 4;

// intra-wave LDS hand-off (lanes of one wave run in lockstep; this orders the compiler)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
constexpr uint32_t kStage = 128;  // staged record-prefix bytes per lane

struct RecReader {
  const uint8_t* seg;
  const Frag* frags;
  uint32_t start_off;
  const uint8_t* stage;  // LDS, kStage bytes (valid for pos < nstaged)
  uint32_t nstaged;
  uint32_t f_first, f_last;
  // cache of the current fragment for the slow path
  uint32_t cf;
  uint64_t cbeg, clen, caddr;
  __device__ uint32_t operator()(uint64_t pos) {
    if (pos < nstaged) return stage[pos];
    if (pos < cbeg) { cf = f_first; cbeg = 0; const Frag f = frags[cf]; clen = f.len; caddr = (uint64_t)start_off + (uint64_t)f.blk * kBlock + f.start; }
    while (pos >= cbeg + clen && cf < f_last) {
      cbeg += clen;
      ++cf;
      const Frag f = frags[cf];
      clen = f.len;
      caddr = (uint64_t)start_off + (uint64_t)f.blk * kBlock + f.start;
    }
    return seg[caddr + (pos - cbeg)];
  }
};

__global__ __launch_bounds__(256) void k_records(const uint8_t* __restrict__ seg, uint64_t seg_len,
                                                 bcw_decode_params p, const Frag* __restrict__ frags,
                                                 const uint32_t* __restrict__ fbase, uint64_t nblocks,
                                                 uint64_t frag_cap, const BlockIn* __restrict__ ins,
                                                 bcw_record_table tab, uint64_t* __restrict__ misc) {
  __shared__ Emit s_emit[kRecWaves][64];
  __shared__ __attribute__((aligned(16))) uint8_t s_stage[kRecWaves][64][kStage];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = threadIdx.x >> 6;
  const uint64_t b = (uint64_t)blockIdx.x * kRecWaves + wave;
  if (b >= nblocks) return;
  const BlockIn in = ins[b];
  if (!in.live) return;
  uint64_t g0 = fbase[b], g1 = fbase[b + 1];
  if (g1 > frag_cap) g1 = frag_cap;
  const uint64_t err_frag = misc[M_ERR_FRAG];
  if (g1 > err_frag) g1 = err_frag;  // nothing at or after the first failing fragment is emitted
  uint64_t acc = in.acc, off = in.off;
  uint32_t first = in.first;
  uint64_t rec = in.rec_base;
  uint64_t g = g0;
  // lane 0 walks fragments and emits records in batches of 64; the wave parses the batch
  while (true) {
    uint32_t ne = 0;
    if (lane == 0) {
      while (g < g1 && ne < 64) {
        const Frag f = frags[g];
        const uint64_t doff = (uint64_t)p.start_off + (uint64_t)f.blk * kBlock + f.start;
        if (acc == 0) { off = doff; first = (uint32_t)g; }
        if (f.type == BCW_RECORD_FULL) {
          s_emit[wave][ne++] = Emit{off, f.len, (uint32_t)g, (uint32_t)g};
          acc = 0;
        } else if (f.type == BCW_RECORD_LAST) {
          acc += f.len;
          s_emit[wave][ne++] = Emit{off, acc, first, (uint32_t)g};
          acc = 0;
        } else {
          acc += f.len;
        }
        ++g;
      }
    }
    ne = __shfl(ne, 0, 64);
    wave_sync();
    if (lane < ne) {
      const Emit em = s_emit[wave][lane];
      const uint64_t r = rec + lane;
      // stage the record prefix: fast path when its first fragment holds it
      const Frag f0 = frags[em.first];
      const uint64_t a0 = (uint64_t)p.start_off + (uint64_t)f0.blk * kBlock + f0.start;
      uint64_t want = em.size < kStage ? em.size : kStage;
      uint32_t nst = 0;
      uint8_t* st = s_stage[wave][lane];
      if (f0.len >= want) {
        nst = (uint32_t)want;
        for (uint32_t k = 0; k < nst; ++k) st[k] = seg[a0 + k];
      }
      RecReader rd{seg, frags, p.start_off, st, nst, em.first, em.emit, em.first, 0, f0.len, a0};
      const uint64_t len = em.size;
      uint8_t status = BCW_ST_OK, hdr = 0, flags = 0, etag_off = 0;
      uint64_t key_len = 0, val_len = 0, meta_len = 0, expire = 0, aux0 = 0, aux1 = 0;
      uint32_t used;
      if (p.mode == BCW_MODE_RECORD) {
        // RecordFromBytes, record.go:140-239
        const uint64_t min_hdr = 1ull + p.ns_size + 1ull + 3ull;
        if (len < min_hdr) {
          status = BCW_ST_INVALID;
        } else {
          uint64_t o = 0;
          const uint64_t header = rd(0);
          o = 1 + p.ns_size;
          const uint32_t flag = rd(o);
          ++o;
          key_len = uvarint(rd, o, len, used); o += used;
          val_len = uvarint(rd, o, len, used); o += used;
          meta_len = uvarint(rd, o, len, used); o += used;
          const uint64_t etag_len = (flag & 1u) ? 0 : p.etag_size;
          uint64_t expire_size = 0;
          hdr = (uint8_t)header; flags = (uint8_t)flag; etag_off = (uint8_t)o;
          if ((flag & 2u) == 0) {
            if (o + etag_len > len) {
              status = BCW_ST_PANIC;  // data[offset+etagLen:] out of range (record.go:186)
            } else {
              expire = uvarint(rd, o + etag_len, len, used);
              expire_size = used;
              expire += p.base_time;
            }
          }
          if (status == BCW_ST_OK) {
            const int64_t cur_hdr = (int64_t)o + (int64_t)etag_len + (int64_t)expire_size;
            const int64_t cur_total = cur_hdr + (int64_t)(key_len + val_len + meta_len);
            if ((uint64_t)cur_hdr != header || cur_total != (int64_t)len) {
              status = BCW_ST_INVALID;
            } else {
              const uint64_t s1 = key_len + val_len;
              const uint64_t s2 = s1 + meta_len;
              const bool wrapped = (s1 < key_len) || (s2 < s1);
              if ((int64_t)key_len < 0 || (int64_t)val_len < 0 || (int64_t)meta_len < 0 || wrapped)
                status = BCW_ST_PANIC;
              else if (key_len > 0xffffffffull || val_len > 0xffffffffull || meta_len > 0xffffffffull ||
                       len > 0xffffffffull)
                status = BCW_ST_UNSUPPORTED;
            }
          }
        }
      } else {
        // HintRecord.Decode, hint.go:50-84
        const uint64_t min_sz = (uint64_t)p.ns_size + 5ull;
        if (len < min_sz) {
          status = BCW_ST_INVALID;
        } else {
          int64_t o = p.ns_size;
          key_len = uvarint(rd, (uint64_t)o, len, used);
          o += used;
          const int64_t key_off = o;
          o = (int64_t)((uint64_t)o + key_len);
          hdr = (uint8_t)key_off;
          if (o < 0 || o > (int64_t)len) {
            status = BCW_ST_PANIC;
          } else {
            expire = uvarint(rd, (uint64_t)o, len, used); o += used;  // fid
            aux0 = uvarint(rd, (uint64_t)o, len, used); o += used;    // off
            aux1 = uvarint(rd, (uint64_t)o, len, used); o += used;    // size
            if (o != (int64_t)len) status = BCW_ST_INVALID;
            else if ((int64_t)key_len < 0) status = BCW_ST_PANIC;
          }
        }
      }
      if (r < tab.capacity) {
        tab.foff[r] = em.foff;
        tab.size[r] = em.size;
        tab.expire[r] = expire;
        if (tab.aux0) tab.aux0[r] = aux0;
        if (tab.aux1) tab.aux1[r] = aux1;
        tab.key_len[r] = (uint32_t)key_len;
        tab.val_len[r] = (uint32_t)val_len;
        tab.meta_len[r] = (uint32_t)meta_len;
        tab.first_frag[r] = em.first;
        tab.emit_frag[r] = em.emit;
        tab.hdr_size[r] = hdr;
        tab.flags[r] = flags;
        tab.etag_off[r] = etag_off;
        tab.status[r] = status;
      }
      if (status != BCW_ST_OK) atomicMin((unsigned long long*)&misc[M_FIRST_BAD], (unsigned long long)r);
    }
    rec += ne;
    wave_sync();
    if (ne < 64) break;
  }
}

__device__ void finalize(const uint64_t* __restrict__ misc, uint64_t nblocks, uint64_t frag_total,
                           uint64_t frag_cap, const Frag* __restrict__ frags, uint32_t start_off, uint32_t tail_panic,
                           bcw_decode_result* __restrict__ res) {
  bcw_decode_result r{};
  r.n_records = misc[M_NREC];
  r.n_records_total = misc[M_NREC];
  r.err_frag = misc[M_ERR_FRAG];
  r.err_class = (int32_t)misc[M_ERR_CLASS];
  r.n_frags = r.err_frag != ~0ull ? r.err_frag + 1 : frag_total;
  // a last block of 1..6 bytes makes the reference iterator panic after every earlier record
  // (wal_iterator.go:62-76 re-slices a header from its stale buffer, then buf[7:7+negative])
  if (r.err_class == BCW_ERR_NONE && tail_panic) r.err_class = BCW_ERR_PANIC;
  r.err_file_off = 0;
  if (r.err_frag != ~0ull && r.err_frag < frag_cap) {
    const Frag f = frags[r.err_frag];
    r.err_file_off = (uint64_t)start_off + (uint64_t)f.blk * kBlock + f.start - kHdr;
  }
  const uint64_t fb = misc[M_FIRST_BAD];
  r.first_bad_record = fb == ~0ull ? -1 : (int32_t)(fb < 0x7fffffffull ? fb : 0x7fffffffull);
  r.n_blocks = nblocks;
  r.retry_frag_capacity = frag_total > frag_cap ? frag_total : 0;
  *res = r;
}

__global__ void k_export_frags(const Frag* __restrict__ frags, const uint64_t* __restrict__ misc, uint64_t cap,
                               uint32_t start_off, bcw_frag_table out) {
  const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t n = misc[M_NFRAGS];
  if (g >= n || g >= cap || g >= out.capacity) return;
  const Frag f = frags[g];
  out.data_off[g] = (uint64_t)start_off + (uint64_t)f.blk * kBlock + f.start;
  out.len[g] = f.len;
  out.stored_crc[g] = f.crc;
  out.type[g] = f.type;
  out.crc_ok[g] = f.ok;
}

__global__ void k_finalize_dev(const uint64_t* __restrict__ misc, uint64_t nblocks, uint64_t frag_cap,
                               const Frag* __restrict__ frags, uint32_t start_off, uint32_t tail_panic,
                               bcw_decode_result* __restrict__ res);

// ------------------------------------------------------------------------------------------
hipError_t launch_decode(const uint8_t* d_seg, const bcw_decode_params& p, const bcw_record_table& t,
                         bcw_decode_result* d_result, const Tables& tabs, Scratch& s, uint64_t nblocks,
                         hipStream_t stream, int num_cus, Prof* prof) {
  Prof dummy;
  Prof& pr = prof ? *prof : dummy;
  hipEvent_t ev = nullptr;
  const uint32_t nb_grid = (uint32_t)((nblocks + 255) / 256);
  pr.begin(K_CHASE_COUNT, stream, ev);
  k_chase<<<nb_grid, 256, 0, stream>>>(d_seg, p.seg_len, p.start_off, nblocks, s.nfrag, nullptr, nullptr, 0, 0);
  pr.end(K_CHASE_COUNT, stream, ev);
  pr.begin(K_SCAN, stream, ev);
  k_scan_u32<<<1, 1024, 0, stream>>>(s.nfrag, s.fbase, nblocks, &s.misc[M_NFRAGS]);
  pr.end(K_SCAN, stream, ev);
  pr.begin(K_CHASE_WRITE, stream, ev);
  k_chase<<<nb_grid, 256, 0, stream>>>(d_seg, p.seg_len, p.start_off, nblocks, s.nfrag, s.fbase, s.frags,
                                       s.frag_cap, 1);
  pr.end(K_CHASE_WRITE, stream, ev);
  pr.begin(K_CRC, stream, ev);
  k_crc<<<(uint32_t)num_cus, 1024, kCrcLds, stream>>>(d_seg, p.seg_len, p.start_off, nblocks, s.fbase, s.frags,
                                                      s.frag_cap, tabs);
  pr.end(K_CRC, stream, ev);
  pr.begin(K_BLOCKSUM, stream, ev);
  k_blocksum<<<nb_grid, 256, 0, stream>>>(s.frags, s.fbase, nblocks, p.start_off, s.frag_cap, s.sums);
  pr.end(K_BLOCKSUM, stream, ev);
  pr.begin(K_BLOCKSCAN, stream, ev);
  k_blockscan<<<1, 1024, 0, stream>>>(s.sums, nblocks, s.ins, s.misc);
  pr.end(K_BLOCKSCAN, stream, ev);
  pr.begin(K_RECORDS, stream, ev);
  k_records<<<(uint32_t)((nblocks + kRecWaves - 1) / kRecWaves), 64 * kRecWaves, 0, stream>>>(
      d_seg, p.seg_len, p, s.frags, s.fbase, nblocks, s.frag_cap, s.ins, t, s.misc);
  pr.end(K_RECORDS, stream, ev);
  const uint64_t tail = (p.seg_len - p.start_off) % kBlock;
  const uint32_t tail_panic = (tail > 0 && tail < kHdr) ? 1u : 0u;
  pr.begin(K_FINALIZE, stream, ev);
  k_finalize_dev<<<1, 1, 0, stream>>>(s.misc, nblocks, s.frag_cap, s.frags, p.start_off, tail_panic, d_result);
  pr.end(K_FINALIZE, stream, ev);
  return hipGetLastError();
}

__global__ void k_finalize_dev(const uint64_t* __restrict__ misc, uint64_t nblocks, uint64_t frag_cap,
                               const Frag* __restrict__ frags, uint32_t start_off, uint32_t tail_panic,
                               bcw_decode_result* __restrict__ res) {
  finalize(misc, nblocks, misc[M_NFRAGS], frag_cap, frags, start_off, tail_panic, res);
}

hipError_t launch_export_frags(const Scratch& s, const bcw_frag_table& out, uint32_t start_off, hipStream_t stream,
                               uint64_t n) {
  if (n == 0) return hipSuccess;
  k_export_frags<<<(uint32_t)((n + 255) / 256), 256, 0, stream>>>(s.frags, s.misc, s.frag_cap, start_off, out);
  return hipGetLastError();
}

}  // namespace bcw
