// bcw_encode.hip -- MI355X (gfx950) kernels for bitcaskDB WAL encode: the compaction re-encode
// (compactOneWal, compaction.go:294-327 = Record.Encode record.go:57-138 + Wal.WriteRecord
// wal.go:490-553 + HintRecord.Encode hint.go:32-48) and the hint rebuild (NewHintByWal,
// hint.go:123-161). Input: a source WAL image and its decoded record + fragment tables (the
// decode pipeline of bcw_decode.hip, same context). Output: the bytes the reference appends to
// the destination WAL and the hint WAL, and the offset WriteRecord returns for every record.
//
// Pipeline (one HIP stream, no host synchronisation; DESIGN.md "Encode"):
//   k_enc_prep      per source row: keep / Encode errors / re-encoded payload size     record.go:57-138
//   k_tile_*        3-phase scan: dense list of written records, y-coordinates a_j
//   k_ev_win/walk/emit/fix  the writer's layout recurrence as an event scan              wal.go:505-549
//   k_recoff        per record: the file offset WriteRecord returns                     wal.go:514-516
//   (compaction) k_hint_sizes + scan + event scan + k_recoff for the hint WAL           hint.go:32-48
//   k_recdesc_w     per dst record: payload as literal prefix | source range | literal suffix, and the
//                   record's CRC from the source fragments' verified check words (CRC combine)
//   k_wcopy         the dst WAL, one wave per record in one or two fragments: a re-layout copy, only
//                   the shorter piece of a split record is hashed (utils.go:24-29)
//   k_write         the other dst records (more fragments, irregular sources): 16 B units copied and
//                   folded into each fragment's CRC-32C
//   k_write_general the rare records with more literal bytes than the descriptor holds
//   k_hwrite        the hint WAL, one record per lane, staged per wave in LDS
//   k_enc_finalize  bcw_encode_result
//
// Layout as an event scan. Concatenate the records' (7 B header + payload) units into a y axis:
// record j occupies [a_j, a_{j+1}), a_j = sum_{i<j}(n_i + 7). A block either starts with a
// continuation header (y-length L-7 = M of payload+headers) or exactly at a record header
// (y-length L). The writer's rules (pad when < 7 B are left, zero-length First when exactly 7 are
// left) make block k end at E_k = Y_k + L - 7c_k and the next block start at Y_{k+1} = a_i when
// some record header a_i lies in [E_k - 6, E_k] (an "event": exact fill or pad of E_k - a_i
// bytes), else at E_k with a continuation header. Between events every block start is congruent
// mod M, so with rho = (next block end) mod M, record i is an event iff (rho - a_i) mod M <= 6,
// and after it rho = (a_i + 7) mod M. That is a scan with a 15-bit state that is the identity on
// all but rare records (~7/M of them). The scan runs in parallel over windows of 16384 records
// (per-window next-event chains and state tables, one sequential table read per window, see k_ev_win),
// and every other quantity (event blocks, record offsets, and from them fragment types, lengths and
// pads) follows in parallel from the event list.
#include <algorithm>
#include <cstdlib>

#include "bcw_internal.h"

namespace bcw {
namespace enc {

constexpr uint32_t kL = kBlock;           // 32768
constexpr uint32_t kM = kBlock - kHdr;    // 32761
constexpr int kTileItems = 4096;          // scan tile: 256 threads x 16 items
constexpr int kEvWin = 16384;          // records per event-scan window (14-bit record index in a window)
constexpr int kEvShift = 14;
constexpr uint32_t kEvTab = 32768;     // residue table entries (>= M)

// emisc slots
enum {
  X_NIN = 0,      // source rows delivered (IterateRecord)
  X_ERR = 1,      // min over rows of (row << 2 | class) of Record.Encode failures
  X_SRCERR = 2,   // source error class (BCW_ENC_ERR_SRC when iteration stopped on a bad row / fragment)
  X_NDENSE = 3,   // records written
  X_FAIL = 4,     // BCW_ENC_ERR_TABLE / BCW_ENC_ERR_STALE: the source inputs are unusable, nothing encoded
  X_WL16 = 5,     // dst records k_wcopy leaves to k_write<16> (work list from the front of wl)
  X_WLG = 6,      // ... and to k_write_general (from the back of wl)
  X_LAY = 8,      // per layout (wal: 8, hint: 16): +0 A_N, +1 nev, +2 k_end, +3 end, +4 b0, +5 U, +6 ok
};
constexpr int kLayStride = 8;

__device__ __forceinline__ uint32_t uvlen(uint64_t v) {
  uint32_t n = 1;
  while (v >= 0x80) { v >>= 7; ++n; }
  return n;
}
__device__ __forceinline__ uint32_t uvput(uint8_t* p, uint64_t v) {
  uint32_t n = 0;
  while (v >= 0x80) { p[n++] = (uint8_t)(v | 0x80); v >>= 7; }
  p[n++] = (uint8_t)v;
  return n;
}

// a shift operator (nibble images: 8 x 16 words) applied to x
__device__ __forceinline__ uint32_t op_apply_s(const uint32_t* __restrict__ op, uint32_t x) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= op[i * 16 + ((x >> (4 * i)) & 15u)];
  return r;
}
// A_{8m}(x) (m zero bytes appended to a raw CRC-32C state) from the power-of-two operators p2[k] =
// A_{8*2^k} (or their inverses: A_{8m}^-1), one operator per set bit of m
__device__ __forceinline__ uint32_t shift_by(const uint32_t* __restrict__ p2, uint32_t x, uint64_t m) {
  for (int k = 0; m != 0 && x != 0; ++k, m >>= 1)
    if (m & 1u) x = op_apply_s(p2 + k * 128, x);
  return x;
}

// ---- source payload access: the record's bytes are the data of fragments [f0, f1] ----
struct SrcRec {
  uint32_t f0, f1;
};
__device__ __forceinline__ SrcRec src_rec(const bcw_record_table& t, const Frag* __restrict__ frags, uint64_t row) {
  SrcRec r;
  r.f1 = t.emit_frag[row];
  r.f0 = t.first_frag[row];
  if (frags[r.f1].type == BCW_RECORD_FULL) r.f0 = r.f1;  // a Full emission carries only its own data
  return r;
}
__device__ __forceinline__ uint64_t frag_file(const Frag& f, uint32_t start_off) {
  return (uint64_t)start_off + (uint64_t)f.blk * kL + f.start;
}
// byte z of the source payload
__device__ uint8_t src_byte(const uint8_t* __restrict__ seg, const Frag* __restrict__ frags, uint32_t start_off,
                            SrcRec r, uint64_t z) {
  uint32_t f = r.f0;
  for (;;) {
    const Frag F = frags[f];
    if (z < F.len || f >= r.f1) return seg[frag_file(F, start_off) + z];
    z -= F.len;
    ++f;
  }
}

// AppMetaSize == 0 for the canonical msgpack forms of an empty map (oracle oc_meta_app_size_zero):
// Record.Encode then drops the meta (record.go:82-86, meta.go:38-49)
__device__ bool meta_dropped(const uint8_t* __restrict__ seg, const Frag* __restrict__ frags, uint32_t start_off,
                             SrcRec r, uint64_t moff, uint64_t mlen) {
  if (mlen == 0 || mlen > 31) return false;
  const uint32_t b0 = src_byte(seg, frags, start_off, r, moff);
  if (mlen == 1) return b0 == 0xc0 || b0 == 0x80;
  if ((b0 & 0xf0) != 0x80 || mlen != 1 + 2 * (uint64_t)(b0 & 0x0f)) return false;
  for (uint64_t i = 1; i < mlen; ++i) {
    const uint32_t b = src_byte(seg, frags, start_off, r, moff + i);
    if (b != 0xa0 && b != 0xc0) return false;
  }
  return true;
}

struct EncDev {
  const uint8_t* seg;
  uint64_t src_len;
  const Frag* frags;
  bcw_record_table t;
  const bcw_decode_result* sres;
  const uint8_t* keep;
  uint64_t dst_base, fid;
  uint64_t gen;  // generation of the context's latest decode (its fragment table is `frags`)
  uint32_t start_off, mode, ns, etag;
};

// ------------------------------------------------------------------------------------------
// k_enc_prep: per delivered source row, the payload size the writer will append (0 = nothing).
//   compaction: Record.Encode of the kept rows (record.go:57-138): flags recomputed (noEtag from
//   the etag length, tombstone kept, noExpire when Expire == 0), expire re-based on the dst
//   baseTime ("invalid expire" when below it; a delta of >= 2^35 overflows the 5-byte varint
//   array and panics), meta dropped when its app size is 0.
//   hint rebuild: HintRecord{ns, key, fid, foff - 7, size}.Encode (hint.go:32-48,131-145).
__global__ __launch_bounds__(256) void k_enc_prep(EncDev e, uint64_t rows, uint32_t* __restrict__ sz,
                                                   uint8_t* __restrict__ mflag, uint64_t* __restrict__ rec_off,
                                                   uint64_t* __restrict__ emisc) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  const bcw_decode_result* R = e.sres;
  const uint64_t nrec = R->n_records;
  // the source must be the context's latest decode (its fragment table), fit the table and not be a decode that gave
  // up on an internal wait (BCW_ERR_INTERNAL)
  const uint32_t fail = R->generation != e.gen ? BCW_ENC_ERR_STALE
                        : (nrec > rows || R->err_class == BCW_ERR_INTERNAL) ? BCW_ENC_ERR_TABLE : 0u;
  const uint64_t nin = fail ? 0
                       : (R->first_bad_record >= 0 && (uint64_t)R->first_bad_record < nrec)
                           ? (uint64_t)R->first_bad_record : nrec;
  if (i == 0) {
    emisc[X_NIN] = nin;
    emisc[X_FAIL] = fail;
    emisc[X_SRCERR] = (!fail && (nin < nrec || R->err_class != BCW_ERR_NONE)) ? 1u : 0u;
  }
  if (i >= rows) return;
  if (rec_off && i < nrec && !fail) rec_off[i] = ~0ull;
  if (i >= nin) { sz[i] = 0; return; }
  const bcw_record_table& t = e.t;
  const uint64_t klen = t.key_len[i];
  uint32_t n = 0;
  if (e.mode == BCW_ENC_HINT) {
    const uint64_t off = t.foff[i] - kHdr, size = t.size[i];
    n = e.ns + uvlen(klen) + (uint32_t)klen + uvlen(e.fid) + uvlen(off) + uvlen(size);
  } else if (e.keep[i]) {
    const uint32_t flags = t.flags[i];
    const uint64_t vlen = t.val_len[i], mlen0 = t.meta_len[i], expire = t.expire[i], size = t.size[i];
    const uint32_t el = (flags & 1u) ? 0u : e.etag;
    const SrcRec sr = src_rec(t, e.frags, i);
    const bool drop = meta_dropped(e.seg, e.frags, e.start_off, sr, size - mlen0, mlen0);
    mflag[i] = drop ? 1 : 0;
    const uint64_t mlen = drop ? 0 : mlen0;
    uint32_t ve = 0;
    if (expire != 0) {
      if (expire < e.dst_base) { atomicMin((unsigned long long*)&emisc[X_ERR], (unsigned long long)(i << 2 | BCW_ENC_ERR_EXPIRE)); sz[i] = 0; return; }
      const uint64_t d = expire - e.dst_base;
      if (d >= (1ull << 35)) { atomicMin((unsigned long long*)&emisc[X_ERR], (unsigned long long)(i << 2 | BCW_ENC_ERR_PANIC)); sz[i] = 0; return; }
      ve = uvlen(d);
    }
    const uint64_t hn = 2 + e.ns + uvlen(klen) + uvlen(vlen) + uvlen(mlen) + el + ve;
    n = (uint32_t)(hn + klen + vlen + mlen);
  }
  sz[i] = n;
}

// rows that are written: [0, nin) cut at the first Record.Encode error
__device__ __forceinline__ uint64_t eff_rows(const uint64_t* emisc) {
  const uint64_t nin = emisc[X_NIN], err = emisc[X_ERR];
  return (err >> 2) < nin ? (err >> 2) : nin;
}

// ------------------------------------------------------------------------------------------
// 3-phase scan over item sizes: tile sums, a one-workgroup scan of the tiles, then a rescan that
// writes the dense y-coordinates a_j (and, over source rows, the dense -> row map).
struct TileSum {
  uint64_t cnt, bytes;
};

__device__ __forceinline__ uint64_t wave_incl_u64(uint64_t v, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t t = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += t;
  }
  return v;
}

// item count of a scan: source rows (compaction: cut at the first Encode error) or dense records
__device__ __forceinline__ uint64_t scan_items(const uint64_t* emisc, int over_rows) {
  return over_rows ? eff_rows(emisc) : emisc[X_NDENSE];
}

__global__ __launch_bounds__(256) void k_tile_sums(const uint32_t* __restrict__ sz, const uint64_t* __restrict__ emisc,
                                                    int over_rows, TileSum* __restrict__ ts) {
  const uint64_t n = scan_items(emisc, over_rows);
  const uint64_t base = blockIdx.x * (uint64_t)kTileItems;
  if (base >= n) return;
  uint64_t c = 0, b = 0;
  for (int k = 0; k < 16; ++k) {
    const uint64_t i = base + (uint64_t)k * 256 + threadIdx.x;
    if (i < n) {
      const uint32_t s = sz[i];
      if (s) { c += 1; b += s + kHdr; }
    }
  }
  __shared__ uint64_t sc[4], sb[4];
  for (int d = 32; d >= 1; d >>= 1) { c += __shfl_xor(c, d, 64); b += __shfl_xor(b, d, 64); }
  if ((threadIdx.x & 63) == 0) { sc[threadIdx.x >> 6] = c; sb[threadIdx.x >> 6] = b; }
  __syncthreads();
  if (threadIdx.x == 0) ts[blockIdx.x] = {sc[0] + sc[1] + sc[2] + sc[3], sb[0] + sb[1] + sb[2] + sb[3]};
}

// one workgroup: exclusive scan of the tile sums; totals -> emisc (count, A_N), da[count] = A_N
__global__ __launch_bounds__(1024) void k_tile_scan(TileSum* __restrict__ ts, uint64_t* __restrict__ emisc,
                                                     int over_rows, int lay, uint64_t* __restrict__ da) {
  const uint64_t n = scan_items(emisc, over_rows);
  const uint64_t ntiles = (n + kTileItems - 1) / kTileItems;
  __shared__ uint64_t wc[16], wb[16];
  __shared__ uint64_t carry_c, carry_b;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) { carry_c = 0; carry_b = 0; }
  __syncthreads();
  for (uint64_t b0 = 0; b0 < ntiles; b0 += 1024) {
    const uint64_t t = b0 + threadIdx.x;
    TileSum v = t < ntiles ? ts[t] : TileSum{0, 0};
    const uint64_t ic = wave_incl_u64(v.cnt, lane), ib = wave_incl_u64(v.bytes, lane);
    if (lane == 63) { wc[wave] = ic; wb[wave] = ib; }
    __syncthreads();
    uint64_t pc = carry_c, pb = carry_b;
    for (uint32_t w = 0; w < wave; ++w) { pc += wc[w]; pb += wb[w]; }
    if (t < ntiles) ts[t] = {pc + ic - v.cnt, pb + ib - v.bytes};
    __syncthreads();
    if (threadIdx.x == 1023) { carry_c = pc + ic; carry_b = pb + ib; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (over_rows) emisc[X_NDENSE] = carry_c;
    emisc[X_LAY + lay * kLayStride + 0] = carry_b;
    da[carry_c] = carry_b;
  }
}

__global__ __launch_bounds__(256) void k_tile_scatter(const uint32_t* __restrict__ sz, const uint64_t* __restrict__ emisc,
                                                       int over_rows, const TileSum* __restrict__ ts,
                                                       uint32_t* __restrict__ dsrc, uint64_t* __restrict__ da) {
  const uint64_t n = scan_items(emisc, over_rows);
  const uint64_t base = blockIdx.x * (uint64_t)kTileItems;
  if (base >= n) return;
  // each thread: 16 consecutive items (so the dense order is the row order)
  const uint64_t i0 = base + threadIdx.x * 16ull;
  uint32_t s[16];
  uint64_t c = 0, b = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    s[k] = (i0 + k < n) ? sz[i0 + k] : 0u;
    if (s[k]) { c += 1; b += s[k] + kHdr; }
  }
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t ic = wave_incl_u64(c, lane), ib = wave_incl_u64(b, lane);
  __shared__ uint64_t wc[4], wb[4];
  if (lane == 63) { wc[wave] = ic; wb[wave] = ib; }
  __syncthreads();
  uint64_t pc = ts[blockIdx.x].cnt, pb = ts[blockIdx.x].bytes;
  for (uint32_t w = 0; w < wave; ++w) { pc += wc[w]; pb += wb[w]; }
  pc += ic - c;
  pb += ib - b;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (s[k]) {
      if (over_rows) dsrc[pc] = (uint32_t)(i0 + k);
      da[pc] = pb;
      pc += 1;
      pb += s[k] + kHdr;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Layout events (see the file header). ev[0] is the virtual event of the writer's start position
// q0 (Y = -U in block b0 = q0 / L, no continuation header); ev[g] for g >= 1: record rec starts
// block blk exactly at its header (Y = a_rec), after `pad` zero bytes ended block blk-1.
struct Ev {
  uint64_t blk;
  int64_t ya;
  uint32_t rec;  // dense record index; 0xffffffff for the virtual event
  uint32_t pad;
};

// The scan in parallel. Records are cut into windows of kEvWin. For record q, let hn(q) be the next
// event if q is one: the first q' > q with r_q' in {r_q + 1, ..., r_q + 7} (mod M). Within a window the
// events after any event are the hn-chain from it, so:
//   k_ev_win   one workgroup per window: per-residue lists in LDS (atomic exchange; link = old head),
//              hn inside the window by walking 7 lists, then pointer jumping gives every record's
//              chain end in the window and chain length; finally, for every state rho, the window's
//              first event q (the first record with r_q in {rho - 6, ..., rho}) and what its chain
//              leaves behind: T_w[rho] = q | events << 16 | r_last << 32 (q = 0xffff: no event, rho
//              passes through unchanged). Window 0 also resolves the writer's start (record 0 excluded,
//              or the forced event at record 0 when its header does not fit the first block).
//   k_ev_walk  one thread: rho through the windows, one T read per window: each window's first event,
//              its entry state and the events before it.
//   k_ev_emit  one thread per window: the window's events along its hn-chain (record, pad).
//   k_ev_fix   event blocks / y-coordinates, the layout end.
constexpr uint16_t kNone16 = 0xffffu;
constexpr uint64_t kTNone = 0xffffull;
constexpr int kEvPer = kEvWin / 1024;

__global__ __launch_bounds__(1024) void k_ev_win(const uint64_t* __restrict__ da, uint64_t* __restrict__ emisc,
                                                 int lay, uint64_t q0, uint64_t* __restrict__ evt,
                                                 uint16_t* __restrict__ hnl) {
  const uint64_t N = emisc[X_NDENSE];
  const uint64_t w = blockIdx.x, base = w * kEvWin;
  if (base >= N) return;
  const uint32_t nq = (uint32_t)(N - base < (uint64_t)kEvWin ? N - base : (uint64_t)kEvWin);
  __shared__ uint32_t s_a[kEvTab];  // list heads; then F[32768] (u16), P[16384] (u16), C[16384] (u16)
  __shared__ uint16_t s_b[kEvWin];  // list links; then the residue of every record
  uint16_t* F = reinterpret_cast<uint16_t*>(s_a);
  uint16_t* Pp = F + kEvTab;
  uint16_t* Cc = Pp + kEvWin;
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  for (uint32_t i = tid; i < kEvTab; i += 1024) s_a[i] = 0xffffffffu;
  uint32_t r[kEvPer];
#pragma unroll
  for (int k = 0; k < kEvPer; ++k) {
    const uint32_t q = (uint32_t)k * 1024 + tid;
    r[k] = q < nq ? (uint32_t)(da[base + q] % kM) : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kEvPer; ++k) {
    const uint32_t q = (uint32_t)k * 1024 + tid;
    if (q < nq) {
      const uint32_t old = atomicExch(&s_a[r[k]], q);
      s_b[q] = old == 0xffffffffu ? kNone16 : (uint16_t)old;
    }
  }
  __syncthreads();
  // min q' > after in the list of residue v (lists are in arbitrary order: walked to the end)
  auto walk = [&](uint32_t v, int32_t after) -> uint32_t {
    uint32_t best = kNone16;
    uint32_t t = s_a[v];
    while (t != 0xffffffffu) {
      if ((int32_t)t > after && t < best) best = t;
      const uint16_t nx = s_b[t];
      t = nx == kNone16 ? 0xffffffffu : nx;
    }
    return best;
  };
  uint16_t fv[kEvTab / 1024];
#pragma unroll
  for (int k = 0; k < (int)(kEvTab / 1024); ++k) {
    const uint32_t v = (uint32_t)k * 1024 + tid;
    fv[k] = v < kM ? (uint16_t)walk(v, -1) : kNone16;
  }
  uint16_t hn[kEvPer];
#pragma unroll
  for (int k = 0; k < kEvPer; ++k) {
    const uint32_t q = (uint32_t)k * 1024 + tid;
    uint32_t b = kNone16;
    if (q < nq)
      for (uint32_t d = 1; d <= kHdr; ++d) {
        const uint32_t v = r[k] + d >= kM ? r[k] + d - kM : r[k] + d;
        b = min(b, walk(v, (int32_t)q));
      }
    hn[k] = (uint16_t)b;
  }
  // window 0: the first event after the writer's start position q0
  uint32_t qs = kNone16;
  if (w == 0 && tid < 64) {
    const int64_t U = (int64_t)(q0 % kL);
    if (kL - U < (int64_t)kHdr) {
      qs = 0;  // record 0's header does not fit: pad, event at record 0
    } else {
      const uint32_t rho0 = (uint32_t)((kL - U) % kM);
      uint32_t c = kNone16;
      if (lane < kHdr) c = walk(rho0 >= lane ? rho0 - lane : rho0 + kM - lane, 0);  // record 0 never tested
#pragma unroll
      for (int s2 = 4; s2 >= 1; s2 >>= 1) c = min(c, (uint32_t)__shfl_xor((int)c, s2, 64));
      qs = c;
    }
  }
  __syncthreads();  // every list read is done: the LDS is reused
#pragma unroll
  for (int k = 0; k < (int)(kEvTab / 1024); ++k) F[(uint32_t)k * 1024 + tid] = fv[k];
#pragma unroll
  for (int k = 0; k < kEvPer; ++k) {
    const uint32_t q = (uint32_t)k * 1024 + tid;
    if (q < nq) {
      Pp[q] = hn[k] == kNone16 ? (uint16_t)q : hn[k];
      Cc[q] = hn[k] == kNone16 ? 0 : 1;
      s_b[q] = (uint16_t)r[k];
      hnl[base + q] = hn[k];
    }
  }
  __syncthreads();
  // pointer jumping: P -> the chain's last record in the window, C -> hops to it
  for (int round = 0; round < kEvShift; ++round) {
    uint16_t np[kEvPer], nc[kEvPer];
#pragma unroll
    for (int k = 0; k < kEvPer; ++k) {
      const uint32_t q = (uint32_t)k * 1024 + tid;
      np[k] = 0;
      nc[k] = 0;
      if (q < nq) {
        const uint32_t pq = Pp[q];
        np[k] = Pp[pq];
        nc[k] = (uint16_t)(Cc[q] + Cc[pq]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kEvPer; ++k) {
      const uint32_t q = (uint32_t)k * 1024 + tid;
      if (q < nq) {
        Pp[q] = np[k];
        Cc[q] = nc[k];
      }
    }
    __syncthreads();
  }
  auto entry = [&](uint32_t q) -> uint64_t {
    return q == kNone16 ? kTNone
                        : ((uint64_t)q | ((uint64_t)(Cc[q] + 1u) << 16) | ((uint64_t)s_b[Pp[q]] << 32));
  };
  uint64_t* T = evt + w * kEvTab;
#pragma unroll 4
  for (int k = 0; k < (int)(kEvTab / 1024); ++k) {
    const uint32_t rho = (uint32_t)k * 1024 + tid;
    uint64_t ent = kTNone;
    if (rho < kM) {
      uint32_t q = kNone16;
      for (uint32_t d = 0; d < kHdr; ++d) q = min(q, (uint32_t)F[rho >= d ? rho - d : rho + kM - d]);
      ent = entry(q);
    }
    T[rho] = ent;
  }
  if (w == 0 && tid == 0) emisc[X_LAY + lay * kLayStride + 6] = entry(qs);
}

// one thread: the state through the windows (ev[0] = the writer's start; evw[w] = {first event of window
// w (0xffffffff: none), state entering it, events before it})
__global__ void k_ev_walk(uint64_t* __restrict__ emisc, int lay, uint64_t q0, const uint64_t* __restrict__ evt,
                          uint32_t* __restrict__ evw, Ev* __restrict__ ev) {
  if (threadIdx.x != 0) return;
  const uint64_t N = emisc[X_NDENSE];
  uint64_t* X = emisc + X_LAY + lay * kLayStride;
  const int64_t U = (int64_t)(q0 % kL);
  const uint64_t b0 = q0 / kL;
  ev[0] = {b0, -U, 0xffffffffu, 0};
  const uint64_t nwin = (N + kEvWin - 1) / kEvWin;
  uint32_t rho = (uint32_t)((kL - U) % kM);
  uint64_t total = 0;
  for (uint64_t w = 0; w < nwin; ++w) {
    const uint64_t ent = w == 0 ? X[6] : evt[w * kEvTab + rho];
    const uint32_t q = (uint32_t)(ent & 0xffffu);
    evw[3 * w + 2] = (uint32_t)total;
    if (q == kNone16) {
      evw[3 * w] = 0xffffffffu;
      continue;
    }
    evw[3 * w] = q;
    evw[3 * w + 1] = rho;
    total += (ent >> 16) & 0xffffu;
    rho = (uint32_t)(((ent >> 32) & 0xffffu) + kHdr) % kM;
  }
  X[1] = 1 + total;
  X[4] = b0;
  X[5] = (uint64_t)U;
}

// one thread per window: its events along the hn-chain; evb[w] = index of the last event before it
__global__ __launch_bounds__(64) void k_ev_emit(const uint64_t* __restrict__ da, const uint64_t* __restrict__ emisc,
                                                const uint32_t* __restrict__ evw, const uint16_t* __restrict__ hnl,
                                                Ev* __restrict__ ev, uint32_t* __restrict__ evb) {
  const uint64_t N = emisc[X_NDENSE];
  const uint64_t w = blockIdx.x * 64ull + threadIdx.x;
  if (w * kEvWin >= N) return;
  const uint32_t before = evw[3 * w + 2];
  evb[w] = before;
  uint32_t q = evw[3 * w];
  if (q == 0xffffffffu) return;
  uint32_t rho = evw[3 * w + 1];
  uint64_t g = 1ull + before;
  const uint64_t base = w * kEvWin;
  for (;;) {
    const uint64_t rec = base + q;
    const uint16_t nx = hnl[rec];
    const uint32_t rq = (uint32_t)(da[rec] % kM);
    const uint32_t d = rho >= rq ? rho - rq : rho + kM - rq;  // (rho - r) mod M <= 6: the pad
    ev[g++] = {0, 0, (uint32_t)rec, d};
    rho = (rq + kHdr) % kM;
    if (nx == kNone16) break;
    q = nx;
  }
}

// Event blocks and y-coordinates: ev[g].ya = a_rec, the block it starts is kb_g = kb_{g-1} + m_g + 1 with
// m_g = (E_g - ya_{g-1} - L) / M blocks between (E_g = a_rec + pad: the block end that hit the header),
// an inclusive scan over the events; then the layout's end (X[2], X[3]). One workgroup.
__global__ __launch_bounds__(1024) void k_ev_fix(const uint64_t* __restrict__ da, uint64_t* __restrict__ emisc,
                                                 int lay, Ev* __restrict__ ev) {
  const uint64_t N = emisc[X_NDENSE];
  uint64_t* X = emisc + X_LAY + lay * kLayStride;
  const uint64_t AN = X[0], nev = X[1], b0 = X[4];
  const int64_t U = (int64_t)X[5];
  __shared__ uint32_t s_w[16];
  __shared__ uint64_t s_tot;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  uint64_t kb = b0;
  for (uint64_t g0 = 1; g0 < nev; g0 += 1024) {
    const uint64_t g = g0 + tid;
    uint32_t steps = 0;
    int64_t ya = 0;
    if (g < nev) {
      const Ev e = ev[g];
      ya = (int64_t)da[e.rec];
      const int64_t yp = g == 1 ? -U : (int64_t)da[ev[g - 1].rec];
      const int64_t E = ya + (int64_t)e.pad;
      steps = (uint32_t)((uint64_t)(E - yp - (int64_t)kL) / kM + 1);
    }
    uint32_t incl = steps;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t t = (uint32_t)__shfl_up((int)incl, d, 64);
      if (lane >= (uint32_t)d) incl += t;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t wb = 0, tot = 0;
    for (uint32_t k = 0; k < 16; ++k) {
      if (k < wave) wb += s_w[k];
      tot += s_w[k];
    }
    if (g < nev) {
      ev[g].blk = kb + wb + incl;
      ev[g].ya = ya;
    }
    if (tid == 0) s_tot = tot;
    __syncthreads();
    kb += s_tot;
    __syncthreads();
  }
  if (tid == 0) {
    const int64_t ya = nev > 1 ? (int64_t)da[ev[nev - 1].rec] : -U;
    if (N == 0) {
      X[2] = b0 - 1;  // no blocks
      X[3] = 40 + b0 * kL + (uint64_t)U;
    } else {
      // the block whose end E_k >= A_N first: E_kb = ya + L, E_{kb+m} = ya + L + m M
      const int64_t over = (int64_t)AN - ya - (int64_t)kL;
      const uint64_t m = over > 0 ? ((uint64_t)over + kM - 1) / kM : 0;
      const uint64_t ke = kb + m;
      const int64_t Y = m == 0 ? ya : ya + (int64_t)kL + (int64_t)(m - 1) * kM;
      const uint64_t c = m == 0 ? 0 : 1;
      X[2] = ke;
      X[3] = 40 + ke * kL + kHdr * c + (uint64_t)((int64_t)AN - Y);
    }
  }
}

// file offset WriteRecord returns for dense record j (wal.go:514-516): its header position
__device__ __forceinline__ uint64_t rec_phys(const Ev& e, uint32_t g, uint64_t j, uint64_t aj) {
  if (g >= 1 && e.rec == j) return 40 + e.blk * kL;
  const int64_t rel = (int64_t)aj - e.ya;
  if (rel < (int64_t)kL) return 40 + e.blk * kL + (uint64_t)rel;  // in the event block (c = 0)
  const uint64_t m = (uint64_t)(rel - (int64_t)kL) / kM;
  const int64_t Y = e.ya + (int64_t)kL + (int64_t)m * kM;
  return 40 + (e.blk + 1 + m) * kL + kHdr + (uint64_t)((int64_t)aj - Y);
}

__global__ __launch_bounds__(256) void k_recoff(const uint64_t* __restrict__ da, const uint32_t* __restrict__ dsrc,
                                                 const uint64_t* __restrict__ emisc, int lay, const Ev* __restrict__ ev,
                                                 const uint32_t* __restrict__ evb, uint64_t* __restrict__ dpos,
                                                 uint64_t* __restrict__ rec_off) {
  const uint64_t j = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t N = emisc[X_NDENSE];
  if (j >= N) return;
  const uint32_t nev = (uint32_t)emisc[X_LAY + lay * kLayStride + 1];
  uint32_t g = evb[j / kEvWin];
  while (g + 1 < nev && ev[g + 1].rec <= j) ++g;
  const uint64_t p = rec_phys(ev[g], g, j, da[j]);
  dpos[j] = p;
  if (rec_off) rec_off[dsrc[j]] = p;
}

// ------------------------------------------------------------------------------------------
// Payload programs: a record's payload as up to 6 pieces, each literal bytes (computed here, kept by a
// literal sink: a local array, or a thread's dword-interleaved slice of LDS) or a range of the source
// record's payload.
struct Prog {
  uint32_t len[6];
  uint64_t off[6];   // literal: offset into the literals; source: payload offset in the source record
  uint8_t src[6];
  uint32_t n;
};
struct LitLocal {  // a local array
  uint8_t* p;
  __device__ __forceinline__ void put(uint32_t k, uint32_t b) const { p[k] = (uint8_t)b; }
  __device__ __forceinline__ uint32_t get(uint32_t k) const { return p[k]; }
};
struct LitLds {  // byte k of thread t at dword (k / 4) * 256 + t: lanes at one k read consecutive dwords
  uint8_t* base;
  uint32_t t;
  __device__ __forceinline__ uint8_t* at(uint32_t k) const { return base + ((((k >> 2) << 8) + t) << 2) + (k & 3u); }
  __device__ __forceinline__ void put(uint32_t k, uint32_t b) const { *at(k) = (uint8_t)b; }
  __device__ __forceinline__ uint32_t get(uint32_t k) const { return *at(k); }
};
template <class LIT>
__device__ __forceinline__ uint32_t uvput_l(const LIT& l, uint32_t o, uint64_t v) {
  uint32_t n = 0;
  while (v >= 0x80) { l.put(o + n++, (uint32_t)(v | 0x80) & 0xffu); v >>= 7; }
  l.put(o + n++, (uint32_t)v);
  return n;
}

// Record.Encode (record.go:57-138) of source row i against the dst baseTime
template <class LIT>
__device__ void prog_record(const EncDev& e, uint64_t i, bool mdrop, Prog& p, const LIT& lit) {
  const bcw_record_table& t = e.t;
  const uint32_t flags = t.flags[i];
  const uint64_t klen = t.key_len[i], vlen = t.val_len[i], expire = t.expire[i];
  const uint64_t mlen = mdrop ? 0 : t.meta_len[i];
  const uint32_t el = (flags & 1u) ? 0u : e.etag;
  const uint32_t flag = (el == 0 ? 1u : 0u) | (flags & 4u) | (expire == 0 ? 2u : 0u);
  uint32_t o = 1;
  lit.put(o++, flag);
  o += uvput_l(lit, o, klen);
  o += uvput_l(lit, o, vlen);
  o += uvput_l(lit, o, mlen);
  const uint32_t vend = o;
  if (expire != 0) o += uvput_l(lit, o, expire - e.dst_base);
  const uint32_t hn = 1 + e.ns + (vend - 1) + el + (o - vend);
  lit.put(0, hn & 0xffu);  // byte(headerSize) (record.go:109)
  p.n = 6;
  p.src[0] = 0; p.len[0] = 1; p.off[0] = 0;
  p.src[1] = 1; p.len[1] = e.ns; p.off[1] = 1;
  p.src[2] = 0; p.len[2] = vend - 1; p.off[2] = 1;
  p.src[3] = 1; p.len[3] = el; p.off[3] = t.etag_off[i];
  p.src[4] = 0; p.len[4] = o - vend; p.off[4] = vend;
  p.src[5] = 1; p.len[5] = (uint32_t)(klen + vlen + mlen); p.off[5] = t.hdr_size[i];
}

// HintRecord.Encode (hint.go:32-48): ns | uvarint(len(key)) | key | uvarint fid | off | size
template <class LIT>
__device__ void prog_hint(const EncDev& e, uint64_t i, uint64_t off, uint64_t size, Prog& p, const LIT& lit) {
  const bcw_record_table& t = e.t;
  const uint64_t klen = t.key_len[i];
  uint32_t o = uvput_l(lit, 0, klen);
  const uint32_t k1 = o;
  o += uvput_l(lit, o, e.fid);
  o += uvput_l(lit, o, off);
  o += uvput_l(lit, o, size);
  p.n = 4;
  p.src[0] = 1; p.len[0] = e.ns; p.off[0] = 1;
  p.src[1] = 0; p.len[1] = k1; p.off[1] = 0;
  p.src[2] = 1; p.len[2] = (uint32_t)klen; p.off[2] = t.hdr_size[i];
  p.src[3] = 0; p.len[3] = o - k1; p.off[3] = k1;
  p.src[4] = p.src[5] = 0;
  p.len[4] = p.len[5] = 0;
  p.off[4] = p.off[5] = 0;
}

enum { PM_DST = 0, PM_HINT_DST = 1, PM_HINT_SRC = 2 };

// 16 source bytes at an arbitrary address from two aligned 16 B loads (caller checks bounds)
__device__ __forceinline__ uint4 shift16(uint4 v0, uint4 v1, uint32_t sh) {
  // named scalars and two select stages: an array indexed by w would be lowered to a scratch round trip
  const bool s2 = (sh & 8u) != 0, s1 = (sh & 4u) != 0;
  const uint32_t b0 = s2 ? v0.z : v0.x, b1 = s2 ? v0.w : v0.y, b2 = s2 ? v1.x : v0.z, b3 = s2 ? v1.y : v0.w,
                 b4 = s2 ? v1.z : v1.x, b5 = s2 ? v1.w : v1.y;
  const uint32_t c0 = s1 ? b1 : b0, c1 = s1 ? b2 : b1, c2 = s1 ? b3 : b2, c3 = s1 ? b4 : b3, c4 = s1 ? b5 : b4;
  const uint32_t b = sh & 3u;
  uint4 r;
  r.x = __builtin_amdgcn_alignbyte(c1, c0, b);
  r.y = __builtin_amdgcn_alignbyte(c2, c1, b);
  r.z = __builtin_amdgcn_alignbyte(c3, c2, b);
  r.w = __builtin_amdgcn_alignbyte(c4, c3, b);
  return r;
}

// source payload offset z -> file offset (regular records: closed form)
__device__ __forceinline__ uint64_t src_at(uint64_t d0, uint32_t l0, uint32_t start_off, uint64_t z, uint64_t& run) {
  if (z < l0) { run = l0 - z; return d0 + z; }
  const uint64_t zz = z - l0;
  const uint64_t q = zz / kM, r = zz - q * kM;
  const uint64_t blk0 = (d0 - start_off) / kL;
  run = kM - r;
  return (uint64_t)start_off + (blk0 + 1 + q) * kL + kHdr + r;
}

// ------------------------------------------------------------------------------------------
// k_write's per-record descriptor: the payload as materialised prefix bytes | one source range (the
// longest source piece: key+value+meta of a record, the key of a hint) | materialised suffix bytes.
// Records whose prefix + suffix exceed kWLit bytes (NsSize/EtagSize beyond ~60) are marked
// `general` and written by k_write_general instead.
//
// CRC combine (dst WAL records): the source fragments were CRC-verified by the decode, so each one's
// check word chk = ~unmask(stored) ^ A_{8n}(~0) is the raw CRC-32C R (init 0, no final inversion) of
// its data. With the source range running to the end of the source payload src (no suffix), the
// re-encoded payload is pre | src[h, n) (h = mid_off) and by linearity of R
//     R(pre | src[h, n)) = A_{8(n-h)}(R(pre) ^ R(src[0, h))) ^ R(src),
// R(src) = the source fragments' check words chained with shifts. R(pre) ^ R(src[0, h)) is the raw
// CRC of the two header strings right-aligned and XOR-ed (zero when the header is unchanged). The
// record's CRC (rcrc) is thus known before a byte of it is copied, and k_write only computes the
// CRC of the shorter piece of a record that the dst layout splits in two (the other piece follows
// from rcrc); `regular` bit 1 marks such records.
constexpr int kWLit = 92;
struct RecDescW {
  uint64_t d0;       // file offset of the data of the source payload's first fragment
  uint32_t l0;       // its length
  uint32_t f0, f1;   // source fragments
  uint32_t mid_off;  // source payload offset of the source range
  uint32_t mid_len;
  uint8_t npre, nsuf, regular, general;  // regular: bit 0 closed-form source addressing, bit 1 rcrc valid
  uint8_t lit[kWLit];  // prefix bytes, then suffix bytes
  uint32_t rcrc;       // raw CRC-32C of the whole re-encoded payload (regular bit 1)
};
static_assert(sizeof(RecDescW) == 128, "RecDescW layout");

template <int PM, class LIT>
__device__ __forceinline__ void prog_of(const EncDev& e, uint64_t j, uint64_t row, const uint64_t* __restrict__ dst_da,
                                        const uint64_t* __restrict__ dpos, const uint8_t* __restrict__ mflag, Prog& p,
                                        const LIT& lit) {
  if (PM == PM_DST) prog_record(e, row, mflag[row] != 0, p, lit);
  else if (PM == PM_HINT_DST) prog_hint(e, row, dpos[j], dst_da[j + 1] - dst_da[j] - kHdr, p, lit);
  else prog_hint(e, row, e.t.foff[row] - kHdr, e.t.size[row], p, lit);
}

// One thread per dense record. Byte work happens in LDS (a thread's bytes dword-interleaved with its
// neighbours', LitLds): the program's literals, the first 128 bytes of the source payload (staged with
// 16 B loads) and the descriptor under construction, which then leaves as 8 x 16 B stores.
template <int PM>
__global__ __launch_bounds__(256) void k_recdesc_w(EncDev e, const uint64_t* __restrict__ emisc,
                                                    const uint32_t* __restrict__ dsrc, const uint64_t* __restrict__ dst_da,
                                                    const uint64_t* __restrict__ dpos, const uint8_t* __restrict__ mflag,
                                                    const uint32_t* __restrict__ ops, RecDescW* __restrict__ rd) {
  __shared__ uint32_t t0[256];
  __shared__ uint32_t s_src[32 * 256];
  __shared__ uint32_t s_desc[32 * 256];
  __shared__ uint32_t s_plit[12 * 256];
  const uint32_t t = threadIdx.x;
  if (PM == PM_DST) {
    uint32_t c = t;
    for (int b = 0; b < 8; ++b) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    t0[t] = c;
  }
  __syncthreads();
  const uint64_t j = blockIdx.x * 256ull + t;
  if (j >= emisc[X_NDENSE]) return;
  const LitLds plit{reinterpret_cast<uint8_t*>(s_plit), t};
  const LitLds sl{reinterpret_cast<uint8_t*>(s_src), t};
  const LitLds dl{reinterpret_cast<uint8_t*>(s_desc), t};
  const uint64_t row = dsrc[j];
  Prog p;
  prog_of<PM>(e, j, row, dst_da, dpos, mflag, p, plit);
  const SrcRec sr = src_rec(e.t, e.frags, row);
  const Frag F0 = e.frags[sr.f0];
  const uint64_t d0 = frag_file(F0, e.start_off);
  const uint32_t l0 = F0.len;
  bool reg = true;
  for (uint32_t f = sr.f0 + 1; f <= sr.f1 && reg; ++f) {
    const Frag F = e.frags[f];
    reg = F.blk == F0.blk + (f - sr.f0) && F.start == kHdr && (f == sr.f1 || F.len == kM);
  }
  // the source payload's first bytes (those of its first fragment) -> LDS
  const uint32_t nst = l0 < 128u ? l0 : 128u;
  if (d0 + 128 <= e.src_len) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint4 v;
      __builtin_memcpy(&v, e.seg + d0 + 16 * k, 16);
      s_src[(4 * k + 0) * 256 + t] = v.x;
      s_src[(4 * k + 1) * 256 + t] = v.y;
      s_src[(4 * k + 2) * 256 + t] = v.z;
      s_src[(4 * k + 3) * 256 + t] = v.w;
    }
  } else {
    for (uint32_t k = 0; k < nst; ++k) sl.put(k, e.seg[d0 + k]);
  }
  auto srcb = [&](uint64_t z) -> uint32_t {
    if (z < nst) return sl.get((uint32_t)z);
    if (reg) {
      uint64_t run;
      return e.seg[src_at(d0, l0, e.start_off, z, run)];
    }
    return src_byte(e.seg, e.frags, e.start_off, sr, z);
  };
  // the source range: the longest source piece (none: everything is prefix)
  uint32_t m = 6, ml = 0;
  uint64_t moff = 0;
#pragma unroll
  for (int q = 0; q < 6; ++q)
    if ((uint32_t)q < p.n && p.src[q] && p.len[q] > ml) { m = q; ml = p.len[q]; moff = p.off[q]; }
  uint32_t npre = 0, nsuf = 0;
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    if ((uint32_t)q >= p.n) continue;
    if ((uint32_t)q < m) npre += p.len[q];
    else if ((uint32_t)q > m) nsuf += p.len[q];
  }
  const bool general = npre + nsuf > (uint32_t)kWLit;
#pragma unroll
  for (int k = 8; k < 32; ++k) s_desc[k * 256 + t] = 0;  // literal bytes (and rcrc)
  if (!general) {
    uint32_t o = 32;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      if ((uint32_t)q >= p.n || (uint32_t)q == m) continue;
      const bool sq = p.src[q] != 0;
      const uint64_t oq = p.off[q];
      for (uint32_t b = 0; b < p.len[q]; ++b) dl.put(o++, sq ? srcb(oq + b) : plit.get((uint32_t)(oq + b)));
    }
  }
  uint32_t regular = reg ? 1u : 0u, rcrc = 0;
  if (PM == PM_DST && !general && nsuf == 0 && m < 6 && moff + ml == e.t.size[row]) {
    // R(pre) ^ R(src[0, h)): both header strings right-aligned to hl bytes, XOR-ed, one CRC pass
    const uint32_t h = (uint32_t)moff, hl = npre > h ? npre : h;
    uint32_t x = 0;
    for (uint32_t b = 0; b < hl; ++b) {
      uint32_t z = b + npre >= hl ? dl.get(32 + b + npre - hl) : 0u;
      if (b + h >= hl) z ^= srcb(b + h - hl);
      x = (x >> 8) ^ t0[(x ^ z) & 0xffu];
    }
    const uint32_t* p2 = ops + kOpPow2 * 128;
    uint32_t cs = 0;  // R(src): the source fragments' check words, chained
    for (uint32_t f = sr.f0; f <= sr.f1; ++f) {
      const Frag F = e.frags[f];
      cs = shift_by(p2, cs, F.len) ^ F.chk;
    }
    rcrc = shift_by(p2, x, ml) ^ cs;
    regular |= 2u;
  }
  s_desc[0 * 256 + t] = (uint32_t)d0;
  s_desc[1 * 256 + t] = (uint32_t)(d0 >> 32);
  s_desc[2 * 256 + t] = l0;
  s_desc[3 * 256 + t] = sr.f0;
  s_desc[4 * 256 + t] = sr.f1;
  s_desc[5 * 256 + t] = m < 6 ? (uint32_t)moff : 0u;
  s_desc[6 * 256 + t] = ml;
  s_desc[7 * 256 + t] = (general ? 0u : npre) | ((general ? 0u : nsuf) << 8) | (regular << 16) | ((general ? 1u : 0u) << 24);
  s_desc[31 * 256 + t] = rcrc;
  uint4* dst = reinterpret_cast<uint4*>(rd + j);
#pragma unroll
  for (int k = 0; k < 8; ++k)
    dst[k] = make_uint4(s_desc[(4 * k) * 256 + t], s_desc[(4 * k + 1) * 256 + t], s_desc[(4 * k + 2) * 256 + t],
                        s_desc[(4 * k + 3) * 256 + t]);
}

// ------------------------------------------------------------------------------------------
// k_write: the record-parallel WAL writer (Wal.WriteRecord wal.go:505-549) for the dst records k_wcopy
// does not take. One 16-lane group per record, persistent groups striding over the records. A record's fragments
// follow in closed form from its header offset (data up to the block end, continuation headers at
// block starts). A fragment's data is cut into 16 B units aligned to the output address; lane l
// takes k = ceil(units/64) consecutive units (one pass per fragment) and, per unit:
//   fetch   the bytes from the source payload: a lane whose units all lie in the record's source
//           range of one source fragment streams aligned 16 B loads (kWBatch in flight) and shifts
//           each unit out of two neighbours; edge units (fragment ends, literal prefix/suffix, a source
//           fragment boundary) assemble up to four masked pieces;
//   store   one 16 B store, or single bytes for the units at the fragment edges;
//   CRC     a raw CRC-32C chain over its units (slice-by-8, bytes outside the fragment zeroed).
// Each lane's chain is shifted to the end of the fragment's last unit by A_{8*16*d} (d = units after
// it, three nibble operator stages), XOR-ed over the wave, and the zero bytes after the fragment end
// are undone by A_{8t}^-1. Lanes 0..6 then write the header (ComputeCRC32 utils.go:24-29 of the data,
// length, type). The zero pad before a record that starts a block (wal.go:509-512) is written by that
// record.
constexpr int kWT = 512;
constexpr int kWopStride = 144;  // shift-operator tables 16 words apart in bank space: lanes with
                                 // different operators collide only on equal nibbles
constexpr int kWRounds = 3;      // rounds of units whose source loads are in flight together

// one output WAL of a k_write launch
struct WLay {
  const uint64_t* da;    // the layout's y-coordinates (dense, N+1)
  const uint64_t* fpos;  // file offset of each dense record's first header in this layout
  const void* rd;        // RecDescW per dense record
  uint8_t* out;
  uint64_t pos, cap;     // file offset of out[0]; out capacity
  uint32_t lay;          // layout slot in emisc
};

// the layout has blocks and fits the output (otherwise nothing is written; the result says so)
__device__ __forceinline__ bool lay_ok(const uint64_t* __restrict__ emisc, const WLay& w) {
  const uint64_t* X = emisc + X_LAY + w.lay * kLayStride;
  return !(X[2] == X[4] - 1 || X[3] - w.pos > w.cap);
}

struct WArgs {
  EncDev e;
  WLay w[2];              // dst WAL and hint WAL of a compaction (nlay = 2), or the hint WAL
  uint32_t nlay;
  const uint64_t* emisc;
  const uint32_t* wops;   // enc_ops (layout in bcw_internal.h)
  const uint32_t* initc;  // A_{8L}(0xFFFFFFFF)
  uint32_t abl;           // measurement-only ablations of k_wcopy (BCW_ENC_ABL bits 4/8/16); 0 in the product
  uint32_t* wl;           // [rows] k_wcopy's leftover dst records: k_write<16>'s from the front, k_write_general's
  uint64_t rows;          //   from the back (counts in emisc[X_WL16], emisc[X_WLG])
  uint64_t* wcnt;         // emisc + X_WL16
};

__device__ __forceinline__ uint64_t blk_end(uint64_t P) { return P + kL - (P - 40) % kL; }

// the records k_wcopy writes (the others go to k_write): regular source, rcrc valid, not general, at
// most two dst fragments
__device__ __forceinline__ bool wcopy_item(uint32_t h1w, uint64_t P, uint64_t len) {
  if (((h1w >> 16) & 3u) != 3u || (h1w >> 24) != 0) return false;  // regular source, rcrc, not general
  const uint64_t x1 = blk_end(P) - (P + kHdr);
  return len <= x1 || len - x1 <= kM;
}

// file offset just past a record whose first header is at P, with a payload of len > 0 bytes
__device__ __forceinline__ uint64_t rec_end(uint64_t P, uint64_t len) {
  const uint64_t be = blk_end(P), ds = P + kHdr;
  if (ds + len <= be) return ds + len;
  const uint64_t rem = len - (be - ds);
  const uint64_t q = (rem - 1) / kM;  // whole continuation blocks before the last fragment
  return be + q * kL + kHdr + (rem - q * kM);
}

__device__ __forceinline__ uint32_t sel_byte(uint4 v, uint32_t b) {
  const uint32_t w = (b & 8u) ? ((b & 4u) ? v.w : v.z) : ((b & 4u) ? v.y : v.x);
  return (w >> (8 * (b & 3u))) & 0xffu;
}

// bytes [lo, hi) of a 16 B unit
__device__ __forceinline__ uint4 range_mask(int32_t lo, int32_t hi) {
  uint32_t m[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int32_t a = min(max(lo - 4 * k, 0), 4), b = min(max(hi - 4 * k, 0), 4);
    m[k] = (uint32_t)(((1ull << (8 * b)) - 1) & ~((1ull << (8 * a)) - 1));
  }
  return make_uint4(m[0], m[1], m[2], m[3]);
}

// 16 bytes of a wave's staged literals starting at literal offset o (-16 < o <= kWLit)
constexpr int kWLitWords = (16 + kWLit + 32) / 4;
__device__ __forceinline__ uint4 lit_window(const uint32_t* __restrict__ sl, int32_t o) {
  const uint32_t base = (uint32_t)(16 + o), w = base >> 2, sh = base & 3u;
  const uint32_t x0 = sl[w], x1 = sl[w + 1], x2 = sl[w + 2], x3 = sl[w + 3], x4 = sl[w + 4];
  return make_uint4(__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                    __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh));
}

// CRC-32C state after 16 more bytes (raw, slice-by-8: t8[256 k + b] = CRC of byte b and k zeros)
__device__ __forceinline__ uint32_t crc_step16(const uint32_t* __restrict__ t8, uint32_t c, uint4 v) {
  uint32_t x = c ^ v.x, y = v.y;
  c = t8[1792 + (x & 0xffu)] ^ t8[1536 + ((x >> 8) & 0xffu)] ^ t8[1280 + ((x >> 16) & 0xffu)] ^ t8[1024 + (x >> 24)] ^
      t8[768 + (y & 0xffu)] ^ t8[512 + ((y >> 8) & 0xffu)] ^ t8[256 + ((y >> 16) & 0xffu)] ^ t8[y >> 24];
  x = c ^ v.z;
  y = v.w;
  return t8[1792 + (x & 0xffu)] ^ t8[1536 + ((x >> 8) & 0xffu)] ^ t8[1280 + ((x >> 16) & 0xffu)] ^ t8[1024 + (x >> 24)] ^
         t8[768 + (y & 0xffu)] ^ t8[512 + ((y >> 8) & 0xffu)] ^ t8[256 + ((y >> 16) & 0xffu)] ^ t8[y >> 24];
}

// 16 source bytes starting at file offset S (two aligned loads; the caller checks the bounds)
__device__ __forceinline__ uint4 src16(const uint8_t* __restrict__ seg, uint64_t S) {
  const uint64_t Ba = S & ~15ull;
  const uint4 v0 = *reinterpret_cast<const uint4*>(seg + Ba);
  const uint4 v1 = *reinterpret_cast<const uint4*>(seg + Ba + 16);
  return shift16(v0, v1, (uint32_t)(S & 15u));
}

__device__ __forceinline__ void or_masked(uint4& v, uint4 q, uint4 m) {
  v.x |= q.x & m.x;
  v.y |= q.y & m.y;
  v.z |= q.z & m.z;
  v.w |= q.w & m.w;
}

// value of the next lane in the same row of 16 (lane 15: lane 0), DPP row_ror:15
__device__ __forceinline__ uint32_t rot16(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x12f, 0xf, 0xf, false);
}
__device__ __forceinline__ uint64_t rot16_u64(uint64_t x) {
  return (uint64_t)rot16((uint32_t)x) | ((uint64_t)rot16((uint32_t)(x >> 32)) << 32);
}
__device__ __forceinline__ uint4 rot16_u4(uint4 v) { return make_uint4(rot16(v.x), rot16(v.y), rot16(v.z), rot16(v.w)); }

// per-record view for the unit assembly
struct WRec {
  uint64_t d0;
  uint32_t l0;
  SrcRec sr;
  uint32_t mid_off;
  int64_t zA, zB;  // payload offsets of the source range
  int32_t npre;
  bool regular;
};

// bytes [b0, b1) of the unit whose byte 0 is payload offset zb (other bytes 0): literal prefix,
// source range (at most two source fragments: every fragment after the first holds M >= 16 bytes),
// literal suffix
__device__ __forceinline__ uint4 unit_general(const EncDev& e, const WRec& R, const uint32_t* __restrict__ sl,
                                              int64_t zb, int32_t b0, int32_t b1) {
  const int32_t pm = (int32_t)min(max(R.zA - zb, (int64_t)b0), (int64_t)b1);  // prefix [b0, pm)
  const int32_t mm = (int32_t)min(max(R.zB - zb, (int64_t)b0), (int64_t)b1);  // source [pm, mm), suffix [mm, b1)
  uint4 v = make_uint4(0, 0, 0, 0);
  if (pm < mm) {
    const uint64_t zs = R.mid_off + (uint64_t)(zb + pm - R.zA);  // source payload offset of byte pm
    bool done = false;
    if (R.regular) {
      uint64_t run;
      const uint64_t S = src_at(R.d0, R.l0, e.start_off, zs, run);
      const int32_t m1 = (int32_t)min((uint64_t)mm, (uint64_t)pm + run);  // first source run [pm, m1)
      if (S >= (uint64_t)pm && ((S - pm) & ~15ull) + 32 <= e.src_len) {
        or_masked(v, src16(e.seg, S - pm), range_mask(pm, m1));
        done = true;
        if (m1 < mm) {
          uint64_t run2;
          const uint64_t S2 = src_at(R.d0, R.l0, e.start_off, zs + (uint64_t)(m1 - pm), run2);
          if (S2 >= (uint64_t)m1 && ((S2 - m1) & ~15ull) + 32 <= e.src_len) or_masked(v, src16(e.seg, S2 - m1), range_mask(m1, mm));
          else done = false;
        }
      }
    }
    if (!done) {
      uint32_t w[4] = {0, 0, 0, 0};
      for (int32_t b = pm; b < mm; ++b) {
        const uint32_t by = src_byte(e.seg, e.frags, e.start_off, R.sr, zs + (uint64_t)(b - pm));
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if ((b >> 2) == k) w[k] |= by << (8 * (b & 3));
      }
      v = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
  if (b0 < pm) or_masked(v, lit_window(sl, (int32_t)zb), range_mask(b0, pm));
  if (mm < b1) or_masked(v, lit_window(sl, (int32_t)(zb - R.zB + R.npre)), range_mask(mm, b1));
  return v;
}

template <int kG>
__global__ __launch_bounds__(kWT) void k_write(WArgs A) {
  // the dst records k_wcopy listed (usually none: then every workgroup leaves before building its tables)
  const uint64_t nitems = A.wcnt[0];
  if ((uint64_t)blockIdx.x * (kWT / kG) >= nitems) return;
  const EncDev& e = A.e;
  __shared__ uint32_t t8[8 * 256];
  __shared__ uint32_t sop[40 * kWopStride];  // A_{8*16*n}, A_{8*256*n} (n < 16), A_{8*4096*n} (n < 8)
  __shared__ uint32_t sinv[16 * 128];        // A_{8t}^-1
  __shared__ uint32_t sp2[2][15 * 128];      // A_{8*2^k}, A_{8*2^k}^-1 (k < 15): the CRC combine
  __shared__ uint32_t s_lit[kWT / kG][kWLitWords];
  const uint32_t tid = threadIdx.x, lane = tid & 63, gl = tid & (kG - 1), gb = lane & ~(uint32_t)(kG - 1);
  for (uint32_t i = tid; i < 256; i += kWT) {
    uint32_t c = i;
    for (int b = 0; b < 8; ++b) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    t8[i] = c;
  }
  for (uint32_t i = tid; i < 40 * 128; i += kWT) sop[(i >> 7) * kWopStride + (i & 127u)] = A.wops[i];
  for (uint32_t i = tid; i < 16 * 128; i += kWT) sinv[i] = A.wops[kOpInv * 128 + i];
  for (uint32_t i = tid; i < 15 * 128; i += kWT) {
    sp2[0][i] = A.wops[kOpPow2 * 128 + i];
    sp2[1][i] = A.wops[kOpPow2Inv * 128 + i];
  }
  for (uint32_t i = tid; i < (kWT / kG) * kWLitWords; i += kWT) (&s_lit[0][0])[i] = 0;
  __syncthreads();
  for (uint32_t i = tid; i < 256; i += kWT) {
    uint32_t c = t8[i];
    for (int k = 1; k < 8; ++k) { c = (c >> 8) ^ t8[c & 0xffu]; t8[256 * k + i] = c; }
  }
  __syncthreads();
  uint32_t* sl = s_lit[tid / kG];
  const uint64_t ng = (uint64_t)gridDim.x * (kWT / kG);    // groups in the grid
  const uint64_t g0 = (uint64_t)blockIdx.x * (kWT / kG) + tid / kG;
  const bool ok0 = lay_ok(A.emisc, A.w[0]), ok1 = A.nlay > 1 && lay_ok(A.emisc, A.w[1]);
  const uint32_t* hop = sop + (kG < 16 ? kG : 16 + kG / 16) * kWopStride;  // A_{8*16*kG}: one round of the group

  // items: the listed dst records, one per group of kG lanes. An item's descriptor is loaded one item ahead:
  // the RecDescW spread over the group's lanes 0-7 (header, then the literal bytes), da[j], da[j+1] and fpos[j]
  // in every lane.
  static_assert(kG == 16, "group size: the DPP row rotation shares source blocks within rows of 16 lanes");
  struct Pre {
    uint4 q;
    uint64_t a0, a1, fp, j;
  };
  auto fetch = [&](uint64_t it2, Pre& p) {
    p.q = make_uint4(0, 0, 0, 0);
    p.a0 = p.a1 = p.fp = p.j = 0;
    if (it2 >= nitems) return;
    const uint64_t j2 = A.wl[it2];
    const WLay& W2 = A.w[0];
    if (gl < 8) p.q = reinterpret_cast<const uint4*>(static_cast<const RecDescW*>(W2.rd) + j2)[gl];
    p.a0 = W2.da[j2];
    p.a1 = W2.da[j2 + 1];
    p.fp = W2.fpos[j2];
    p.j = j2;
  };
  // the group's lane k holds word x
  auto gw = [&](uint32_t x, uint32_t k) { return (uint32_t)__shfl((int)x, (int)(gb + k), 64); };
  Pre pn;
  fetch(g0, pn);
  for (uint64_t it = g0; it < nitems; it += ng) {
    const Pre pc = pn;
    const uint4 qc = pc.q;
    fetch(it + ng, pn);  // in flight while this item is written
    const uint32_t li = 0;
    const uint64_t j = pc.j;
    const WLay& Ly = li ? A.w[1] : A.w[0];
    if (!(li ? ok1 : ok0)) continue;  // nothing to write / does not fit (the result says so)
    const uint32_t h1w = gw(qc.w, 1);
    if ((h1w >> 24) != 0) continue;  // general record: k_write_general
    uint8_t* const out = Ly.out;
    const uint64_t pos = Ly.pos;
    const uint64_t obase = (uint64_t)(uintptr_t)out;
    const uint64_t P = pc.fp;
    const uint64_t aj = pc.a0;
    const uint64_t len = pc.a1 - aj - kHdr;
    if (li == 0 && wcopy_item(h1w, P, len)) continue;  // k_wcopy
    WRec R;
    R.d0 = (uint64_t)gw(qc.x, 0) | ((uint64_t)gw(qc.y, 0) << 32);
    R.l0 = gw(qc.z, 0);
    R.sr.f0 = gw(qc.w, 0);
    R.sr.f1 = gw(qc.x, 1);
    R.mid_off = gw(qc.y, 1);
    R.npre = (int32_t)(h1w & 0xffu);
    R.zA = R.npre;
    R.zB = (int64_t)R.npre + gw(qc.z, 1);
    R.regular = ((h1w >> 16) & 1u) != 0;
    const uint32_t rcrc = gw(qc.w, 7);
    // stage the literal bytes in LDS (group-private; the previous record's reads are done: LDS
    // executes a wave's operations in order)
    if (gl >= 2 && gl < 8) {
      uint32_t* d = sl + 4 + 4 * (gl - 2);
      d[0] = qc.x;
      d[1] = qc.y;
      d[2] = qc.z;
      d[3] = qc.w;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // zero pad before a record that starts a block (at most 6 bytes)
    if ((P - 40) % kL == 0) {
      const uint64_t prev = j == 0 ? pos : rec_end(Ly.fpos[j - 1], aj - Ly.da[j - 1] - kHdr);
      if (prev + gl < P) out[prev + gl - pos] = 0;
    }

    // CRC combine (see RecDescW): a record in one dst fragment takes rcrc; one split in two computes the
    // shorter piece's CRC and derives the other's, R(data) = A_{8y}(R(First)) ^ R(Last) (y = |Last|)
    const uint64_t x1 = blk_end(P) - (P + kHdr);  // room in the first block
    const uint32_t nfr = len <= x1 ? 1u : (len - x1 <= kM ? 2u : 3u);
    const bool comb = ((h1w >> 17) & 1u) != 0 && nfr <= 2;
    const bool direct_first = len - x1 >= x1;  // (two pieces) the First is the shorter one
    uint32_t a_first = 0;
    uint64_t h_first = 0;
    uint64_t hp = P, x0 = 0;
    for (bool first = true;; first = false) {  // (a zero-length First leaves x0 at 0)
      const uint64_t be = blk_end(hp), ds = hp + kHdr;
      const uint64_t rem = len - x0;
      const uint64_t flen = rem < be - ds ? rem : be - ds;
      const bool last = flen == rem;
      const uint32_t type = first ? (last ? BCW_RECORD_FULL : BCW_RECORD_FIRST)
                                  : (last ? BCW_RECORD_LAST : BCW_RECORD_MIDDLE);
      const uint32_t ic = A.initc[flen];  // in flight during the pass
      const bool crc_on = !comb || (nfr == 2 && first == direct_first);
      uint32_t acc = 0;
      if (flen) {
        const uint64_t as = obase + (ds - pos), ae = as + flen;  // output addresses of the data
        const uint64_t uf = as >> 4, ul = (ae - 1) >> 4;
        const uint32_t nunits = (uint32_t)(ul - uf + 1);
        // lane gl takes units gl, gl + kG, ...: per lane a Horner chain acc = A_{8*16*kG}(acc) ^ crc(unit).
        // Interior units of the source range advance their source address incrementally (S, run:
        // bytes left in that source fragment); edge units go through unit_general.
        uint32_t c = 0;
        const uint32_t rlast = nunits - 1;
        int64_t zb = (int64_t)x0 + (int64_t)((uf + gl) << 4) - (int64_t)as;  // payload offset of unit byte 0
        uint64_t S = 0;
        int64_t run = -1;
        constexpr int64_t kStep = 16 * kG;
        for (uint32_t r0 = gl; r0 - gl < nunits; r0 += kG * kWRounds) {
          // source of the fast units: one aligned block per lane and round; the block after it is the
          // next lane's (lane 15: lane 0's of the next round, or its own extra load in the last round),
          // moved over with a DPP row rotation. Units whose neighbour block is not contiguous take the
          // general path.
          uint4 blk[kWRounds], tail = make_uint4(0, 0, 0, 0);
          uint64_t Bq[kWRounds];
          uint32_t shv[kWRounds];
          bool fast[kWRounds];
#pragma unroll
          for (int q = 0; q < kWRounds; ++q) {
            const uint32_t r = r0 + kG * q;
            const int64_t z = zb + kStep * q;
            fast[q] = false;
            shv[q] = 0;
            Bq[q] = ~0ull;
            blk[q] = make_uint4(0, 0, 0, 0);
            if (r < rlast && r != 0 && R.regular && z >= R.zA && z + 16 <= R.zB) {
              if (run < 16) {
                uint64_t ru;
                S = src_at(R.d0, R.l0, e.start_off, R.mid_off + (uint64_t)(z - R.zA), ru);
                run = (int64_t)ru;
              }
              if (run >= 16 && (S & ~15ull) + 32 <= e.src_len) {
                Bq[q] = S & ~15ull;
                blk[q] = *reinterpret_cast<const uint4*>(e.seg + Bq[q]);
                shv[q] = (uint32_t)(S & 15u);
                fast[q] = true;
              }
            } else {
              run = -1;
            }
            S += kStep;
            run -= kStep;
          }
          if (gl == kG - 1 && fast[kWRounds - 1]) tail = *reinterpret_cast<const uint4*>(e.seg + Bq[kWRounds - 1] + 16);
          uint64_t nbB[kWRounds + 1];
#pragma unroll
          for (int q = 0; q < kWRounds; ++q) nbB[q] = rot16_u64(Bq[q]);
#pragma unroll
          for (int q = 0; q < kWRounds; ++q) {
            const uint64_t nb = gl == kG - 1 ? (q + 1 < kWRounds ? nbB[q + 1] : Bq[q] + 16) : nbB[q];
            fast[q] = fast[q] && nb == Bq[q] + 16;
          }
          uint4 rb[kWRounds];
#pragma unroll
          for (int q = 0; q < kWRounds; ++q) rb[q] = rot16_u4(blk[q]);
#pragma unroll
          for (int q = 0; q < kWRounds; ++q) {
            const uint32_t r = r0 + kG * q;
            if (r >= nunits) continue;
            const uint64_t ua = (uf + r) << 4;
            uint4 v;
            int32_t b0 = 0, b1 = 16;
            if (fast[q]) {
              const uint4 nx = gl == kG - 1 ? (q + 1 < kWRounds ? rb[q + 1] : tail) : rb[q];
              v = shift16(blk[q], nx, shv[q]);
            } else {
              b0 = ua < as ? (int32_t)(as - ua) : 0;
              b1 = ua + 16 > ae ? (int32_t)(ae - ua) : 16;
              v = unit_general(e, R, sl, zb + kStep * q, b0, b1);
            }
            uint8_t* d = reinterpret_cast<uint8_t*>((uintptr_t)ua);
            if (b1 - b0 == 16) {
              __builtin_nontemporal_store(v.x, reinterpret_cast<uint32_t*>(d));
              __builtin_nontemporal_store(v.y, reinterpret_cast<uint32_t*>(d) + 1);
              __builtin_nontemporal_store(v.z, reinterpret_cast<uint32_t*>(d) + 2);
              __builtin_nontemporal_store(v.w, reinterpret_cast<uint32_t*>(d) + 3);
            } else {
              for (int32_t b = b0; b < b1; ++b) d[b] = (uint8_t)sel_byte(v, (uint32_t)b);
            }
            if (crc_on) c = op_apply_s(hop, c) ^ crc_step16(t8, 0u, v);
          }
          zb += kStep * kWRounds;
        }
        if (crc_on) {
        // shift each lane's chain to the end of the fragment's last unit (d < kG units follow it)
        if (gl < nunits) {
          const uint32_t dn = (nunits - 1 - gl) & (kG - 1);
          if (dn & 15u) c = op_apply_s(sop + (dn & 15u) * kWopStride, c);
          if (dn >> 4) c = op_apply_s(sop + (16u + (dn >> 4)) * kWopStride, c);
        }
#pragma unroll
        for (int m = 1; m < kG; m <<= 1) c ^= __shfl_xor(c, m, 64);
        const uint32_t t = (uint32_t)(((ul + 1) << 4) - ae);
        acc = t ? op_apply_s(sinv + t * 128, c) : c;
        }
      }
      auto put_header = [&](uint64_t h, uint32_t r, uint32_t icv, uint64_t fl, uint32_t ty) {
        if (gl < kHdr) {
          const uint32_t crc = ~(r ^ icv);
          const uint32_t masked = ((crc >> 15) | (crc << 17)) + 0xa282ead8u;  // ComputeCRC32 (utils.go:24-29)
          const uint32_t by = gl < 4 ? (masked >> (8 * gl)) : gl == 4 ? (uint32_t)fl : gl == 5 ? (uint32_t)(fl >> 8) : ty;
          out[h - pos + gl] = (uint8_t)by;
        }
      };
      bool put = true;
      if (comb) {
        if (nfr == 1) {
          acc = rcrc;
        } else if (first) {
          if (direct_first) a_first = acc;
          else put = false;  // derived from the Last piece below
          h_first = hp;
        } else if (direct_first) {
          acc = rcrc ^ shift_by(sp2[0], a_first, flen);
        } else {
          const uint32_t af = shift_by(sp2[1], rcrc ^ acc, flen);  // A_{8y}^-1
          put_header(h_first, af, A.initc[x1], x1, BCW_RECORD_FIRST);
        }
      }
      if (put) put_header(hp, acc, ic, flen, type);
      x0 += flen;
      if (last) break;
      hp = be;
    }
  }
}

// The general records of k_write (literal bytes beyond kWLit): one thread per record, bytewise.
template <int PM>
__device__ void write_general_rec(const WArgs& WA, const WLay& A, uint64_t j, const uint32_t* __restrict__ dsrc,
                                  const uint64_t* __restrict__ dst_da, const uint64_t* __restrict__ dpos,
                                  const uint8_t* __restrict__ mflag, const uint32_t* t0, Prog& p, uint8_t* plit) {
  const EncDev& e = WA.e;
  const uint64_t row = dsrc[j];
  const LitLocal lit{plit};
  prog_of<PM>(e, j, row, dst_da, dpos, mflag, p, lit);
  const SrcRec sr = src_rec(e.t, e.frags, row);
  const uint64_t P = A.fpos[j];
  const uint64_t len = A.da[j + 1] - A.da[j] - kHdr;
  if ((P - 40) % kL == 0) {
    const uint64_t prev = j == 0 ? A.pos : rec_end(A.fpos[j - 1], A.da[j] - A.da[j - 1] - kHdr);
    for (uint64_t b = prev; b < P; ++b) A.out[b - A.pos] = 0;
  }
  uint64_t hp = P, z = 0;
  uint32_t q = 0;
  uint64_t qb = 0;  // payload offset of piece q
  for (bool first = true;; first = false) {
    const uint64_t be = blk_end(hp), ds = hp + kHdr;
    const uint64_t rem = len - z;
    const uint64_t flen = rem < be - ds ? rem : be - ds;
    const bool last = flen == rem;
    const uint32_t type = first ? (last ? BCW_RECORD_FULL : BCW_RECORD_FIRST)
                                : (last ? BCW_RECORD_LAST : BCW_RECORD_MIDDLE);
    uint32_t crc = 0xffffffffu;
    for (uint64_t i = 0; i < flen; ++i, ++z) {
      while (z >= qb + p.len[q]) { qb += p.len[q]; ++q; }
      const uint32_t by = p.src[q] ? src_byte(e.seg, e.frags, e.start_off, sr, p.off[q] + (z - qb))
                                   : plit[p.off[q] + (z - qb)];
      A.out[ds + i - A.pos] = (uint8_t)by;
      crc = (crc >> 8) ^ t0[(crc ^ by) & 0xffu];
    }
    crc = ~crc;
    const uint32_t masked = ((crc >> 15) | (crc << 17)) + 0xa282ead8u;
    uint8_t* h = A.out + (hp - A.pos);
    h[0] = (uint8_t)masked;
    h[1] = (uint8_t)(masked >> 8);
    h[2] = (uint8_t)(masked >> 16);
    h[3] = (uint8_t)(masked >> 24);
    h[4] = (uint8_t)flen;
    h[5] = (uint8_t)(flen >> 8);
    h[6] = (uint8_t)type;
    if (last) break;
    hp = be;
  }
}

// The records come from k_wcopy's work list (the back of wl, emisc[X_WLG] of them; usually none, and then every
// workgroup leaves at once); persistent grid. The payload program and its literals live in LDS (no scratch).
template <int PM>
__global__ __launch_bounds__(256) void k_write_general(WArgs WA, uint32_t li, const uint32_t* __restrict__ dsrc,
                                                        const uint64_t* __restrict__ dst_da,
                                                        const uint64_t* __restrict__ dpos,
                                                        const uint8_t* __restrict__ mflag) {
  const uint64_t nitems = WA.wcnt[1];
  if ((uint64_t)blockIdx.x * 256 >= nitems) return;
  const WLay A = li ? WA.w[1] : WA.w[0];
  __shared__ uint32_t t0[256];
  __shared__ Prog s_prog[256];
  __shared__ uint8_t s_plit[256][48];
  for (uint32_t i = threadIdx.x; i < 256; i += 256) {
    uint32_t c = i;
    for (int b = 0; b < 8; ++b) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    t0[i] = c;
  }
  __syncthreads();
  if (!lay_ok(WA.emisc, A)) return;
  for (uint64_t it = blockIdx.x * 256ull + threadIdx.x; it < nitems; it += (uint64_t)gridDim.x * 256)
    write_general_rec<PM>(WA, A, WA.wl[WA.rows - 1 - it], dsrc, dst_da, dpos, mflag, t0, s_prog[threadIdx.x],
                          s_plit[threadIdx.x]);
}


// ------------------------------------------------------------------------------------------
// k_wcopy: the dst WAL records whose CRC follows from rcrc (RecDescW `regular` bits 0 and 1) and that
// the dst layout puts in at most two fragments -- nearly every record of a compaction (k_write takes
// the others). One wave per record: the literal prefix is written with byte stores, the source range
// as runs (one per source fragment) of 16 B units aligned to the output, each from two aligned source
// loads funnel-shifted. A record split in two computes the raw CRC of its shorter piece (lane chunks,
// bytewise, shifted to the piece end and XOR-ed over the wave) and derives the other piece's from
// rcrc: R(data) = A_{8y}(R(First)) ^ R(Last).
constexpr int kCT = 256;
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
  return (uint64_t)uni((uint32_t)x) | ((uint64_t)uni((uint32_t)(x >> 32)) << 32);
}
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int kCU = 2;  // units per lane in flight (k_wcopy: 74 VGPRs, 6 waves per SIMD; 1, 3 and 4 measured equal)


// copy m bytes from src to dst (global pointers, any alignment), one wave. Every whole unit (16 B aligned to
// the output) takes its source bytes from two aligned 16 B loads; the partial units at the run's ends are written
// bytewise, one byte per lane, after the loop.
__device__ __forceinline__ void copy_run(uint8_t* dst, const uint8_t* src, uint64_t m, const uint8_t* seg,
                                         uint64_t seg_len, uint32_t lane) {
  if (m == 0) return;
  const uint64_t da = uni64((uint64_t)(uintptr_t)dst), de = da + uni64(m);
  const uint64_t u0 = da >> 4, nu = ((de - 1) >> 4) - u0 + 1;
  const uint64_t delta = uni64((uint64_t)(uintptr_t)src) - da;  // modular
  const uint64_t sbeg = uni64((uint64_t)(uintptr_t)seg), send = sbeg + uni64(seg_len);
  for (uint64_t k0 = 0; k0 < nu; k0 += 64 * kCU) {
    uint4 v[kCU];
    bool ok[kCU];
#pragma unroll
    for (int q = 0; q < kCU; ++q) {
      const uint64_t k = k0 + (uint64_t)q * 64 + lane;
      const uint64_t ua = (u0 + k) << 4;
      const uint64_t sa = ua + delta, sw = sa & ~15ull;
      v[q] = make_uint4(0, 0, 0, 0);
      ok[q] = k < nu && sw >= sbeg && sw + 32 <= send;
      if (ok[q]) {
        // addresses as offsets from the segment / output pointers (not integer-to-pointer casts): the compiler then
        // knows they are global memory and emits global_ (not flat_) loads and stores
        const uint4* w = reinterpret_cast<const uint4*>(seg + (sw - sbeg));
        v[q] = shift16(w[0], w[1], (uint32_t)(sa & 15u));
      }
    }
#pragma unroll
    for (int q = 0; q < kCU; ++q) {
      const uint64_t k = k0 + (uint64_t)q * 64 + lane;
      if (k >= nu) continue;
      const uint64_t ua = (u0 + k) << 4;
      uint8_t* d = dst + (int64_t)(ua - da);
      if (ua < da || ua + 16 > de) continue;  // a partial unit at the run's ends: below, one byte per lane
      if (ok[q]) {  // one 16 B non-temporal store (d is 16 B aligned)
        const v4u w = {v[q].x, v[q].y, v[q].z, v[q].w};
        __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(d));
      } else {  // the source window touches the segment's ends: bytewise
        for (uint32_t b = 0; b < 16u; ++b) d[b] = seg[(int64_t)(ua + b + delta - sbeg)];
      }
    }
  }
  // the bytes of the partial units at the run's two ends (at most 15 + 15), one per lane: lanes [0, n0) the first
  // unit's from the run's start, lanes [n0, n0 + n1) the last unit's up to its end (as a byte loop per end lane these
  // took ~2.4 of the writer phase's ~25 ms at config E: up to 15 dependent iterations for two lanes)
  const uint64_t ulast = (de - 1) & ~15ull;
  const uint32_t n0 = (da & 15u) ? (uint32_t)(min(de, (da & ~15ull) + 16) - da) : 0u;
  const uint32_t n1 = ((de & 15u) && ulast >= da + n0) ? (uint32_t)(de - ulast) : 0u;
  if (lane < n0 + n1) {
    const uint64_t off = lane < n0 ? lane : (ulast - da) + (lane - n0);  // run-relative byte
    dst[off] = seg[(int64_t)(da + off + delta - sbeg)];
  }
}

// 7 waves per SIMD (71 VGPRs, no spills): 24.0 vs 24.3 ms per encode at the natural 6 (74 VGPRs); 8 waves spill
__global__ __launch_bounds__(kCT) __attribute__((amdgpu_waves_per_eu(7, 7))) void k_wcopy(WArgs A) {
  __shared__ uint32_t t0[256];
  __shared__ uint32_t ts[3][256];        // slice-by-4: T_k[i] = T_{k-1}[i] >> 8 ^ t0[T_{k-1}[i] & 0xff], k = 1..3
  __shared__ uint32_t sp2[2][15 * 128];  // A_{8*2^k}, A_{8*2^k}^-1
  __shared__ uint32_t s_desc[kCT / 64][32];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  {
    uint32_t c = tid;
    for (int b = 0; b < 8; ++b) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    t0[tid] = c;
  }
  for (uint32_t i = tid; i < 15 * 128; i += kCT) {
    sp2[0][i] = A.wops[kOpPow2 * 128 + i];
    sp2[1][i] = A.wops[kOpPow2Inv * 128 + i];
  }
  __syncthreads();
  {
    uint32_t c = t0[tid];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      c = (c >> 8) ^ t0[c & 0xffu];
      ts[k][tid] = c;
    }
  }
  __syncthreads();
  const WLay& W = A.w[0];
  if (!lay_ok(A.emisc, W)) return;
  const EncDev& e = A.e;
  const uint64_t N = A.emisc[X_NDENSE];
  uint32_t* sd = s_desc[wave];
  const uint8_t* lit = reinterpret_cast<const uint8_t*>(sd) + 32;
  uint8_t* const out = W.out;
  const uint64_t pos = W.pos;
  const uint64_t nw = (uint64_t)gridDim.x * (kCT / 64);
  // the next record's descriptor word (lanes 0..31), header offset and y-coordinates, one record ahead
  uint32_t ndw = 0;
  uint64_t nP = 0, na0 = 0, na1 = 0;
  auto fetch = [&](uint64_t jj) {
    if (jj >= N) return;
    ndw = lane < 32 ? reinterpret_cast<const uint32_t*>(static_cast<const RecDescW*>(W.rd) + jj)[lane] : 0u;
    nP = W.fpos[jj];
    na0 = W.da[jj];
    na1 = W.da[jj + 1];
  };
  fetch((uint64_t)blockIdx.x * (kCT / 64) + wave);
  for (uint64_t j = (uint64_t)blockIdx.x * (kCT / 64) + wave; j < N; j += nw) {
    const uint32_t dw = ndw;
    const uint64_t P = uni64(nP), aj = uni64(na0), len = uni64(na1) - aj - kHdr;
    fetch(j + nw);
    const uint32_t h1w = uni((uint32_t)__shfl((int)dw, 7, 64));
    if (!wcopy_item(h1w, P, len)) {  // k_write<16>'s or, with long literals, k_write_general's
      if (lane == 0) {
        if ((h1w >> 24) != 0) A.wl[A.rows - 1 - atomicAdd((unsigned long long*)&A.wcnt[1], 1ull)] = (uint32_t)j;
        else A.wl[atomicAdd((unsigned long long*)&A.wcnt[0], 1ull)] = (uint32_t)j;
      }
      continue;
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < 32) sd[lane] = dw;  // the previous record's reads are done (LDS keeps a wave's order)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t d0 = uni64((uint64_t)sd[0] | ((uint64_t)sd[1] << 32));
    const uint32_t l0 = uni(sd[2]), mid_off = uni(sd[5]), npre = h1w & 0xffu, rcrc = uni(sd[31]);
    // zero pad before a record that starts a block (wal.go:509-512)
    if ((P - 40) % kL == 0) {
      const uint64_t prev = j == 0 ? pos : rec_end(W.fpos[j - 1], aj - W.da[j - 1] - kHdr);
      if (prev + lane < P) out[prev + lane - pos] = 0;
    }
    const uint64_t be = blk_end(P), x1 = be - (P + kHdr);
    const uint32_t nfr = len <= x1 ? 1u : 2u;
    uint32_t cr0 = rcrc, cr1 = 0;
    if (nfr == 2 && !(A.abl & 16)) {
      // the shorter piece's raw CRC: lane chunks of [pa, pb) (whole 16 B units of the payload, loaded
      // up to kPU at a time), each chunk's CRC shifted to pb
      const bool df = len - x1 >= x1;
      const uint64_t pa = df ? 0 : x1, pb = df ? x1 : len;
      const uint64_t c = (((pb - pa + 63) / 64) + 15) & ~15ull;
      const uint64_t a0 = pa + lane * c, a1 = a0 + c < pb ? a0 + c : pb;
      uint32_t x = 0;
      constexpr int kPU = 4;
      for (uint64_t zb = a0; zb < a1; zb += 16 * kPU) {
        uint4 u[kPU];
#pragma unroll
        for (int q = 0; q < kPU; ++q) {
          const uint64_t z = zb + 16 * q;
          u[q] = make_uint4(0, 0, 0, 0);
          if (z >= a1) continue;
          uint64_t run = 0;
          const uint64_t S = z >= npre ? src_at(d0, l0, e.start_off, mid_off + (z - npre), run) : 0;
          if (z >= npre && run >= 16 && S + 16 <= e.src_len) {
            __builtin_memcpy(&u[q], e.seg + S, 16);
          } else {
            uint32_t wv[4] = {0, 0, 0, 0};
            for (uint32_t b = 0; b < 16 && z + b < a1; ++b) {
              const uint64_t zz = z + b;
              uint32_t by;
              if (zz < npre) {
                by = lit[zz];
              } else {
                uint64_t r2;
                by = e.seg[src_at(d0, l0, e.start_off, mid_off + (zz - npre), r2)];
              }
#pragma unroll
              for (int k = 0; k < 4; ++k)
                if ((b >> 2) == (uint32_t)k) wv[k] |= by << (8 * (b & 3));
            }
            u[q] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
          }
        }
#pragma unroll
        for (int q = 0; q < kPU; ++q) {
          const uint64_t z = zb + 16 * q;
          const uint32_t nb = z >= a1 ? 0u : (a1 - z < 16 ? (uint32_t)(a1 - z) : 16u);
          const uint32_t wq[4] = {u[q].x, u[q].y, u[q].z, u[q].w};
          if (nb == 16u) {  // slice-by-4 (the bytewise loop cost ~2.7 of the writer phase's ~25 ms at config E)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const uint32_t y = x ^ wq[k];
              x = ts[2][y & 0xffu] ^ ts[1][(y >> 8) & 0xffu] ^ ts[0][(y >> 16) & 0xffu] ^ t0[y >> 24];
            }
          } else {
            for (uint32_t b = 0; b < nb; ++b) x = (x >> 8) ^ t0[(x ^ (wq[b >> 2] >> (8 * (b & 3)))) & 0xffu];
          }
        }
      }
      x = a0 < a1 ? shift_by(sp2[0], x, pb - a1) : 0u;
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) x ^= (uint32_t)__shfl_xor((int)x, m, 64);
      const uint64_t y = len - x1;
      if (df) {
        cr0 = x;
        cr1 = rcrc ^ shift_by(sp2[0], x, y);
      } else {
        cr1 = x;
        cr0 = shift_by(sp2[1], rcrc ^ x, y);  // A_{8y}^-1
      }
    }
    for (uint32_t k = 0; k < nfr; ++k) {
      const uint64_t hp = k == 0 ? P : be, x0 = k == 0 ? 0 : x1;
      const uint64_t fl = nfr == 1 ? len : (k == 0 ? x1 : len - x1);
      const uint32_t type = nfr == 1 ? BCW_RECORD_FULL : (k == 0 ? BCW_RECORD_FIRST : BCW_RECORD_LAST);
      if (lane < kHdr && !(A.abl & 8)) {
        const uint32_t crc = ~((k == 0 ? cr0 : cr1) ^ A.initc[fl]);
        const uint32_t masked = ((crc >> 15) | (crc << 17)) + 0xa282ead8u;  // ComputeCRC32 (utils.go:24-29)
        const uint32_t by = lane < 4 ? (masked >> (8 * lane)) : lane == 4 ? (uint32_t)fl
                          : lane == 5 ? (uint32_t)(fl >> 8) : type;
        out[hp - pos + lane] = (uint8_t)by;
      }
      const uint64_t dd = hp + kHdr - pos;  // out index of the fragment's data
      const uint64_t ze = x0 + fl, le = ze < npre ? ze : npre;
      if (!(A.abl & 8))
        for (uint64_t z = x0 + lane; z < le; z += 64) out[dd + (z - x0)] = lit[z];
      if (!(A.abl & 4))
      for (uint64_t z = x0 > npre ? x0 : npre; z < ze;) {
        uint64_t run;
        const uint64_t S = src_at(d0, l0, e.start_off, mid_off + (z - npre), run);
        const uint64_t m = run < ze - z ? run : ze - z;
        copy_run(out + dd + (z - x0), e.seg + S, m, e.seg, e.src_len, lane);
        z += m;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// k_hwrite: the hint WAL (HintRecord.Encode hint.go:32-48 appended with Wal.WriteRecord). Hint records
// are short (NsSize + key + a few varints), so one lane generates one record: its payload bytes in
// order (namespace and key streamed from the source payload in 16 B loads, varints computed), folded
// into the fragment's CRC-32C (bytewise table). Fragments follow the writer's rule (data up to the
// block end, continuation headers at block starts); a header is written once its fragment's CRC is
// known. The 64 records of a wave are contiguous in the output: they are assembled in a staging
// area in LDS (with the zero pads before block-start records) and leave as aligned 16 B stores; a wave
// whose records span more than the staging area writes its bytes straight to HBM instead.
constexpr int kHStage = 9472;  // staging bytes per wave: 64 config-E hint records (~137 B each) fit, and 4 workgroups
                                // per CU instead of 3 (12288: 23.6 vs 23.35 ms per encode)

struct HintOut {
  uint8_t* dst;        // where file offset `org` lives (LDS staging area or the output in HBM)
  uint64_t org;
  const uint32_t* t0;  // byte table (LDS)
  uint64_t a = 0;      // file offset of the next data byte
  uint64_t fend = 0;   // end of the current fragment's data
  uint64_t hp = 0;     // its header
  uint64_t rem = 0;    // payload bytes not yet placed in a fragment
  uint32_t fl = 0, type = 0, crc = 0;
  bool first = true;
  __device__ __forceinline__ void open(uint64_t h) {  // a fragment whose header is at file offset h
    hp = h;
    const uint64_t be = h + kL - (h - 40) % kL, ds = h + kHdr;
    const uint64_t f = rem < be - ds ? rem : be - ds;
    fl = (uint32_t)f;
    type = first ? (f == rem ? BCW_RECORD_FULL : BCW_RECORD_FIRST) : (f == rem ? BCW_RECORD_LAST : BCW_RECORD_MIDDLE);
    first = false;
    rem -= f;
    a = ds;
    fend = ds + f;
    crc = 0xffffffffu;
  }
  __device__ __forceinline__ void close() {  // header of the current fragment
    const uint32_t c = ~crc;
    const uint32_t masked = ((c >> 15) | (c << 17)) + 0xa282ead8u;  // ComputeCRC32 (utils.go:24-29)
    uint8_t* h = dst + (hp - org);
    h[0] = (uint8_t)masked;
    h[1] = (uint8_t)(masked >> 8);
    h[2] = (uint8_t)(masked >> 16);
    h[3] = (uint8_t)(masked >> 24);
    h[4] = (uint8_t)fl;
    h[5] = (uint8_t)(fl >> 8);
    h[6] = (uint8_t)type;
  }
  __device__ __forceinline__ void put(uint32_t b) {
    while (a == fend) {  // the fragment is full (or zero-length): the next one starts at the block end
      close();
      open(fend);
    }
    crc = (crc >> 8) ^ t0[(crc ^ b) & 0xffu];
    dst[a - org] = (uint8_t)b;
    ++a;
  }
  __device__ __forceinline__ void uv(uint64_t v) {
    while (v >= 0x80) { put((uint32_t)(v | 0x80) & 0xffu); v >>= 7; }
    put((uint32_t)v);
  }
};

template <int PM>
__global__ __launch_bounds__(256) void k_hwrite(WArgs A, uint32_t li, const uint32_t* __restrict__ dsrc,
                                                 const uint64_t* __restrict__ dst_da, const uint64_t* __restrict__ dpos) {
  __shared__ uint32_t t0[256];
  __shared__ __attribute__((aligned(16))) uint8_t s_stage[4][kHStage];
  {
    uint32_t c = threadIdx.x;
    for (int b = 0; b < 8; ++b) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    t0[threadIdx.x] = c;
  }
  __syncthreads();
  const WLay& W = li ? A.w[1] : A.w[0];
  if (!lay_ok(A.emisc, W)) return;
  const uint64_t N = A.emisc[X_NDENSE];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t j0 = blockIdx.x * 256ull + wave * 64ull, j = j0 + lane;
  if (j0 >= N) return;
  const bool act = j < N;
  const EncDev& e = A.e;
  const uint64_t row = act ? dsrc[j] : 0;
  uint64_t P = 0, len = 0, prev = 0;
  if (act) {
    P = W.fpos[j];
    len = W.da[j + 1] - W.da[j] - kHdr;
    // the record's region starts after the previous record (the zero pad before a block start, wal.go:509-512)
    prev = P;
    if ((P - 40) % kL == 0) prev = j == 0 ? W.pos : rec_end(W.fpos[j - 1], W.da[j] - W.da[j - 1] - kHdr);
  }
  const uint64_t end = act ? rec_end(P, len) : 0;
  // the wave's output span [lo, hi): its records are consecutive
  const uint64_t lo = uni64(prev), hi = __shfl(end, (int)(N - j0 < 64 ? N - j0 - 1 : 63), 64);
  uint8_t* const out = W.out - W.pos;  // file offset -> memory
  // staging offset of file offset f: f - lo + (address of lo mod 16), so output units are aligned in LDS
  const uint64_t ma = (uint64_t)(uintptr_t)(out + lo), me = ma + (hi - lo);
  const bool staged = hi - lo + 16 <= (uint64_t)kHStage;
  uint8_t* stage = s_stage[wave];
  if (act) {
    uint64_t off, size;
    if (PM == PM_HINT_DST) {
      off = dpos[j];
      size = dst_da[j + 1] - dst_da[j] - kHdr;
    } else {
      off = e.t.foff[row] - kHdr;
      size = e.t.size[row];
    }
    const uint64_t klen = e.t.key_len[row], hdr = e.t.hdr_size[row];
    const SrcRec sr = src_rec(e.t, e.frags, row);
    const Frag F0 = e.frags[sr.f0];
    const uint64_t d0 = frag_file(F0, e.start_off);
    const uint32_t l0 = F0.len;
    bool reg = true;
    for (uint32_t f = sr.f0 + 1; f <= sr.f1 && reg; ++f) {
      const Frag F = e.frags[f];
      reg = F.blk == F0.blk + (f - sr.f0) && F.start == kHdr && (f == sr.f1 || F.len == kM);
    }
    HintOut o;
    o.dst = staged ? stage : out;
    o.org = staged ? lo - (ma & 15u) : 0;
    o.t0 = t0;
    for (uint64_t b = prev; b < P; ++b) o.dst[b - o.org] = 0;
    o.rem = len;
    o.open(P);
    // source payload bytes [z, z + n), in 16 B loads within each source run
    auto src = [&](uint64_t z, uint64_t n) {
      while (n > 0) {
        uint64_t run = 0, S = 0;
        if (reg) S = src_at(d0, l0, e.start_off, z, run);
        const uint32_t c = (uint32_t)(n < 16 ? n : 16);
        if (reg && run >= c && S + 16 <= e.src_len) {
          uint4 v;
          __builtin_memcpy(&v, e.seg + S, 16);
          const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (uint32_t k = 0; k < 16; ++k)
            if (k < c) o.put((w4[k >> 2] >> (8 * (k & 3))) & 0xffu);
          z += c;
          n -= c;
        } else {
          o.put(reg ? e.seg[S] : src_byte(e.seg, e.frags, e.start_off, sr, z));
          ++z;
          --n;
        }
      }
    };
    src(1, e.ns);  // namespace
    o.uv(klen);
    src(hdr, klen);  // key
    o.uv(e.fid);
    o.uv(off);
    o.uv(size);
    o.close();
  }
  if (!staged) return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // the staged span -> HBM: 16 B units aligned to the output memory, partial units at the ends bytewise
  const uint64_t u0 = ma >> 4, nu = ((me - 1) >> 4) - u0 + 1;
  for (uint64_t k = lane; k < nu; k += 64) {
    const uint64_t ua = (u0 + k) << 4;
    uint8_t* d = reinterpret_cast<uint8_t*>((uintptr_t)ua);
    const uint8_t* sp = stage + 16 * k;  // unit k of the staging area
    if (ua >= ma && ua + 16 <= me) {
      *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(sp);
    } else {
      const uint64_t b0 = ua < ma ? ma - ua : 0, b1 = ua + 16 > me ? me - ua : 16;
      for (uint64_t b = b0; b < b1; ++b) d[b] = sp[b];
    }
  }
}

// hint payload sizes of the written records of a compaction (hint.go:32-48 with off/size of the
// dst record, compaction.go:314-320)
__global__ __launch_bounds__(256) void k_hint_sizes(EncDev e, const uint64_t* __restrict__ emisc,
                                                     const uint32_t* __restrict__ dsrc, const uint64_t* __restrict__ da,
                                                     const uint64_t* __restrict__ dpos, uint32_t* __restrict__ hsz) {
  const uint64_t j = blockIdx.x * 256ull + threadIdx.x;
  if (j >= emisc[X_NDENSE]) return;
  const uint64_t row = dsrc[j];
  const uint64_t klen = e.t.key_len[row];
  const uint64_t size = da[j + 1] - da[j] - kHdr;
  hsz[j] = e.ns + uvlen(klen) + (uint32_t)klen + uvlen(e.fid) + uvlen(dpos[j]) + uvlen(size);
}

__global__ void k_enc_finalize(const uint64_t* __restrict__ emisc, uint32_t mode, uint64_t wal_pos, uint64_t wal_cap,
                               uint64_t hint_pos, uint64_t hint_cap, const bcw_decode_result* __restrict__ sres,
                               bcw_encode_result* __restrict__ r) {
  const uint64_t nin = emisc[X_NIN], err = emisc[X_ERR];
  const int hint_lay = (mode == BCW_ENC_HINT) ? 0 : 1;
  bcw_encode_result o{};
  o.n_in = nin;
  o.n_written = emisc[X_NDENSE];
  o.err_record = -1;
  o.src_err_class = sres->err_class;
  if (emisc[X_FAIL]) {
    o.err_class = (int32_t)emisc[X_FAIL];
  } else if ((err >> 2) < nin) {
    o.err_class = (int32_t)(err & 3u);
    o.err_record = (int64_t)(err >> 2);
    o.n_in = err >> 2;  // the callback error stops the iteration there
  } else if (emisc[X_SRCERR]) {
    o.err_class = BCW_ENC_ERR_SRC;
    o.err_record = nin < sres->n_records ? (int64_t)nin : -1;
  }
  if (mode == BCW_ENC_COMPACT) {
    o.wal_end = emisc[X_LAY + 3];
    o.wal_need = o.wal_end - wal_pos;
    o.wal_events = (uint32_t)emisc[X_LAY + 1] - 1;
  } else {
    o.wal_end = wal_pos;
  }
  const uint64_t* H = emisc + X_LAY + hint_lay * kLayStride;
  o.hint_end = H[3];
  o.hint_need = o.hint_end - hint_pos;
  o.hint_events = (uint32_t)H[1] - 1;
  o.fits = (o.wal_need <= wal_cap && o.hint_need <= hint_cap) ? 1 : 0;
  *r = o;
}

}  // namespace enc

// ------------------------------------------------------------------------------------------
hipError_t launch_encode(const EncLaunch& L, EncScratch& s, hipStream_t st, Prof* prof) {
  using namespace enc;
  Prof dummy;
  Prof& pr = prof ? *prof : dummy;
  hipEvent_t ev0 = nullptr;
  EncDev e;
  e.seg = L.d_src;
  e.src_len = L.p.src_len;
  e.frags = L.frags;
  e.t = L.table;
  e.sres = L.d_src_result;
  e.keep = L.d_keep;
  e.dst_base = L.p.dst_base_time;
  e.fid = L.p.fid;
  e.start_off = L.p.src_start_off;
  e.mode = L.p.mode;
  e.ns = L.p.ns_size;
  e.etag = L.p.etag_size;
  e.gen = L.gen;
  const uint64_t rows = L.rows;
  const bool compact = L.p.mode == BCW_ENC_COMPACT;
  TileSum* tiles = static_cast<TileSum*>(s.tiles);
  Ev* evs = static_cast<Ev*>(s.ev);
  (void)hipMemsetAsync(s.emisc, 0, 64 * sizeof(uint64_t), st);
  (void)hipMemsetAsync(s.emisc + X_ERR, 0xff, sizeof(uint64_t), st);
  pr.begin(K_ENC_PREP, st, ev0);
  if (rows) k_enc_prep<<<(uint32_t)((rows + 255) / 256), 256, 0, st>>>(e, rows, s.sz, s.mflag, L.out.rec_off, s.emisc);
  pr.end(K_ENC_PREP, st, ev0);
  const uint32_t ntiles = (uint32_t)((rows + kTileItems - 1) / kTileItems) + 1;
  auto scan = [&](const uint32_t* sz, int over_rows, int lay, uint64_t* da) {
    k_tile_sums<<<ntiles, 256, 0, st>>>(sz, s.emisc, over_rows, tiles);
    k_tile_scan<<<1, 1024, 0, st>>>(tiles, s.emisc, over_rows, lay, da);
    k_tile_scatter<<<ntiles, 256, 0, st>>>(sz, s.emisc, over_rows, tiles, s.dsrc, da);
  };

  WArgs W{};
  W.e = e;
  W.emisc = s.emisc;
  W.wops = L.crc_ops;
  W.initc = L.initc;
  static const int abl_env = [] { const char* v = getenv("BCW_ENC_ABL"); return v ? atoi(v) : 0; }();
  W.abl = (uint32_t)abl_env;
  const uint32_t rgrid = (uint32_t)((rows + 255) / 256) + 1;
  RecDescW* wd = static_cast<RecDescW*>(s.recdesc);
  // persistent write grid: as many workgroups per CU as are resident
  auto wgrid = [&](int g) {
    static int n = 0;
    if (n == 0) {
      const hipError_t rc = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_write<16>, kWT, 0);
      if (rc != hipSuccess || n < 1) n = 2;
    }
    const uint64_t groups = (uint64_t)kWT / g;
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((rows + groups - 1) / groups, (uint64_t)L.num_cus * n));
  };
  auto layout = [&](int lay, const uint64_t* da, uint64_t pos) {
    const int kid = lay == 1 ? K_ENC_EVENTS_HINT : K_ENC_EVENTS;
    pr.begin(kid, st, ev0);
    const uint32_t nwin = (uint32_t)(L.rows / kEvWin + 1);
    k_ev_win<<<nwin, 1024, 0, st>>>(da, s.emisc, lay, pos - 40, s.evt, s.hnl);
    k_ev_walk<<<1, 64, 0, st>>>(s.emisc, lay, pos - 40, s.evt, s.evw, evs);
    k_ev_emit<<<(nwin + 63) / 64, 64, 0, st>>>(da, s.emisc, s.evw, s.hnl, evs, s.evb);
    k_ev_fix<<<1, 1024, 0, st>>>(da, s.emisc, lay, evs);
    pr.end(kid, st, ev0);
  };
  if (compact) {
    // stream st: the layouts and the writers; stream aux: the dst records' payload descriptors (after the
    // dense scan), built while the layouts run
    pr.begin(K_ENC_SCAN, st, ev0);
    scan(s.sz, 1, 0, s.da);
    pr.end(K_ENC_SCAN, st, ev0);
    (void)hipEventRecord(s.ev_scan, st);
    (void)hipStreamWaitEvent(s.aux, s.ev_scan, 0);
    k_recdesc_w<PM_DST><<<rgrid, 256, 0, s.aux>>>(e, s.emisc, s.dsrc, nullptr, nullptr, s.mflag, L.crc_ops, wd);
    (void)hipEventRecord(s.ev_desc, s.aux);
    layout(0, s.da, L.p.wal_pos);
    k_recoff<<<rgrid, 256, 0, st>>>(s.da, s.dsrc, s.emisc, 0, evs, s.evb, s.dpos, L.out.rec_off);
    // the hint WAL's layout needs the dst offsets (its records carry them)
    pr.begin(K_ENC_HINT_LAYOUT, st, ev0);
    k_hint_sizes<<<rgrid, 256, 0, st>>>(e, s.emisc, s.dsrc, s.da, s.dpos, s.hsz);
    scan(s.hsz, 0, 1, s.hda);
    pr.end(K_ENC_HINT_LAYOUT, st, ev0);
    layout(1, s.hda, L.p.hint_pos);
    k_recoff<<<rgrid, 256, 0, st>>>(s.hda, s.dsrc, s.emisc, 1, evs, s.evb, s.hpos, nullptr);
    (void)hipStreamWaitEvent(st, s.ev_desc, 0);
    W.w[0] = WLay{s.da, s.dpos, wd, L.out.wal, L.p.wal_pos, L.out.wal_cap, 0};
    W.w[1] = WLay{s.hda, s.hpos, nullptr, L.out.hint, L.p.hint_pos, L.out.hint_cap, 1};
    W.nlay = 1;
    W.wl = s.wl;
    W.rows = rows;
    W.wcnt = s.emisc + X_WL16;
    const int abl = abl_env & 3;
    pr.begin(K_ENC_WRITE, st, ev0);
    // measurement-only ablation (BCW_ENC_ABL: 1 = dst WAL only, 2 = hint WAL only); 0 in the product
    if (abl != 2) {
      // as many workgroups as are resident at once (each takes a fixed share of the records: a grid of 8 per CU with
      // 6 resident ran its last 2 per CU after the others, at a third of the occupancy)
      // (cached per context: the query runs on the context's device, and no state is shared between contexts)
      if (s.wcopy_resident == 0 &&
          (hipOccupancyMaxActiveBlocksPerMultiprocessor(&s.wcopy_resident, k_wcopy, kCT, 0) != hipSuccess ||
           s.wcopy_resident < 1))
        s.wcopy_resident = 4;
      k_wcopy<<<(uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((rows + 3) / 4, (uint64_t)L.num_cus * s.wcopy_resident)), kCT, 0,
                st>>>(W);
      k_write<16><<<wgrid(16), kWT, 0, st>>>(W);
      k_write_general<PM_DST><<<std::min<uint32_t>(rgrid, (uint32_t)L.num_cus * 4), 256, 0, st>>>(W, 0, s.dsrc, nullptr,
                                                                                            nullptr, s.mflag);
    }
    if (abl != 1) k_hwrite<PM_HINT_DST><<<rgrid, 256, 0, st>>>(W, 1, s.dsrc, s.da, s.dpos);
    pr.end(K_ENC_WRITE, st, ev0);
  } else {
    pr.begin(K_ENC_SCAN, st, ev0);
    scan(s.sz, 1, 0, s.hda);
    pr.end(K_ENC_SCAN, st, ev0);
    layout(0, s.hda, L.p.hint_pos);
    k_recoff<<<rgrid, 256, 0, st>>>(s.hda, s.dsrc, s.emisc, 0, evs, s.evb, s.hpos, nullptr);
    W.w[0] = WLay{s.hda, s.hpos, nullptr, L.out.hint, L.p.hint_pos, L.out.hint_cap, 0};
    W.w[1] = W.w[0];
    W.nlay = 1;
    pr.begin(K_ENC_WRITE, st, ev0);
    k_hwrite<PM_HINT_SRC><<<rgrid, 256, 0, st>>>(W, 0, s.dsrc, nullptr, nullptr);
    pr.end(K_ENC_WRITE, st, ev0);
  }
  k_enc_finalize<<<1, 1, 0, st>>>(s.emisc, L.p.mode, L.p.wal_pos, L.out.wal_cap, L.p.hint_pos, L.out.hint_cap,
                                  L.d_src_result, L.d_result);
  return hipGetLastError();
}

size_t enc_sizeof_ev() { return sizeof(enc::Ev); }
size_t enc_sizeof_recdesc() { return sizeof(enc::RecDescW); }
size_t enc_sizeof_tile() { return sizeof(enc::TileSum); }
int enc_tile_items() { return enc::kTileItems; }
int enc_ev_win() { return enc::kEvWin; }

}  // namespace bcw
