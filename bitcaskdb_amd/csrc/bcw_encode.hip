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
//   k_events        the writer's layout recurrence as an event scan (one workgroup)    wal.go:505-549
//   k_blkdesc       per output block: start y, continuation flag, pad, first record
//   k_recoff        per record: the file offset WriteRecord returns                     wal.go:514-516
//   k_pack<PM>      per output 32 KiB block: LDS image of headers + payload bytes, CRC-32C per
//                   fragment (utils.go:24-29), streamed out with aligned 16 B stores
//   (compaction) k_hint_sizes + scan + events + blkdesc + k_pack<hint> for the hint WAL
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
// all but rare records (~7/M of them): k_events runs it over 4096 records per step with a
// workgroup-wide ballot, and every other quantity (block starts, record offsets, fragment types
// and lengths) follows in parallel from the event list.
#include <algorithm>
#include <cstdlib>

#include "bcw_internal.h"

namespace bcw {
namespace enc {

constexpr uint32_t kL = kBlock;           // 32768
constexpr uint32_t kM = kBlock - kHdr;    // 32761
constexpr int kTileItems = 4096;          // scan tile: 256 threads x 16 items
constexpr int kEvThreads = 1024;
constexpr int kEvPer = 4;
constexpr int kEvWin = 4096;  // records per k_events step (LDS double buffer: 2 x 40 KiB)
constexpr int kJobCap = 1024;
constexpr int kJobsPerRec = 8;

// emisc slots
enum {
  X_NIN = 0,      // source rows delivered (IterateRecord)
  X_ERR = 1,      // min over rows of (row << 2 | class) of Record.Encode failures
  X_SRCERR = 2,   // source error class (BCW_ENC_ERR_SRC when iteration stopped on a bad row / fragment)
  X_NDENSE = 3,   // records written
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
  const uint64_t nin = (R->first_bad_record >= 0 && (uint64_t)R->first_bad_record < nrec)
                           ? (uint64_t)R->first_bad_record : nrec;
  if (i == 0) {
    emisc[X_NIN] = nin;
    emisc[X_SRCERR] = (nin < nrec || R->err_class != BCW_ERR_NONE) ? 1u : 0u;
  }
  if (i >= rows) return;
  if (rec_off && i < nrec) rec_off[i] = ~0ull;
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

// One workgroup of kEvThreads, kEvWin = kEvThreads * kEvPer records per window in registers. A round:
// every thread tests its records after the last event against rho, the wave minima meet in LDS, and
// the owner of the first hit records the event and advances the scan state. Rounds per window =
// events in it + 1. (Measured against a barrier-free scanner wave fed by loader waves and against a
// one-barrier-per-round replay from LDS: both slower)
__global__ __launch_bounds__(kEvThreads) void k_events(const uint64_t* __restrict__ da, uint64_t* __restrict__ emisc,
                                                        int lay, uint64_t q0, Ev* __restrict__ ev,
                                                        uint32_t* __restrict__ evb) {
  const uint64_t N = emisc[X_NDENSE];
  uint64_t* X = emisc + X_LAY + lay * kLayStride;
  const uint64_t AN = X[0];
  const int64_t U = (int64_t)(q0 % kL);
  const uint64_t b0 = q0 / kL;
  __shared__ int64_t s_ya;
  __shared__ uint64_t s_kb;
  __shared__ uint32_t s_rho, s_nev, s_best;
  __shared__ uint32_t s_wmin[kEvThreads / 64];
  if (threadIdx.x == 0) {
    ev[0] = {b0, -U, 0xffffffffu, 0};
    int64_t ya = -U;
    uint64_t kb = b0;
    uint32_t nev = 1;
    uint32_t rho = (uint32_t)((kL - U) % kM);  // the virtual block ends at y = L - U
    if (N > 0 && kL - U < (int64_t)kHdr) {    // record 0's header does not fit: pad, event at record 0
      ev[1] = {b0 + 1, 0, 0u, (uint32_t)(kL - U)};
      ya = 0;
      kb = b0 + 1;
      nev = 2;
      rho = kL % kM;
    }
    s_ya = ya; s_kb = kb; s_rho = rho; s_nev = nev;
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (uint64_t base = 0; base < N; base += kEvWin) {
    if (threadIdx.x == 0) evb[base / kEvWin] = s_nev - 1;
    uint64_t a[kEvPer];
    uint32_t r[kEvPer];
#pragma unroll
    for (int k = 0; k < kEvPer; ++k) {
      const uint64_t idx = base + (uint64_t)k * kEvThreads + threadIdx.x;
      a[k] = idx < N ? da[idx] : 0;
      r[k] = (uint32_t)(a[k] % kM);
    }
    // record 0 is never tested against the virtual event (its header is in block b0 or it is ev[1])
    int last = (base == 0) ? 0 : -1;
    uint32_t rho = s_rho;
    for (;;) {
      uint32_t best = 0xffffffffu;
#pragma unroll
      for (int k = kEvPer - 1; k >= 0; --k) {
        const uint32_t q = (uint32_t)k * kEvThreads + threadIdx.x;
        const uint64_t idx = base + q;
        if (idx < N && (int)q > last) {
          int32_t d = (int32_t)rho - (int32_t)r[k];
          if (d < 0) d += kM;
          if (d <= 6) best = q;
        }
      }
      for (int d = 32; d >= 1; d >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, d, 64));
      if (lane == 0) s_wmin[wave] = best;
      __syncthreads();
      if (threadIdx.x == 0) {
        uint32_t m = 0xffffffffu;
        for (int w = 0; w < kEvThreads / 64; ++w) m = min(m, s_wmin[w]);
        s_best = m;
      }
      __syncthreads();
      const uint32_t b = s_best;
      if (b == 0xffffffffu) break;
      if (threadIdx.x == (b & (kEvThreads - 1))) {  // the owner records the event
        const int k = (int)(b / kEvThreads);
        uint64_t ai = a[0];
        uint32_t ri = r[0];
#pragma unroll
        for (int kk = 1; kk < kEvPer; ++kk) if (kk == k) { ai = a[kk]; ri = r[kk]; }
        int32_t d = (int32_t)s_rho - (int32_t)ri;
        if (d < 0) d += kM;
        const int64_t E = (int64_t)ai + d;                         // block end that hits the header
        const uint64_t m = (uint64_t)(E - s_ya - (int64_t)kL) / kM;  // blocks after the event block
        const uint64_t kb = s_kb + m + 1;
        ev[s_nev] = {kb, (int64_t)ai, (uint32_t)(base + b), (uint32_t)d};
        s_nev = s_nev + 1;
        s_kb = kb;
        s_ya = (int64_t)ai;
        s_rho = (ri + kHdr) % kM;
      }
      __syncthreads();
      rho = s_rho;
      last = (int)b;
    }
  }
  if (threadIdx.x == 0) {
    const uint32_t nev = s_nev;
    X[1] = nev;
    X[4] = b0;
    X[5] = (uint64_t)U;
    if (N == 0) {
      X[2] = b0 - 1;  // no blocks
      X[3] = 40 + q0;
    } else {
      const int64_t ya = s_ya;
      const uint64_t kb = s_kb;
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

// per-block descriptor for k_pack
struct BlkDesc {
  int64_t Y;       // y of the block start
  uint32_t first;  // dense record holding Y (or the record whose header is at Y)
  uint32_t lo;     // first image byte the block writes (U for the first block)
  uint32_t hi;     // image end (L, or the file end in the last block)
  uint8_t c;       // continuation header at image 0
  uint8_t pad;     // zero bytes at the block end
  uint16_t _r;
};

__device__ __forceinline__ uint32_t ev_of_block(const Ev* __restrict__ ev, uint32_t nev, uint64_t k) {
  uint32_t lo = 0, hi = nev;  // largest g with ev[g].blk <= k
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (ev[mid].blk <= k) lo = mid; else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void k_blkdesc(const uint64_t* __restrict__ da, const uint64_t* __restrict__ emisc,
                                                  int lay, const Ev* __restrict__ ev, BlkDesc* __restrict__ desc,
                                                  uint64_t desc_cap) {
  const uint64_t* X = emisc + X_LAY + lay * kLayStride;
  const uint64_t b0 = X[4], ke = X[2];
  const uint64_t k = b0 + blockIdx.x * 256ull + threadIdx.x;
  if (k > ke || ke == b0 - 1 || k - b0 >= desc_cap) return;
  const uint32_t nev = (uint32_t)X[1];
  const uint64_t N = emisc[X_NDENSE];
  const uint32_t g = ev_of_block(ev, nev, k);
  const Ev e = ev[g];
  BlkDesc d;
  if (k == e.blk) {
    d.Y = e.ya;
    d.c = 0;
    d.first = (g == 0) ? 0u : e.rec;
  } else {
    d.Y = e.ya + (int64_t)kL + (int64_t)(k - e.blk - 1) * kM;
    d.c = 1;
    // the record holding Y: largest j with a_j < Y, between this event's record and the next one's
    uint64_t lo = (g == 0) ? 0 : e.rec, hi = (g + 1 < nev) ? ev[g + 1].rec : N;
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if ((int64_t)da[mid] < d.Y) lo = mid; else hi = mid;
    }
    d.first = (uint32_t)lo;
  }
  d.pad = (g + 1 < nev && ev[g + 1].blk == k + 1) ? (uint8_t)ev[g + 1].pad : 0;
  d.lo = (k == b0) ? (uint32_t)X[5] : 0u;
  d.hi = (k == ke) ? (uint32_t)(X[3] - 40 - ke * kL) : kL;
  d._r = 0;
  desc[k - b0] = d;
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
// Payload programs: a record's payload as up to 6 pieces, each literal bytes (computed here) or a
// range of the source record's payload.
struct Prog {
  uint32_t len[6];
  uint64_t off[6];   // literal: offset into lit; source: payload offset in the source record
  uint8_t src[6];
  uint32_t n;
  uint8_t lit[48];
};

// Record.Encode (record.go:57-138) of source row i against the dst baseTime
__device__ void prog_record(const EncDev& e, uint64_t i, bool mdrop, Prog& p) {
  const bcw_record_table& t = e.t;
  const uint32_t flags = t.flags[i];
  const uint64_t klen = t.key_len[i], vlen = t.val_len[i], expire = t.expire[i];
  const uint64_t mlen = mdrop ? 0 : t.meta_len[i];
  const uint32_t el = (flags & 1u) ? 0u : e.etag;
  uint8_t flag = (uint8_t)((el == 0 ? 1u : 0u) | (flags & 4u) | (expire == 0 ? 2u : 0u));
  uint32_t o = 1;
  p.lit[o++] = flag;
  o += uvput(p.lit + o, klen);
  o += uvput(p.lit + o, vlen);
  o += uvput(p.lit + o, mlen);
  const uint32_t vend = o;
  if (expire != 0) o += uvput(p.lit + o, expire - e.dst_base);
  const uint32_t hn = 1 + e.ns + (vend - 1) + el + (o - vend);
  p.lit[0] = (uint8_t)hn;  // byte(headerSize) (record.go:109)
  p.n = 6;
  p.src[0] = 0; p.len[0] = 1; p.off[0] = 0;
  p.src[1] = 1; p.len[1] = e.ns; p.off[1] = 1;
  p.src[2] = 0; p.len[2] = vend - 1; p.off[2] = 1;
  p.src[3] = 1; p.len[3] = el; p.off[3] = t.etag_off[i];
  p.src[4] = 0; p.len[4] = o - vend; p.off[4] = vend;
  p.src[5] = 1; p.len[5] = (uint32_t)(klen + vlen + mlen); p.off[5] = t.hdr_size[i];
}

// HintRecord.Encode (hint.go:32-48): ns | uvarint(len(key)) | key | uvarint fid | off | size
__device__ void prog_hint(const EncDev& e, uint64_t i, uint64_t off, uint64_t size, Prog& p) {
  const bcw_record_table& t = e.t;
  const uint64_t klen = t.key_len[i];
  uint32_t o = uvput(p.lit, klen);
  const uint32_t k1 = o;
  o += uvput(p.lit + o, e.fid);
  o += uvput(p.lit + o, off);
  o += uvput(p.lit + o, size);
  p.n = 4;
  p.src[0] = 1; p.len[0] = e.ns; p.off[0] = 1;
  p.src[1] = 0; p.len[1] = k1; p.off[1] = 0;
  p.src[2] = 1; p.len[2] = (uint32_t)klen; p.off[2] = t.hdr_size[i];
  p.src[3] = 0; p.len[3] = o - k1; p.off[3] = k1;
}

enum { PM_DST = 0, PM_HINT_DST = 1, PM_HINT_SRC = 2 };

// CRC-32C helpers: raw (init 0, no final xor) byte update; shift operators as nibble tables
__device__ __forceinline__ uint32_t op_apply(const uint32_t* __restrict__ op, uint32_t x) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= op[i * 16 + ((x >> (4 * i)) & 15u)];
  return r;
}

struct PackArgs {
  EncDev e;
  const uint64_t* da;       // this layout's y-coordinates (dense, N+1)
  const void* rd;           // RecDesc per dense record (k_recdesc)
  const BlkDesc* desc;
  const uint64_t* emisc;
  int lay;
  uint8_t* out;
  uint64_t pos, cap;        // file offset of out[0]; out capacity
  const uint32_t* crc_ops;  // [2][16][8][16]: A_{8*128*m}, A_{8*2048*m}, m < 16
  const uint32_t* initc;    // A_{8L}(0xFFFFFFFF)
  uint32_t abl;             // ablation bits for measurements only (0 in the product): 1 no CRC, 2 no copy, 8 no store
};

// Per written record: its payload as up to 6 pieces (literal bytes or ranges of the source payload)
// and the source payload's placement in the source file. Built once per record by k_recdesc, read
// by the one or two k_pack workgroups whose blocks hold the record.
struct RecDesc {
  uint64_t d0;       // file offset of the data of the source payload's first fragment
  uint32_t l0;       // its length
  uint32_t f0, f1;   // source fragments (irregular records are walked)
  uint16_t regular;  // fragments after the first are whole blocks' data: closed-form placement
  uint8_t npieces, psrc;  // psrc bit q: piece q is a source range
  uint32_t plen[6];
  uint32_t poff[6];  // source payload offset (source piece) or offset into lit
  uint8_t lit[48];
  uint64_t _pad;
};
static_assert(sizeof(RecDesc) == 128, "RecDesc layout");

template <int PM>
__global__ __launch_bounds__(256) void k_recdesc(EncDev e, const uint64_t* __restrict__ emisc,
                                                  const uint32_t* __restrict__ dsrc, const uint64_t* __restrict__ dst_da,
                                                  const uint64_t* __restrict__ dpos, const uint8_t* __restrict__ mflag,
                                                  RecDesc* __restrict__ rd) {
  const uint64_t j = blockIdx.x * 256ull + threadIdx.x;
  if (j >= emisc[X_NDENSE]) return;
  const uint64_t row = dsrc[j];
  Prog p;
  if (PM == PM_DST) prog_record(e, row, mflag[row] != 0, p);
  else if (PM == PM_HINT_DST) prog_hint(e, row, dpos[j], dst_da[j + 1] - dst_da[j] - kHdr, p);
  else prog_hint(e, row, e.t.foff[row] - kHdr, e.t.size[row], p);
  const SrcRec sr = src_rec(e.t, e.frags, row);
  const Frag F0 = e.frags[sr.f0];
  RecDesc d;
  d.d0 = frag_file(F0, e.start_off);
  d.l0 = F0.len;
  d.f0 = sr.f0;
  d.f1 = sr.f1;
  bool reg = true;
  for (uint32_t f = sr.f0 + 1; f <= sr.f1 && reg; ++f) {
    const Frag F = e.frags[f];
    reg = F.blk == F0.blk + (f - sr.f0) && F.start == kHdr && (f == sr.f1 || F.len == kM);
  }
  d.regular = reg ? 1 : 0;
  d.npieces = (uint8_t)p.n;
  d.psrc = 0;
  for (uint32_t q = 0; q < 6; ++q) {
    d.plen[q] = q < p.n ? p.len[q] : 0;
    d.poff[q] = q < p.n ? (uint32_t)p.off[q] : 0;
    if (q < p.n && p.src[q]) d.psrc |= (uint8_t)(1u << q);
  }
#pragma unroll
  for (int b = 0; b < 48; ++b) d.lit[b] = p.lit[b];
  uint4* dst = reinterpret_cast<uint4*>(rd + j);
  const uint4* s = reinterpret_cast<const uint4*>(&d);
#pragma unroll
  for (int k = 0; k < 8; ++k) dst[k] = s[k];
}

// The LDS block image is skewed by one dword per 128 B (word w lives at w + w/32): lanes reading
// consecutive 128 B CRC windows would otherwise all hit the same bank. 16 B chunks (the copy and
// store units) never straddle a pad word.
__device__ __forceinline__ uint32_t iw(uint32_t w) { return w + (w >> 5); }
__device__ __forceinline__ uint8_t img_get(const uint32_t* img, uint32_t b) {
  return (uint8_t)(img[iw(b >> 2)] >> ((b & 3u) * 8));
}
__device__ __forceinline__ void img_put(uint32_t* img, uint32_t b, uint8_t v) {
  reinterpret_cast<uint8_t*>(img)[iw(b >> 2) * 4 + (b & 3u)] = v;
}

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

constexpr int kPT = 512;   // k_pack threads
constexpr int kPWaves = kPT / 64;
constexpr int kRecBatch = kPT;

// k_pack: persistent workgroups, one output block at a time: (1) each record with a fragment in the
// block writes its literal bytes into the LDS image and queues source copy jobs; (2) the waves copy
// the jobs (lanes over 16 B image chunks, loads issued ahead of the LDS writes); (3) CRC-32C of every
// fragment: 128 B windows aligned to the fragment end, two slice-by-4 chains per window, shifted to
// the fragment end with A_{8*128*m} and XOR-ed into the fragment's accumulator; headers written;
// (4) the image streams out with aligned 16 B stores.
template <int PM>
__global__ __launch_bounds__(kPT) __attribute__((amdgpu_waves_per_eu(4))) void k_pack(PackArgs A) {
  const uint64_t* X = A.emisc + X_LAY + A.lay * kLayStride;
  const uint64_t b0 = X[4], ke = X[2];
  if (ke == b0 - 1 || X[3] - A.pos > A.cap) return;  // nothing to write / does not fit (result says so)
  const uint64_t K = ke - b0 + 1;
  const EncDev& e = A.e;
  const uint64_t N = A.emisc[X_NDENSE];
  const RecDesc* __restrict__ RD = static_cast<const RecDesc*>(A.rd);

  __shared__ __attribute__((aligned(16))) uint32_t img[kL / 4 + kL / 128 + 8];
  __shared__ uint32_t tab[4 * 256];
  __shared__ uint32_t ops[2 * 16 * 128];
  __shared__ uint32_t half[128];
  __shared__ uint16_t f_hdr[kRecBatch], f_dat[kRecBatch], f_len[kRecBatch];
  __shared__ uint8_t f_type[kRecBatch];
  __shared__ uint32_t f_acc[kRecBatch], f_win[kRecBatch + 1];
  __shared__ uint16_t j_img[kJobCap], j_len[kJobCap];
  __shared__ uint64_t j_src[kJobCap];
  __shared__ uint32_t j_pre[kJobCap + 1];
  __shared__ uint32_t s_njobs, s_nrec, s_scan[kPWaves];

  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // slice-by-4 tables (tab[256*k + b] = CRC of byte b followed by k zero bytes) and operators
  for (uint32_t i = tid; i < 256; i += kPT) {
    uint32_t c = i;
    for (int b = 0; b < 8; ++b) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    tab[i] = c;
  }
  for (uint32_t i = tid; i < 2 * 16 * 128; i += kPT) ops[i] = A.crc_ops[i];
  __syncthreads();
  if (tid < 256) {
    uint32_t c = tab[tid];
    for (int k = 1; k < 4; ++k) { c = (c >> 8) ^ tab[c & 0xffu]; tab[256 * k + tid] = c; }
  }
  // A_{8*64}: 64 zero bytes (half-window join)
  if (tid < 128) {
    const uint32_t i = tid >> 4, n = tid & 15u;
    uint32_t x = n << (4 * i);
    for (int b = 0; b < 64; ++b) x = (x >> 8) ^ tab[x & 0xffu];
    half[tid] = x;
  }
  __syncthreads();

  for (uint64_t kb = blockIdx.x; kb < K; kb += gridDim.x) {
    const uint64_t k = b0 + kb;
    const BlkDesc D = A.desc[kb];
    const int64_t Y = D.Y;
    const int64_t E = Y + (int64_t)kL - (int64_t)kHdr * D.c;
    if (D.pad) for (uint32_t b = kL - D.pad + tid; b < kL; b += kPT) img_put(img, b, 0);

    for (uint64_t rb = D.first;; rb += kRecBatch) {
      if (tid == 0) { s_njobs = 0; s_nrec = 0; }
      __syncthreads();
      // ---- (1) one record per thread: fragment geometry, literals, copy jobs ----
      const uint64_t j = rb + tid;
      bool act = false;
      uint64_t aj = 0, aj1 = 0;
      uint4 rv[5];  // descriptor bytes [0, 80): everything but the literals (static indexing only)
      if (j < N) {
        // the descriptor load does not depend on the y-coordinates: both in flight together
        const uint4* sp = reinterpret_cast<const uint4*>(RD + j);
#pragma unroll
        for (int q = 0; q < 5; ++q) rv[q] = sp[q];
        aj = A.da[j];
        aj1 = A.da[j + 1];
        act = ((int64_t)aj < Y) || ((int64_t)aj + (int64_t)kHdr <= E);
      }
      if (act) atomicAdd(&s_nrec, 1u);
      f_acc[tid] = 0;
      if (act) {
        const bool cont = (int64_t)aj < Y;
        const int64_t y0 = cont ? Y : (int64_t)aj + kHdr;
        const int64_t y1 = (int64_t)aj1 < E ? (int64_t)aj1 : E;
        const uint32_t hdr = cont ? 0u : (uint32_t)(kHdr * D.c + ((int64_t)aj - Y));
        const uint32_t d0 = hdr + kHdr;
        const uint32_t len = (uint32_t)(y1 - y0);
        const bool ends = (int64_t)aj1 <= E;
        f_hdr[tid] = (uint16_t)hdr;
        f_dat[tid] = (uint16_t)d0;
        f_len[tid] = (uint16_t)len;
        f_type[tid] = cont ? (ends ? BCW_RECORD_LAST : BCW_RECORD_MIDDLE) : (ends ? BCW_RECORD_FULL : BCW_RECORD_FIRST);
        const uint64_t x0 = (uint64_t)(y0 - (int64_t)aj - kHdr), x1 = x0 + len;
        const uint8_t* litg = RD[j].lit;  // literal bytes straight from the (cached) descriptor line
        struct {
          uint64_t d0;
          uint32_t l0, f0, f1;
          bool regular;
        } d;
        d.d0 = (uint64_t)rv[0].x | ((uint64_t)rv[0].y << 32);
        d.l0 = rv[0].z;
        d.f0 = rv[0].w;
        d.f1 = rv[1].x;
        d.regular = (rv[1].y & 0xffffu) != 0;
        const uint32_t npieces = (rv[1].y >> 16) & 0xffu, psrc = rv[1].y >> 24;
        const uint32_t plen[6] = {rv[1].z, rv[1].w, rv[2].x, rv[2].y, rv[2].z, rv[2].w};
        const uint32_t poff[6] = {rv[3].x, rv[3].y, rv[3].z, rv[3].w, rv[4].x, rv[4].y};
        uint64_t pb = 0;
        bool slow = false;
#pragma unroll
        for (uint32_t q = 0; q < 6; ++q) {
          if (q >= npieces) break;
          const uint64_t pe = pb + plen[q];
          const uint64_t s0 = pb > x0 ? pb : x0, s1 = pe < x1 ? pe : x1;
          if (s0 < s1) {
            uint32_t io = d0 + (uint32_t)(s0 - x0);
            if (!((psrc >> q) & 1u)) {
              for (uint64_t s = s0; s < s1; ++s) img_put(img, io++, litg[poff[q] + (s - pb)]);
            } else {
              uint64_t z = poff[q] + (s0 - pb), l = s1 - s0;
              // irregular source records: walk their fragments
              uint32_t f = d.f0;
              Frag F{};
              uint64_t cum = 0;
              if (!d.regular) {
                F = e.frags[f];
                while (z >= cum + F.len && f < d.f1) { cum += F.len; ++f; F = e.frags[f]; }
              }
              while (l > 0) {
                uint64_t src, take;
                if (d.regular) {
                  src = src_at(d.d0, d.l0, e.start_off, z, take);
                } else {
                  const uint64_t in = z - cum;
                  take = F.len - in;
                  if (f >= d.f1) take = l;
                  src = frag_file(F, e.start_off) + in;
                }
                if (take > l) take = l;
                uint32_t slot = kJobCap;
                if (!slow) {
                  slot = atomicAdd(&s_njobs, 1u);
                  if (slot >= kJobCap) slow = true;
                }
                if (slow) {
                  for (uint64_t b = 0; b < take; ++b) img_put(img, io + (uint32_t)b, e.seg[src + b]);
                } else {
                  j_img[slot] = (uint16_t)io;
                  j_len[slot] = (uint16_t)take;
                  j_src[slot] = src;
                }
                io += (uint32_t)take;
                z += take;
                l -= take;
                if (!d.regular && l > 0) { cum += F.len; ++f; F = e.frags[f]; }
              }
            }
          }
          pb = pe;
        }
      }
      __syncthreads();
      const uint32_t nrec = s_nrec;
      const uint32_t njobs = min(s_njobs, (uint32_t)kJobCap);
      if (nrec == 0) break;
      // ---- (2) copy jobs: prefix of the jobs' 16 B image chunks, then every thread takes 4 chunks
      //      per round (job lookup, both loads of all 4 issued before any LDS write) ----
      for (uint32_t base = 0; base < njobs; base += kPT) {
        const uint32_t q = base + tid;
        uint32_t cnt = 0;
        if (q < njobs) {
          const uint32_t o = j_img[q], l = j_len[q];
          cnt = l ? ((o + l + 15) >> 4) - (o >> 4) : 0;
        }
        uint32_t incl = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) { const uint32_t t = __shfl_up(incl, d, 64); if (lane >= (uint32_t)d) incl += t; }
        if (lane == 63) s_scan[wave] = incl;
        __syncthreads();
        uint32_t pre = base ? j_pre[base] : 0;
        for (uint32_t w = 0; w < wave; ++w) pre += s_scan[w];
        if (q < njobs) j_pre[q + 1] = pre + incl;
        if (q == 0) j_pre[0] = 0;
        __syncthreads();
      }
      const uint32_t nunits = (njobs && !(A.abl & 2)) ? j_pre[njobs] : 0;
      for (uint32_t u0 = tid; u0 < nunits; u0 += 4 * kPT) {
        uint4 v0[4], v1[4];
        uint32_t c0s[4], c1s[4];
        uint64_t ss[4];
        bool full[4];
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) {
          const uint32_t u = u0 + (uint32_t)k2 * kPT;
          full[k2] = false;
          c0s[k2] = c1s[k2] = 0;
          ss[k2] = 0;
          if (u < nunits) {
            uint32_t lo = 0, hi = njobs;  // largest q with j_pre[q] <= u
            while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (j_pre[mid] <= u) lo = mid; else hi = mid; }
            const uint32_t o = j_img[lo], l = j_len[lo];
            const uint32_t c = (o >> 4) + (u - j_pre[lo]);
            const uint32_t c0 = c * 16 > o ? c * 16 : o;
            const uint32_t c1 = c * 16 + 16 < o + l ? c * 16 + 16 : o + l;
            const uint64_t sv = j_src[lo] + (c0 - o);
            c0s[k2] = c0;
            c1s[k2] = c1;
            ss[k2] = sv;
            if (c1 - c0 == 16 && (sv & ~15ull) + 32 <= e.src_len) {
              full[k2] = true;
              v0[k2] = *reinterpret_cast<const uint4*>(e.seg + (sv & ~15ull));
              v1[k2] = *reinterpret_cast<const uint4*>(e.seg + (sv & ~15ull) + 16);
            }
          }
        }
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) {
          if (full[k2]) {
            *reinterpret_cast<uint4*>(&img[iw(c0s[k2] >> 2)]) = shift16(v0[k2], v1[k2], (uint32_t)(ss[k2] & 15u));
          } else {
            for (uint32_t b = c0s[k2]; b < c1s[k2]; ++b) img_put(img, b, e.seg[ss[k2] + (b - c0s[k2])]);
          }
        }
      }
      // window counts of the fragments (128 B windows, end-aligned)
      {
        const uint32_t cw = (tid < nrec) ? ((uint32_t)f_len[tid] + 127u) >> 7 : 0u;
        uint32_t incl = cw;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) { const uint32_t t = __shfl_up(incl, d, 64); if (lane >= (uint32_t)d) incl += t; }
        if (lane == 63) s_scan[wave] = incl;
        __syncthreads();  // also: the copies are complete
        uint32_t pre = 0;
        for (uint32_t w = 0; w < wave; ++w) pre += s_scan[w];
        f_win[tid + 1] = pre + incl;
        if (tid == 0) f_win[0] = 0;
        __syncthreads();
      }
      // ---- (3) CRC windows ----
      const uint32_t nwin = (A.abl & 1) ? 0 : f_win[nrec];
      for (uint32_t w = tid; w < nwin; w += kPT) {
        uint32_t lo = 0, hi = nrec;
        while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (f_win[mid] <= w) lo = mid; else hi = mid; }
        const uint32_t f = lo;
        const uint32_t m = f_win[f + 1] - 1 - w;  // windows between this one and the fragment end
        const int32_t fs = f_dat[f];
        const int32_t we = fs + (int32_t)f_len[f] - 128 * (int32_t)m;
        const int32_t base = we - 128;
        const int32_t dw = base >> 2;  // arithmetic: negative bases read clamped (masked) words
        const uint32_t sh = (uint32_t)(base & 3);
        uint32_t wv[32];
        uint32_t prev = dw >= 0 ? img[iw((uint32_t)dw)] : 0u;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
          const int32_t idx = dw + 1 + i;
          const uint32_t nx = idx >= 0 ? img[iw((uint32_t)idx)] : 0u;
          wv[i] = __builtin_amdgcn_alignbyte(nx, prev, sh);
          prev = nx;
        }
        // zero the bytes before the fragment start (first window only)
        const int32_t zb = fs - base;  // bytes to clear
        if (zb > 0) {
#pragma unroll
          for (int i = 0; i < 32; ++i) {
            int32_t t = zb - 4 * i;
            t = t < 0 ? 0 : (t > 4 ? 4 : t);
            wv[i] &= (uint32_t)(0xffffffffull << (8 * t));
          }
        }
        uint32_t ca = 0, cb2 = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          ca ^= wv[i];
          ca = tab[768 + (ca & 0xffu)] ^ tab[512 + ((ca >> 8) & 0xffu)] ^ tab[256 + ((ca >> 16) & 0xffu)] ^ tab[ca >> 24];
          cb2 ^= wv[16 + i];
          cb2 = tab[768 + (cb2 & 0xffu)] ^ tab[512 + ((cb2 >> 8) & 0xffu)] ^ tab[256 + ((cb2 >> 16) & 0xffu)] ^ tab[cb2 >> 24];
        }
        uint32_t c = op_apply(half, ca) ^ cb2;
        if (m & 15u) c = op_apply(&ops[(m & 15u) * 128], c);
        if (m >> 4) c = op_apply(&ops[2048 + (m >> 4) * 128], c);
        atomicXor(&f_acc[f], c);
      }
      __syncthreads();
      if (tid < nrec) {
        const uint32_t len = f_len[tid];
        const uint32_t crc = ~(f_acc[tid] ^ A.initc[len]);
        const uint32_t masked = ((crc >> 15) | (crc << 17)) + 0xa282ead8u;  // ComputeCRC32 (utils.go:24-29)
        const uint32_t h = f_hdr[tid];
        img_put(img, h + 0, (uint8_t)masked);
        img_put(img, h + 1, (uint8_t)(masked >> 8));
        img_put(img, h + 2, (uint8_t)(masked >> 16));
        img_put(img, h + 3, (uint8_t)(masked >> 24));
        img_put(img, h + 4, (uint8_t)len);
        img_put(img, h + 5, (uint8_t)(len >> 8));
        img_put(img, h + 6, f_type[tid]);
      }
      __syncthreads();
      if (nrec < kRecBatch) break;
    }
    // ---- (4) store image [lo, hi) at out[file - pos]: aligned 16 B stores, bytes at the edges ----
    if (!(A.abl & 8)) {
      const int64_t base = (int64_t)(40 + k * kL) - (int64_t)A.pos;  // out offset of image byte 0
      const int64_t o0 = base + D.lo, o1 = base + D.hi;
      const int64_t a0 = (o0 + 15) & ~15ll, a1 = o1 & ~15ll;
      if (a0 >= a1) {
        for (int64_t o = o0 + tid; o < o1; o += kPT) A.out[o] = img_get(img, (uint32_t)(o - base));
      } else {
        for (int64_t o = o0 + tid; o < a0; o += kPT) A.out[o] = img_get(img, (uint32_t)(o - base));
        for (int64_t o = a1 + tid; o < o1; o += kPT) A.out[o] = img_get(img, (uint32_t)(o - base));
        const uint32_t sh = (uint32_t)((a0 - base) & 3);
        for (int64_t o = a0 + 16 * (int64_t)tid; o < a1; o += 16 * kPT) {
          const uint32_t ib = (uint32_t)(o - base);
          const uint32_t w0 = ib >> 2;
          uint4 v;
          if (sh == 0) {
            if ((w0 & 3u) == 0) v = *reinterpret_cast<const uint4*>(&img[iw(w0)]);
            else v = make_uint4(img[iw(w0)], img[iw(w0 + 1)], img[iw(w0 + 2)], img[iw(w0 + 3)]);
          } else {
            const uint32_t x0 = img[iw(w0)], x1 = img[iw(w0 + 1)], x2 = img[iw(w0 + 2)], x3 = img[iw(w0 + 3)],
                           x4 = img[iw(w0 + 4)];
            v = make_uint4(__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                           __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh));
          }
          __builtin_nontemporal_store(v.x, reinterpret_cast<uint32_t*>(A.out + o));
          __builtin_nontemporal_store(v.y, reinterpret_cast<uint32_t*>(A.out + o) + 1);
          __builtin_nontemporal_store(v.z, reinterpret_cast<uint32_t*>(A.out + o) + 2);
          __builtin_nontemporal_store(v.w, reinterpret_cast<uint32_t*>(A.out + o) + 3);
        }
      }
    }
    __syncthreads();  // the image is reused by the next block
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
  if ((err >> 2) < nin) {
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
  const uint64_t rows = L.rows;
  const bool compact = L.p.mode == BCW_ENC_COMPACT;
  TileSum* tiles = static_cast<TileSum*>(s.tiles);
  Ev* evs = static_cast<Ev*>(s.ev);
  BlkDesc* desc_w = static_cast<BlkDesc*>(s.desc_w);
  BlkDesc* desc_h = static_cast<BlkDesc*>(s.desc_h);
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
  auto layout = [&](int lay, const uint64_t* da, uint64_t pos, BlkDesc* desc, uint64_t desc_cap) {
    const int kid = lay == 1 ? K_ENC_EVENTS_HINT : K_ENC_EVENTS;
    pr.begin(kid, st, ev0);
    k_events<<<1, kEvThreads, 0, st>>>(da, s.emisc, lay, pos - 40, evs, s.evb);
    pr.end(kid, st, ev0);
    k_blkdesc<<<(uint32_t)((desc_cap + 255) / 256), 256, 0, st>>>(da, s.emisc, lay, evs, desc, desc_cap);
  };
  PackArgs A{};
  A.e = e;
  A.rd = s.recdesc;
  A.emisc = s.emisc;
  A.crc_ops = L.crc_ops;
  A.initc = L.initc;
  {
    static const char* ev = getenv("BCW_PACK_ABL");
    A.abl = ev ? (uint32_t)atoi(ev) : 0u;
  }
  const uint32_t rgrid = (uint32_t)((rows + 255) / 256) + 1;
  RecDesc* rdp = static_cast<RecDesc*>(s.recdesc);
  // persistent pack grid: two 512-thread workgroups per CU (LDS ~75 KiB each)
  auto pgrid = [&](uint64_t blocks) { return (uint32_t)std::min<uint64_t>(blocks, (uint64_t)L.num_cus * 2); };
  if (compact) {
    pr.begin(K_ENC_SCAN, st, ev0);
    scan(s.sz, 1, 0, s.da);
    pr.end(K_ENC_SCAN, st, ev0);
    layout(0, s.da, L.p.wal_pos, desc_w, s.blk_cap_w);
    k_recoff<<<rgrid, 256, 0, st>>>(s.da, s.dsrc, s.emisc, 0, evs, s.evb, s.dpos, L.out.rec_off);
    A.da = s.da;
    A.desc = desc_w;
    A.lay = 0;
    A.out = L.out.wal;
    A.pos = L.p.wal_pos;
    A.cap = L.out.wal_cap;
    pr.begin(K_ENC_PACK, st, ev0);
    k_recdesc<PM_DST><<<rgrid, 256, 0, st>>>(e, s.emisc, s.dsrc, nullptr, nullptr, s.mflag, rdp);
    k_pack<PM_DST><<<pgrid(s.blk_cap_w), kPT, 0, st>>>(A);
    pr.end(K_ENC_PACK, st, ev0);
    // the hint WAL only needs the dst offsets: its layout and pack run on the auxiliary stream,
    // beside the dst pack
    hipStream_t sh = L.aux ? L.aux : st;
    if (L.aux) {
      (void)hipEventRecord(L.ev_fork, st);
      (void)hipStreamWaitEvent(sh, L.ev_fork, 0);
    }
    k_hint_sizes<<<rgrid, 256, 0, sh>>>(e, s.emisc, s.dsrc, s.da, s.dpos, s.hsz);
    {
      hipStream_t keep = st;
      st = sh;
      scan(s.hsz, 0, 1, s.hda);
      layout(1, s.hda, L.p.hint_pos, desc_h, s.blk_cap_h);
      st = keep;
    }
    PackArgs H = A;
    H.da = s.hda;
    H.rd = s.recdesc_h;
    H.desc = desc_h;
    H.lay = 1;
    H.out = L.out.hint;
    H.pos = L.p.hint_pos;
    H.cap = L.out.hint_cap;
    pr.begin(K_ENC_PACK_HINT, sh, ev0);
    k_recdesc<PM_HINT_DST><<<rgrid, 256, 0, sh>>>(e, s.emisc, s.dsrc, s.da, s.dpos, s.mflag,
                                                  static_cast<RecDesc*>(s.recdesc_h));
    k_pack<PM_HINT_DST><<<pgrid(s.blk_cap_h), kPT, 0, sh>>>(H);
    pr.end(K_ENC_PACK_HINT, sh, ev0);
    if (L.aux) {
      (void)hipEventRecord(L.ev_join, sh);
      (void)hipStreamWaitEvent(st, L.ev_join, 0);
    }
  } else {
    pr.begin(K_ENC_SCAN, st, ev0);
    scan(s.sz, 1, 0, s.hda);
    pr.end(K_ENC_SCAN, st, ev0);
    layout(0, s.hda, L.p.hint_pos, desc_h, s.blk_cap_h);
    A.da = s.hda;
    A.desc = desc_h;
    A.lay = 0;
    A.out = L.out.hint;
    A.pos = L.p.hint_pos;
    A.cap = L.out.hint_cap;
    pr.begin(K_ENC_PACK_HINT, st, ev0);
    k_recdesc<PM_HINT_SRC><<<rgrid, 256, 0, st>>>(e, s.emisc, s.dsrc, nullptr, nullptr, s.mflag, rdp);
    k_pack<PM_HINT_SRC><<<pgrid(s.blk_cap_h), kPT, 0, st>>>(A);
    pr.end(K_ENC_PACK_HINT, st, ev0);
  }
  k_enc_finalize<<<1, 1, 0, st>>>(s.emisc, L.p.mode, L.p.wal_pos, L.out.wal_cap, L.p.hint_pos, L.out.hint_cap,
                                  L.d_src_result, L.d_result);
  return hipGetLastError();
}

size_t enc_sizeof_ev() { return sizeof(enc::Ev); }
size_t enc_sizeof_recdesc() { return sizeof(enc::RecDesc); }
size_t enc_sizeof_desc() { return sizeof(enc::BlkDesc); }
size_t enc_sizeof_tile() { return sizeof(enc::TileSum); }
int enc_tile_items() { return enc::kTileItems; }
int enc_ev_win() { return enc::kEvWin; }

}  // namespace bcw
