// bcw_decode.hip -- MI355X (gfx950) kernels for bitcaskDB WAL segment decode + CRC verify.
//
// Pipeline (one HIP stream, no host synchronisation inside):
//   k_chase    one lane per 32 KiB block: header chase (wal_iterator.go:45-77), workgroup scan of the
//              fragment counts, decoupled look-back over workgroups, fragment table
//   k_crc      one workgroup per CU: per-fragment masked CRC-32C verify as a zero test
//              (wal_iterator.go:79 / utils.go:24-29), then the record-state transforms of the iterator's
//              state machine (wal_iterator.go:69-96) per block, per wave, per workgroup; the last
//              workgroup scans the workgroup aggregates (record bases, first error)
//   k_records  record emission + RecordFromBytes (record.go:140-239) / HintRecord.Decode
//              (hint.go:50-84), one lane per record; the last workgroup writes bcw_decode_result
#include <hip/hip_runtime.h>

#include <cstdint>

#include "bcw_internal.h"
#include "bcw_parse.h"

namespace bcw {

// ------------------------------------------------------------------------------------------
// misc counters (Scratch::misc)
enum { M_FIRST_BAD = 0,  // first record whose parse fails (atomicMin in k_crc's emission)
       M_NE = 1,         // Full/Last fragments of the whole segment (k_chase)
       M_NFRAGS = 4, M_DONE_CRC = 5,
       M_T_CRC0 = 10, M_T_FIN = 11,  // wall_clock64 stamps (diagnostics)
       M_ABORT = 12,     // k_scan: the wait site that timed out (0: none); reported as BCW_ERR_INTERNAL
       M_TICKET = 13,    // k_chase workgroup tickets (monotonic across launches)
       M_BAD_CRC = 14,   // first fragment failing its CRC (atomicMin in k_crc; reset by the finalize)
       M_BAD_TYPE = 15 };  // first fragment of an unknown type (atomicMin in k_chase; reset by k_crc's finalize)

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
// Workgroup-level exclusive scan helpers (256 threads = 4 waves).
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += t;
  }
  return v;
}
// ---- wave-level scans on DPP (row_shr 1/2/4/8, row_bcast 15/31), no LDS round trips ----
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
// zero-filled DPP move: lanes without a source (row edges, rows outside ROWMASK) read 0, so inclusive OR / ADD /
// unsigned-MAX scans need no per-step lane conditions (one DPP-operand VALU per step)
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ uint32_t dpp_z(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWMASK, 0xf, true);
}
template <typename Op>
__device__ __forceinline__ uint32_t wave_scan_z(uint32_t v, Op op) {
  v = op(v, dpp_z<0x111>(v));
  v = op(v, dpp_z<0x112>(v));
  v = op(v, dpp_z<0x114>(v));
  v = op(v, dpp_z<0x118>(v));
  v = op(v, dpp_z<0x142, 0xa>(v));  // row 0 / 2 totals into rows 1 / 3
  v = op(v, dpp_z<0x143, 0xc>(v));  // lane 31 into rows 2, 3
  return v;
}
__device__ __forceinline__ uint32_t wave_max_scan(uint32_t v, uint32_t) {
  return wave_scan_z(v, [](uint32_t x, uint32_t y) { return max(x, y); });
}
__device__ __forceinline__ uint32_t wave_or_scan(uint32_t v, uint32_t) {
  return wave_scan_z(v, [](uint32_t x, uint32_t y) { return x | y; });
}
__device__ __forceinline__ uint32_t wave_add_scan(uint32_t v, uint32_t) {
  return wave_scan_z(v, [](uint32_t x, uint32_t y) { return x + y; });
}

// returns the exclusive prefix of v over the workgroup; *total = workgroup sum
__device__ __forceinline__ uint32_t wg256_excl_scan(uint32_t v, uint32_t* sm4, uint32_t& total) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t incl = wave_incl_scan_u32(v, lane);
  if (lane == 63) sm4[wave] = incl;
  __syncthreads();
  uint32_t base = 0;
  for (uint32_t k = 0; k < wave; ++k) base += sm4[k];
  total = sm4[0] + sm4[1] + sm4[2] + sm4[3];
  __syncthreads();
  return base + incl - v;
}

// ------------------------------------------------------------------------------------------
// Single-pass header chase with a decoupled look-back over workgroups: every lane of a one-wave
// workgroup chases one block (keeping its first kChaseHold headers in LDS), the wave scans the counts,
// publishes its aggregate and walks back over earlier workgroups' published values for its fragment
// base, then writes the fragment table (a block with more headers chases its tail again; the lines are
// cache-resident by then). Workgroups take tickets in launch order, so a workgroup only ever waits on
// ones already running. Look-back words: epoch << 40 | flag << 38 | count (flag 1: aggregate,
// 2: inclusive prefix). One wave per workgroup spreads the blocks over every CU: the chase is a chain
// of scattered header reads, bound by latency and by each CU's address-processing rate.
//
// The chase is the iterator's header loop (wal_iterator.go:45-77: the block's buffer is
// min(32768, Size - fileOff) bytes, a header is parsed while bufOff + 7 <= bufSize, the data length is
// clamped to the buffer), a dependent chain of header reads. To shorten it, once two consecutive Full
// fragments of the block had the same length (a run of equal-size records, as in every 4 KiB-value
// block), a round issues kSpec header loads at once at the positions that stride predicts and consumes
// them while each lies exactly where the chain arrives; the round ends at the first mismatch and the
// next one starts from the true position. Without that evidence a round reads one header. (Speculating
// right after the first Full fragment, until a prediction fails, measured slower: config B k_chase
// 27.4 -> 28.2 us, config C 83 -> 91 us.)
// A bounded wait (k_chase, k_scan): every spin gives up after 200 ms (a correct wait lasts microseconds)
// or once another wave has given up, records its site in misc[M_ABORT] and lets the kernel run to its end; the decode
// then reports BCW_ERR_INTERNAL instead of hanging the device.
struct Spin {
  uint64_t t0 = 0;
  __device__ __forceinline__ bool go(uint64_t* misc, uint32_t site) {  // true: keep waiting
    const uint64_t t = wall_clock64();
    if (t0 == 0) t0 = t;
    if (t - t0 < 20000000ull &&
        __hip_atomic_load(&misc[M_ABORT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0ull) {
      __builtin_amdgcn_s_sleep(1);
      return true;
    }
    atomicMax(reinterpret_cast<unsigned long long*>(&misc[M_ABORT]), (unsigned long long)site);
    return false;
  }
};

constexpr int kSpec = 8;
constexpr int kChaseHold = 16;
constexpr uint64_t kLbAgg = 1, kLbInc = 2, kLbMask = (1ull << 38) - 1;
constexpr int kDirect = BCW_CHASE_DIRECT_MAX;  // k_chase workgroups up to which each sums all predecessors' aggregates

// visit(k, start, len, crc, type) for every header of the block; returns the fragment count
template <typename V>
__device__ __forceinline__ uint32_t chase_block(const uint8_t* __restrict__ seg, uint64_t seg_len, uint64_t boff,
                                                uint32_t bufsize, V&& visit, uint32_t h = 0, uint32_t n = 0) {
  uint32_t s = 0;      // predicted distance to the next header (0: read one header)
  uint32_t lfull = 0;  // length of the last Full fragment (+1; 0: none)
  while (h + kHdr <= bufsize) {
    uint32_t cr[kSpec], ln[kSpec], ty[kSpec];
    read_header(seg, seg_len, boff + h, cr[0], ln[0], ty[0]);
#pragma unroll
    for (int j = 1; j < kSpec; ++j) {
      const uint32_t p = h + (uint32_t)j * s;
      cr[j] = ln[j] = ty[j] = 0;
      if (s != 0 && p + kHdr <= bufsize) read_header(seg, seg_len, boff + p, cr[j], ln[j], ty[j]);
    }
    const uint32_t h0 = h, s0 = s;
#pragma unroll
    for (int j = 0; j < kSpec; ++j) {
      if (j > 0 && (s0 == 0 || h != h0 + (uint32_t)j * s0 || h + kHdr > bufsize)) break;
      const uint32_t start = h + kHdr;
      uint32_t len = ln[j];
      if (len > bufsize - start) len = bufsize - start;
      visit(n, start, len, cr[j], ty[j]);
      ++n;
      h = start + len;
      if (ty[j] == BCW_RECORD_FULL) {
        s = (lfull == len + 1) ? kHdr + len : 0;
        lfull = len + 1;
      } else {
        s = 0;
      }
    }
  }
  return n;
}

// the fragment table entry; the stored CRC is kept as the check word J (see Frag)
__device__ __forceinline__ void put_frag(Frag* __restrict__ frags, uint64_t g, uint64_t frag_cap, uint32_t b,
                                         uint32_t start, uint32_t len, uint32_t crc, uint32_t type,
                                         const uint32_t* __restrict__ initc) {
  if (g >= frag_cap) return;
  Frag f;
  f.blk = b;
  f.start = (uint16_t)start;
  f.len = (uint16_t)len;
  f.chk = ~rotl32(crc - 0xa282ead8u, 15) ^ initc[len];
  f.type = (uint8_t)type;
  f.ok = 0;
  f.pad = 0;
  frags[g] = f;
}

// Block summary for the record state machine (wal_iterator.go:69-96), written by k_chase from the headers alone:
// the state of the iterator after a block depends only on the fragment types and lengths before it (a CRC
// failure or unknown type ends the iteration, and nothing after the first failing fragment is emitted), so
// record emission needs no CRC verdict. x = tail length | tail first non-empty fragment (block-local index,
// 0xffff: none) << 16; y = that fragment's block-relative start | has-Full/Last << 16. The tail is the part
// after the block's last Full/Last fragment (the whole block when it has none).
constexpr uint32_t kSumHasE = 1u << 16;
constexpr int kEqStride = 32;  // k_crc's per-XCD emission queue heads: 128 B apart

// ABL: ablation bits for tools/kbench only (0 in the product): 1 no predecessor sum, 2 no table writes,
// 16 phase cycles (chase, sum, writes; s_memtime) summed into misc[7..9]
template <int ABL = 0>
__global__ __launch_bounds__(64) void k_chase(const uint8_t* __restrict__ seg, uint64_t seg_len, uint32_t start_off,
                                              uint64_t nblocks, uint32_t* __restrict__ fbase,
                                              uint32_t* __restrict__ rbase, uint2* __restrict__ bsum,
                                              Frag* __restrict__ frags, uint64_t frag_cap, uint64_t* __restrict__ lb,
                                              uint64_t* __restrict__ lbe, uint64_t* __restrict__ misc,
                                              uint64_t ticket_base, uint64_t epoch, const uint32_t* __restrict__ initc,
                                              uint32_t direct_max, uint32_t* __restrict__ equeue) {
  // {crc, start | len << 16} and type of each lane's headers: 9 KiB, so a k_chase workgroup fits beside a k_crc
  // workgroup (which leaves 11 KiB of the CU's LDS) when another segment's decode is in flight
  // (ABL & 256, kbench: 64 held headers per lane)
  constexpr int kHold = (ABL & 256) ? 64 : kChaseHold;
  __shared__ uint32_t s_hold[kHold][2][64];
  __shared__ uint8_t s_type[kHold][64];
  const uint32_t lane = threadIdx.x;
  const uint64_t tc0 = (ABL & 16) ? __builtin_amdgcn_s_memtime() : 0;
  uint64_t wg = 0;
  if (lane == 0) wg = atomicAdd(reinterpret_cast<unsigned long long*>(&misc[M_TICKET]), 1ull) - ticket_base;
  wg = (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)wg) |
       ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(wg >> 32)) << 32);
  const uint64_t b = wg * 64 + lane;
  uint32_t bufsize = 0;
  uint64_t boff = 0;
  if (b < nblocks) {
    boff = (uint64_t)start_off + b * kBlock;
    bufsize = (uint32_t)((seg_len - boff) < kBlock ? (seg_len - boff) : kBlock);
  }
  // record-state summary of the block (see kSumHasE) and its first unknown-type fragment
  uint32_t ne = 0, tacc = 0, tnz = 0xffffu, tst = 0, badk = 0xffffffffu;
  uint32_t hres = 0;  // where the first header past the held ones starts (the table pass resumes there)
  const uint32_t n = chase_block(seg, seg_len, boff, bufsize,
                                 [&](uint32_t k, uint32_t start, uint32_t len, uint32_t crc, uint32_t type) {
                                   if (k < (uint32_t)kHold) {
                                     s_hold[k][0][lane] = crc;
                                     s_hold[k][1][lane] = start | (len << 16);
                                     s_type[k][lane] = (uint8_t)type;
                                   }
                                   if (k == (uint32_t)kHold - 1u) hres = start + len;
                                   if (type == BCW_RECORD_FULL || type == BCW_RECORD_LAST) {
                                     ++ne;
                                     tacc = 0;
                                     tnz = 0xffffu;
                                   } else {
                                     if (len > 0 && tnz == 0xffffu) { tnz = k; tst = start; }
                                     tacc += len;
                                     if ((type < BCW_RECORD_FULL || type > BCW_RECORD_LAST) && badk == 0xffffffffu) badk = k;
                                   }
                                 });
  const uint64_t tc1 = (ABL & 16) ? __builtin_amdgcn_s_memtime() : 0;
  const uint32_t incl = wave_add_scan(n, lane);
  const uint32_t tot = __builtin_amdgcn_readlane(incl, 63);
  const uint32_t incl_e = wave_add_scan(ne, lane);
  const uint32_t tot_e = __builtin_amdgcn_readlane(incl_e, 63);
  // publish, then sum the predecessors. Up to kDirect workgroups (a 2 GiB segment) every workgroup publishes
  // only its aggregate (fragment and Full/Last counts packed: at most 64 * 4681 < 2^19 each) and sums all of its
  // predecessors' at once (up to kDirect / 64 loads per lane, all in flight); beyond that, the decoupled look-back
  // (64 predecessors per step, stopping at the nearest inclusive prefix, one word array per count), whose chain of
  // inclusive prefixes would otherwise serialize the workgroups.
  const uint64_t tag = epoch << 40;
  const uint64_t nwg_all = (nblocks + 63) / 64;
  uint64_t excl = 0, excl_e = 0;
  if (ABL & 1) {
  } else if (nwg_all <= (uint64_t)direct_max) {  // direct_max <= kDirect (bcw_ctx_set_option)
    if (lane == 0)
      __hip_atomic_store(&lb[wg], tag | (kLbAgg << 38) | tot | ((uint64_t)tot_e << 19), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    uint64_t v[kDirect / 64];
#pragma unroll
    for (int k = 0; k < kDirect / 64; ++k) {
      const uint64_t q = lane + 64u * k;
      v[k] = q < wg ? __hip_atomic_load(&lb[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : tag;
    }
    uint64_t c = 0, ce = 0;
#pragma unroll
    for (int k = 0; k < kDirect / 64; ++k) {
      const uint64_t q = lane + 64u * k;
      Spin sp;  // bounded (BCW_ERR_INTERNAL), like every k_scan wait
      while ((v[k] >> 40) != epoch) {
        if (!sp.go(misc, 9)) break;
        v[k] = __hip_atomic_load(&lb[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (q < wg) {
        c += v[k] & 0x7ffffu;
        ce += (v[k] >> 19) & 0x7ffffu;
      }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      c += (uint64_t)__shfl_xor((long long)c, d, 64);
      ce += (uint64_t)__shfl_xor((long long)ce, d, 64);
    }
    excl = c;
    excl_e = ce;
  } else {
    const uint64_t fl = (wg == 0 ? kLbInc : kLbAgg) << 38;
    if (lane == 0) {
      __hip_atomic_store(&lb[wg], tag | fl | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&lbe[wg], tag | fl | tot_e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // both counts walk back together; each stops at its own nearest inclusive prefix (the two words of a
    // predecessor turn inclusive one after the other)
    bool dn = false, de = false;
    for (uint64_t top = wg; top > 0 && !(dn && de);) {  // predecessors [top - 64, top)
      const uint64_t q = top - 1 - lane;  // lane 0: the nearest
      uint64_t vn = 0, ve = 0;
      if (top > lane) {
        Spin sp;
        if (!dn)
          while (((vn = __hip_atomic_load(&lb[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 40) != epoch)
            if (!sp.go(misc, 10)) break;
        if (!de)
          while (((ve = __hip_atomic_load(&lbe[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 40) != epoch)
            if (!sp.go(misc, 11)) break;
      }
      auto step = [&](uint64_t v, bool& done, uint64_t& acc) {
        if (done) return;
        const uint64_t inc = __ballot(top > lane && ((v >> 38) & 3u) == kLbInc);
        const uint32_t stop = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;  // nearest inclusive prefix
        uint64_t c = (lane <= stop && top > lane) ? (v & kLbMask) : 0ull;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) c += (uint64_t)__shfl_xor((long long)c, d, 64);
        acc += c;
        done = inc != 0;
      };
      step(vn, dn, excl);
      step(ve, de, excl_e);
      top = top > 64 ? top - 64 : 0;
    }
    if (lane == 0 && wg != 0) {
      __hip_atomic_store(&lb[wg], tag | (kLbInc << 38) | ((excl + tot) & kLbMask), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&lbe[wg], tag | (kLbInc << 38) | ((excl_e + tot_e) & kLbMask), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  const uint64_t g0 = excl + incl - n;
  const uint64_t tc2 = (ABL & 16) ? __builtin_amdgcn_s_memtime() : 0;
  if (b < nblocks && !(ABL & 2)) {
    fbase[b] = (uint32_t)(g0 < 0xffffffffull ? g0 : 0xffffffffull);
    const uint64_t r0 = excl_e + incl_e - ne;
    rbase[b] = (uint32_t)(r0 < 0xffffffffull ? r0 : 0xffffffffull);
    bsum[b] = make_uint2(tacc | (tnz << 16), tst | (ne ? kSumHasE : 0u));
    if (badk != 0xffffffffu)  // the first unknown-type fragment of the segment (reset by the previous finalize)
      atomicMin(reinterpret_cast<unsigned long long*>(&misc[M_BAD_TYPE]), (unsigned long long)(g0 + badk));
    const uint32_t nh = n < (uint32_t)kHold ? n : (uint32_t)kHold;
    for (uint32_t k = 0; k < nh; ++k) {
      const uint32_t sl = s_hold[k][1][lane];
      put_frag(frags, g0 + k, frag_cap, (uint32_t)b, sl & 0xffffu, sl >> 16, s_hold[k][0][lane], s_type[k][lane],
               initc);
    }
    if (n > (uint32_t)kHold)  // the tail of a block with more headers than held, chased again from the first of them
      chase_block(seg, seg_len, boff, bufsize, [&](uint32_t k, uint32_t start, uint32_t len, uint32_t crc, uint32_t type) {
        put_frag(frags, g0 + k, frag_cap, (uint32_t)b, start, len, crc, type, initc);
      }, hres, (uint32_t)kHold);
  }
  if (ABL & 16) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t tc3 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
      atomicAdd(reinterpret_cast<unsigned long long*>(&misc[7]), (unsigned long long)(tc1 - tc0));
      atomicAdd(reinterpret_cast<unsigned long long*>(&misc[8]), (unsigned long long)(tc2 - tc1));
      atomicAdd(reinterpret_cast<unsigned long long*>(&misc[9]), (unsigned long long)(tc3 - tc2));
    }
  }
  const uint64_t nwg = (nblocks + 63) / 64;
  if (lane == 63 && !(ABL & 2)) {
    // the bases at the end of the workgroup's blocks (the next workgroup's first block writes the same values): a
    // k_crc over a leading chunk of the segment reads them before the rest is chased. k_crc's completion counter and
    // first-failure words were reset by the previous decode's finalize (or the scratch setup).
    const uint64_t total = excl + tot, total_e = excl_e + tot_e;
    const uint64_t be = wg * 64 + 64 < nblocks ? wg * 64 + 64 : nblocks;
    fbase[be] = (uint32_t)(total < 0xffffffffull ? total : 0xffffffffull);
    rbase[be] = (uint32_t)(total_e < 0xffffffffull ? total_e : 0xffffffffull);
    if (wg == nwg - 1) {
      misc[M_NFRAGS] = total;
      misc[M_NE] = total_e;
    }
  }
  if (wg == 0 && lane < 8u) equeue[lane * kEqStride] = 0;  // k_crc's emission queues
}

// ------------------------------------------------------------------------------------------
// k_crc: per-fragment CRC verify.
//
// For fragment f with data at global offsets [gs, ge) let GE = 16*ceil((ge + 4)/16) and tile
// [GE-128C, GE) with C = ceil((GE - gs)/128) windows of 128 B (16 B aligned). A raw (init 0)
// CRC-32C chain over the windows, with the bytes before gs zeroed and the bytes [ge, ge+4)
// replaced by
//     J = ~unmask(stored) ^ A_{8L}(0xFFFFFFFF)          (L = ge - gs)
// and zeros after, ends in state 0 exactly when ComputeCRC32(data) == stored (linearity of CRC:
// the init 0xFFFFFFFF contributes A_{8L}(~0) at ge, the XOR-out is folded into ~unmask). So the
// CRC check becomes a zero test of a linear functional, and windows can be computed by separate
// lanes and combined with fixed shift operators:
//   * a wave appends its fragments (64 at a time, the next group's descriptors prefetched) to a ring
//     with their window counts; every pass then takes the next 64 windows of consecutive fragments,
//     one per lane, consecutive windows of a fragment on consecutive lanes (a fragment's first window
//     has the bytes before its data masked off, its last window holds the J word). Lane l maps its end
//     state into a common frame
//     with F_l = A_{8*128*(63-l)} (lane-replicated nibble tables), a segmented XOR scan combines
//     the fragment's windows, and the lane holding the last window tests the total for zero.
//     A fragment continuing past lane 63 carries its state to the next pass, where it seeds lane 0's chain.
//     Each window runs as two independent 64 B half-chains joined by A_{8*64}; the next pass's
//     descriptors and window loads are issued before the current pass's chains (software pipeline).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int kRing = 128;               // ring of multi-window fragments per wave
constexpr int kRingWords = 6;            // cpre, cend (SoA) + 4-word entry record (AoS)
constexpr int kWaveLds = kRing * kRingWords;
constexpr size_t kCrcLds = (size_t)(kLdsSlice + kLdsFwd + kLdsOps + kCrcWaves * kWaveLds) * 4;

// CRC-32C (zero xor-out, no final inversion) of one 128 B window from state `seed`: two slice-by-4
// chains over the two 64 B halves (16 dependent steps each), joined with the half operator A_{8*64}.
// LDS slice layout: 256-B rows, row e = { T3[e] x16, T2[e] x16, T1[e] x16, T0[e] x16 } (T_k: a byte
// followed by k zero bytes), so a lookup address is (index byte << 8) | table slot | lane slot, built by
// one v_perm_b32 with a per-lane selector. Lanes 0-15 / 16-31 of each 32-lane bank group look up the
// tables of a pair in opposite orders (T3,T2 / T2,T3, then T1,T0 / T0,T1): the two table copies of a
// pair sit 16 banks apart, so every ds_read_b32 is conflict-free with 16 copies per table.
// Each chain carries x = state ^ next word: a step is 4 perm, 4 ds_read, 2 xor3.
struct SliceLane {
  uint32_t lbx, lby;    // lane slot | table-pair slot of the first / second lookup of a pair
  uint32_t s0, s1;      // perm selectors: byte k of x into byte 1, the lane base into byte 0
};
__device__ __forceinline__ SliceLane slice_lane(uint32_t lane) {
  const bool hi = (lane & 16u) != 0u;
  const uint32_t slot = (lane & 15u) * 4u;
  SliceLane s;
  s.lbx = slot + (hi ? 64u : 0u);
  s.lby = slot + (hi ? 0u : 64u);
  s.s0 = hi ? 0x0c0c0500u : 0x0c0c0400u;  // lanes 0-15: byte 0 -> T3 (slot 0); 16-31: byte 1 -> T2 (slot 64)
  s.s1 = hi ? 0x0c0c0400u : 0x0c0c0500u;
  return s;
}
__device__ __forceinline__ uint32_t slice4_step(const uint8_t* __restrict__ tb, const SliceLane& sl, uint32_t x,
                                                uint32_t next) {
  const uint32_t a0 = *reinterpret_cast<const uint32_t*>(tb + __builtin_amdgcn_perm(x, sl.lbx, sl.s0));
  const uint32_t a1 = *reinterpret_cast<const uint32_t*>(tb + __builtin_amdgcn_perm(x, sl.lby, sl.s1));
  const uint32_t a2 = *reinterpret_cast<const uint32_t*>(tb + __builtin_amdgcn_perm(x, sl.lbx, sl.s0 + 0x200u) + 128u);
  const uint32_t a3 = *reinterpret_cast<const uint32_t*>(tb + __builtin_amdgcn_perm(x, sl.lby, sl.s1 + 0x200u) + 128u);
  return a0 ^ a1 ^ a2 ^ a3 ^ next;
}
__device__ __forceinline__ uint32_t crc_window(const uint32_t* __restrict__ tab, const uint32_t* __restrict__ half,
                                               const SliceLane& sl, uint32_t seed, const uint32_t (&w)[32]) {
  const uint8_t* tb = reinterpret_cast<const uint8_t*>(tab);
  uint32_t xa = seed ^ w[0];
  uint32_t xb = w[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    xa = slice4_step(tb, sl, xa, q < 15 ? w[q + 1] : 0u);
    xb = slice4_step(tb, sl, xb, q < 15 ? w[16 + q + 1] : 0u);
  }
  uint32_t r = xb;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= half[i * 16 + ((xa >> (4 * i)) & 15u)];
  return r;
}
// F_l(x): lane-replicated nibble images, lane l reads its own copy (bank = l % 32)
__device__ __forceinline__ uint32_t apply_fwd(const uint32_t* __restrict__ fwd, uint32_t lane, uint32_t x) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= fwd[((i * 16 + ((x >> (4 * i)) & 15u)) << 6) | lane];
  return r;
}
// uniform operator (one 8x16 nibble table shared by all lanes: 16 distinct banks per lookup)
__device__ __forceinline__ uint32_t apply_op(const uint32_t* __restrict__ c, uint32_t x) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= c[i * 16 + ((x >> (4 * i)) & 15u)];
  return r;
}

// bounds-checked 16 B load (rare: the segment's first/last bytes); a rolled loop keeps it small
__device__ __forceinline__ uint4 load16_slow(const uint8_t* __restrict__ seg, uint64_t seg_len, int64_t o) {
  uint64_t lo = 0, hi = 0;
#pragma unroll 1
  for (int i = 0; i < 16; ++i) {
    const int64_t q = o + i;
    const uint64_t byte = (q >= 0 && (uint64_t)q < seg_len) ? seg[q] : 0u;
    if (i < 8) lo |= byte << (8 * i); else hi |= byte << (8 * (i - 8));
  }
  return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}
__device__ __forceinline__ uint4 load16_safe(const uint8_t* __restrict__ seg, uint64_t seg_len, int64_t o) {
  if (o >= 0 && (uint64_t)o + 16 <= seg_len) return *reinterpret_cast<const uint4*>(seg + o);
  return load16_slow(seg, seg_len, o);
}

// 128 B window at seg + goff into w[32]; `inb` (wave-uniform): every active lane's window is in bounds
__device__ __forceinline__ void load_window(const uint8_t* __restrict__ seg, uint64_t seg_len, int64_t goff, bool inb,
                                            uint32_t (&w)[32]) {
  if (inb) {
    const uint4* q = reinterpret_cast<const uint4*>(seg + goff);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const uint4 v = q[g];
      w[4 * g + 0] = v.x; w[4 * g + 1] = v.y; w[4 * g + 2] = v.z; w[4 * g + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const uint4 v = load16_safe(seg, seg_len, goff + 16 * g);
      w[4 * g + 0] = v.x; w[4 * g + 1] = v.y; w[4 * g + 2] = v.z; w[4 * g + 3] = v.w;
    }
  }
}

// last-window fix: keep bytes < hi (hi in [109,124]), put J at [hi, hi+4), zero the rest (touches words 27..31
// only). Compare-free like mask_first: word 27+i is below / at / right after word hi >> 2 by bits of 5-bit patterns.
__device__ __forceinline__ void fix_last(uint32_t (&w)[32], uint32_t hi, uint32_t J) {
  const uint32_t q = (hi >> 2) - 27u, sh = 8u * (hi & 3u);
  const uint64_t jj = (uint64_t)J << sh;
  const uint32_t jlo = (uint32_t)jj, jhi = (uint32_t)(jj >> 32);
  const uint32_t keep = (uint32_t)((1ull << sh) - 1ull);  // bytes of word hi >> 2 below hi
  const uint32_t lt = (1u << q) - 1u, eq = 1u << q, nx = 2u << q;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const uint32_t L = (uint32_t)((int32_t)(lt << (31 - i)) >> 31);
    const uint32_t E = (uint32_t)((int32_t)(eq << (31 - i)) >> 31);
    const uint32_t N = (uint32_t)((int32_t)(nx << (31 - i)) >> 31);
    w[27 + i] = (w[27 + i] & (L | (E & keep))) | (E & jlo) | (N & jhi);
  }
}

// first-window fix: zero the bytes before `lo` (the previous header / fragment), lo in [0, 127]. Piece p = lo >> 4
// (16 B, words 4p..4p+3) holds the first data byte: earlier pieces are zeroed, piece p keeps the bytes from lo & 15
// on (word masks mj), later pieces are kept. No lane-mask compares (their SGPR results cost hazard nops): -(g > p)
// and -(g < p) are sign-extended single-bit extracts of two 8-bit patterns, and each word takes one bitop3 + one and.
__device__ __forceinline__ void mask_first(uint32_t (&w)[32], uint32_t lo) {
  const uint32_t p = lo >> 4, r = lo & 15u;
  uint32_t mj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int32_t c = min(max((int32_t)r - 4 * j, 0), 4);  // bytes of word j below r
    mj[j] = (uint32_t)(0xffffffffull << (8 * c));
  }
  const uint32_t gt = 0xfeu << p;      // bit g: g > p (kept)
  const uint32_t lt = (1u << p) - 1u;  // bit g: g < p (zeroed)
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const uint32_t G = (uint32_t)((int32_t)(gt << (31 - g)) >> 31);
    const uint32_t L = (uint32_t)((int32_t)(lt << (31 - g)) >> 31);
#pragma unroll
    for (int j = 0; j < 4; ++j) w[4 * g + j] &= (mj[j] & ~L) | G;
  }
}

// global window geometry of a fragment (block-relative s, e)
struct FragGeo {
  int64_t gs, GE;
  uint32_t C;
};
__device__ __forceinline__ FragGeo frag_geo(uint32_t start_off, uint32_t blk, uint32_t s, uint32_t e) {
  const int64_t boff = (int64_t)start_off + (int64_t)blk * kBlock;
  FragGeo g;
  g.gs = boff + s;
  const int64_t ge = boff + e;
  g.GE = (ge + 4 + 15) & ~(int64_t)15;
  g.C = (uint32_t)((g.GE - g.gs + 127) >> 7);
  return g;
}

// one body-pass lane: which window, where, how to seed and finish it
struct BodyDesc {
  uint32_t woff;    // window offset relative to the wave's base (start of its first block - 128)
  uint32_t J;       // last window: the J word (the init contribution and the stored CRC)
  uint32_t fi;      // fragment index relative to the wave's first fragment
  uint32_t meta;    // hi (last window: data end within the window) | cfb << 8 | last << 17 | active << 18
                    // | lo << 19 (first window: bytes before the data)
  __device__ __forceinline__ uint32_t hi() const { return meta & 0xffu; }
  __device__ __forceinline__ uint32_t cfb() const { return (meta >> 8) & 0x1ffu; }  // window index in the fragment
  __device__ __forceinline__ bool last() const { return (meta >> 17) & 1u; }
  __device__ __forceinline__ bool active() const { return (meta >> 18) & 1u; }
  __device__ __forceinline__ uint32_t lo() const { return (meta >> 19) & 0x7fu; }
};

// ------------------------------------------------------------------------------------------
// Record emission. The iterator's per-fragment state machine (wal_iterator.go:69-96: `off` is captured
// while the accumulated record is empty; Full returns the Full's data with that offset; First/Middle
// append; Last appends and returns the record; any other type is an error; a CRC mismatch is an error)
// depends on the CRC verdicts only through the first failing fragment, after which nothing is emitted.
// So every record is emitted from the header chase alone -- by k_crc waves whose CRC passes are done, from
// per-XCD queues of ~64-fragment work items (emit_item) -- and the finalizer counts the records before the
// first failing fragment. The state entering a wave comes from k_chase's block summaries (kSumHasE): the nearest
// earlier block with a Full/Last fragment contributes its tail, the blocks after it their whole length.

// byte `pos` of a register window (N dwords, pos < 4N): a select tree on the bits of the dword index
template <int N>
__device__ __forceinline__ uint32_t reg_byte(const uint32_t (&h)[N], uint32_t pos) {
  uint32_t t[N];
#pragma unroll
  for (int i = 0; i < N; ++i) t[i] = h[i];
  const uint32_t wi = pos >> 2;
  int n = N;
#pragma unroll
  for (int bit = 0; bit < 6; ++bit) {
    if (n <= 1) break;
    const bool hi = (wi >> bit) & 1u;
#pragma unroll
    for (int i = 0; i < (N + 1) / 2; ++i) {
      if (i < (n + 1) / 2) t[i] = (2 * i + 1 < n) ? (hi ? t[2 * i + 1] : t[2 * i]) : t[2 * i];
    }
    n = (n + 1) / 2;
  }
  return (t[0] >> (8u * (pos & 3u))) & 0xffu;
}

// record bytes held in registers, loaded with unaligned 16 B loads (global_load_dwordx4 at any byte address)
constexpr int kHeadWords = 16;  // the record's first 64 B
constexpr int kTailWords = 8;   // its last 32 B (hint mode: fid, offset and size follow the key)

// byte `pos` of a record whose bytes start in fragment f_first (and end in f_last), by a walk over its fragments:
// the reader's rare slow path, out of line so that its code exists once
__device__ __attribute__((noinline)) uint32_t walk_byte(const uint8_t* __restrict__ seg, const Frag* __restrict__ frags,
                                                        uint32_t start_off, uint32_t f_first, uint32_t f_last,
                                                        uint64_t pos) {
  uint64_t beg = 0;
  for (uint32_t cf = f_first;; ++cf) {
    const Frag f = frags[cf];
    if (pos < beg + f.len || cf >= f_last)
      return seg[(uint64_t)start_off + (uint64_t)f.blk * kBlock + f.start + (pos - beg)];
    beg += f.len;
  }
}

// logical byte reader of one record: its first bytes and (hint mode) its last bytes in registers, else a
// walk over its fragments
struct RegReader {
  uint32_t h[kHeadWords];
  uint32_t t[kTailWords];
  uint32_t nhead;        // head: record bytes held
  uint64_t tstart;       // first record byte held by the tail (>= size when none)
  const uint8_t* seg;
  const Frag* frags;
  uint32_t start_off;
  uint32_t f_first, f_last;
  __device__ __forceinline__ uint32_t operator()(uint64_t pos) {
    if (pos < nhead) return reg_byte(h, (uint32_t)pos);
    if (pos >= tstart) return reg_byte(t, (uint32_t)(pos - tstart));
    return walk_byte(seg, frags, start_off, f_first, f_last, pos);
  }
};

// 4N bytes at seg + base (any alignment; bounds-checked bytes where they pass the segment end)
template <int N>
__device__ __forceinline__ void load_words(const uint8_t* __restrict__ seg, uint64_t seg_len, uint64_t base,
                                           uint32_t (&w)[N]) {
  if (base + 4u * N <= seg_len) {
#pragma unroll
    for (int k = 0; k < N / 4; ++k) {
      uint4 v;
      __builtin_memcpy(&v, seg + base + 16 * k, 16);
      w[4 * k + 0] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < N / 4; ++k) {
      const uint4 v = load16_safe(seg, seg_len, (int64_t)(base + 16 * k));
      w[4 * k + 0] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
  }
}

struct EmitArgs {
  const uint8_t* seg;
  uint64_t seg_len;
  bcw_decode_params p;
  const Frag* frags;
  const uint32_t* fbase;
  const uint32_t* rbase;
  const uint2* bsum;
  bcw_record_table tab;
  uint64_t* misc;
  uint32_t* equeue;  // [8 x kEqStride] per-XCD emission work-queue heads (reset by k_chase)
  uint32_t kb_flags; // tools/kbench only (0 in the product): 1 = skip the emission at run time
  uint64_t* kb_stamps;  // tools/kbench only (null in the product): per wave {CRC done, emission done, items}
};


// The iterator state entering block b0 (wave-uniform): the pending record's length, its first non-empty
// fragment as (block, block-local index, block-relative start), and the record row of block b0.
struct EmitState {
  uint64_t acc;
  int64_t nzb;  // -1: no non-empty fragment pending
  uint32_t nzk, nzs;
  uint64_t rec;
};
// the first walk-back step's summaries (lane l: block b0 - 1 - l), loaded ahead by the caller
__device__ __forceinline__ uint2 emit_prefetch(const EmitArgs& A, uint64_t b0, uint32_t lane) {
  return b0 > lane ? A.bsum[b0 - 1 - lane] : make_uint2(0xffff0000u, kSumHasE);
}

// k_scan: the block summaries, fragment table and block bases of an earlier workgroup's blocks (blocks < B0) were
// written inside the same launch by another CU. A wave reads them only after every predecessor has published its
// "written" word (behind an agent release) and the wave has run an agent acquire (MI355X_MICROARCH.md,
// inter-workgroup visibility: one relaxed poll, one agent acquire, s_waitcnt vmcnt(0)) -- lazily, the first time a
// walk-back has to cross B0. k_crc (whose tables come from k_chase, an earlier launch) passes B0 = 0, acq = true.
struct PredSync {
  uint64_t B0 = 0;
  const uint64_t* lbw = nullptr;  // per-workgroup "written" words (epoch << 40 | 1)
  uint64_t wg = 0, epoch = 0;
  uint64_t* misc = nullptr;  // k_scan: bounded waits (Spin)
  bool acq = true;
  __device__ __forceinline__ void acquire(uint32_t lane) {
    for (uint64_t q0 = 0; q0 < wg; q0 += 64) {
      const uint64_t q = q0 + lane;
      Spin sp;
      if (q < wg)
        while ((__hip_atomic_load(&lbw[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 40) != epoch)
          if (!sp.go(misc, 8)) break;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    acq = true;
  }
};
// walk back over the block summaries, 64 blocks a step, to the nearest block with a Full/Last fragment (before
// block 0: an empty state); s = emit_prefetch(A, b0, lane)
__device__ __forceinline__ EmitState emit_state(const EmitArgs& A, uint64_t b0, uint32_t lane, uint2 s, uint32_t rec,
                                                PredSync& ps) {
  EmitState st{0, -1, 0, 0, rec};
  uint64_t acc = 0;
  for (uint64_t top = b0; top > 0;) {
    if (top != b0) {
      const uint64_t q = top - 1 - lane;
      s = top > lane ? A.bsum[q] : make_uint2(0xffff0000u, kSumHasE);
    }
    if (!ps.acq) {  // lanes past B0 read another workgroup's summaries: acquire them unless a nearer block ends a record
      const uint64_t q = top - 1 - lane;
      const bool pred = top > lane && q < ps.B0;
      if (__ballot(pred) != 0ull && __ballot(top > lane && !pred && (s.y & kSumHasE) != 0u) == 0ull) {
        ps.acquire(lane);
        if (pred) s = A.bsum[q];
      }
    }
    const uint64_t he = __ballot((s.y & kSumHasE) != 0u);
    const uint32_t stop = he ? (uint32_t)__builtin_ctzll(he) : 63u;
    const bool contrib = lane <= stop;
    uint32_t ta = contrib ? (s.x & 0xffffu) : 0u;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) ta += (uint32_t)__shfl_xor((int)ta, d, 64);
    acc += (uint32_t)__builtin_amdgcn_readfirstlane(ta);
    const uint64_t nzm = __ballot(contrib && (s.x >> 16) != 0xffffu);
    if (nzm) {  // the earliest block (highest lane) holding a non-empty fragment of the pending record
      const uint32_t L = 63u - __builtin_clzll(nzm);
      st.nzb = (int64_t)(top - 1 - L);
      st.nzk = (uint32_t)__builtin_amdgcn_readlane((int)(s.x >> 16), L);
      st.nzs = (uint32_t)__builtin_amdgcn_readlane((int)(s.y & 0xffffu), L);
    }
    if (he) break;
    top = top > 64 ? top - 64 : 0;
  }
  st.acc = acc;
  return st;
}

// Emit the records completed by fragments [f0, f1) (one wave), entering with state es: rows of the record
// table from es.rec on, RecordFromBytes (record.go:140-239) / HintRecord.Decode (hint.go:50-84) per record,
// one lane each.
// hook(): called once, right after the first chunk's fragment descriptors are requested (the caller issues the
// next work item's loads there, so they fly beside this item's).
template <int ABL = 0, typename Hook>  // kbench ablations: 4096 no parse, 8192 no parse and no record-prefix loads
__device__ __forceinline__ void emit_chunks(const EmitArgs& A, const EmitState& es, uint64_t f0, uint64_t f1,
                                            uint32_t lane, Hook&& hook) {
  if (f0 >= f1) {
    hook();
    return;
  }
  const Frag* __restrict__ frags = A.frags;
  const uint32_t start_off = A.p.start_off;
  uint64_t acc = es.acc, off = 0;
  uint32_t first = 0;
  if (es.nzb >= 0) {
    off = (uint64_t)start_off + (uint64_t)es.nzb * kBlock + es.nzs;
    first = A.fbase[es.nzb] + es.nzk;
  }
  uint64_t rec = es.rec;
  const bool hint = A.p.mode == BCW_MODE_HINT;
  for (uint64_t c0 = f0; c0 < f1; c0 += 64) {
    const uint64_t g = c0 + lane;
    const bool valid = g < f1;
    // unconditional (clamped) load: a branch around it would make the compiler wait for it at the merge
    const uint4 fr = reinterpret_cast<const uint4*>(frags)[valid ? g : f1 - 1];
    if (c0 == f0) hook();
    Frag f;
    __builtin_memcpy(&f, &fr, sizeof f);
    if (!valid) f = Frag{};
    const uint32_t len = valid ? f.len : 0u;
    const uint64_t D = (uint64_t)start_off + (uint64_t)f.blk * kBlock + f.start;
    const bool isE = valid && (f.type == BCW_RECORD_FULL || f.type == BCW_RECORD_LAST);
    const uint64_t E = __ballot(isE);
    const uint64_t NZ = __ballot(valid && len > 0);
    const uint32_t S = wave_add_scan(len, lane);  // inclusive prefix of lengths
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint64_t pm = E & below;
    const int prev = pm ? 63 - __builtin_clzll(pm) : -1;
    const uint32_t S_prev = __shfl(S, prev < 0 ? 0 : prev, 64);
    const uint64_t between = (uint64_t)(S - len) - (prev < 0 ? 0u : S_prev);  // lengths in (prev, lane)
    const uint64_t acc_before = (prev < 0 ? acc : 0ull) + between;
    const uint64_t range = prev < 0 ? below : (below & ~(~0ull >> (63 - prev)));
    const uint64_t nzr = NZ & range;
    const int fnz = nzr ? __builtin_ctzll(nzr) : 0;
    const uint64_t D_fnz = __shfl(D, fnz, 64);
    // chunk carry-out (state after the last emission of the chunk, or the extended incoming state)
    const uint64_t V = __ballot(valid);
    const int last_valid = V ? 63 - __builtin_clzll(V) : -1;
    const uint32_t S_tot = __shfl(S, last_valid < 0 ? 0 : last_valid, 64);
    const int lastE = E ? 63 - __builtin_clzll(E) : -1;
    uint64_t acc2, off2;
    uint32_t first2;
    {
      const uint32_t S_lastE = __shfl(S, lastE < 0 ? 0 : lastE, 64);
      const uint64_t after = lastE < 0 ? V : (V & ~(~0ull >> (63 - lastE)));
      const uint64_t nza = NZ & after;
      const int fa = nza ? __builtin_ctzll(nza) : 0;
      const uint64_t D_fa = __shfl(D, fa, 64);
      if (lastE >= 0) {
        acc2 = (uint64_t)(S_tot - S_lastE);
        off2 = D_fa;
        first2 = (uint32_t)(c0 + fa);
      } else {
        acc2 = acc + S_tot;
        if (acc > 0 || !nza) { off2 = off; first2 = first; }
        else { off2 = D_fa; first2 = (uint32_t)(c0 + fa); }
      }
    }
    // the record each emitting lane completes (evaluated by every lane: the shuffles need all lanes)
    uint64_t foff;
    uint32_t ffrag;
    if (acc_before == 0) { foff = D; ffrag = (uint32_t)g; }
    else if (prev < 0 && acc > 0) { foff = off; ffrag = first; }
    else { foff = D_fnz; ffrag = (uint32_t)(c0 + fnz); }
    const bool full = f.type == BCW_RECORD_FULL;
    const uint32_t src = full ? (uint32_t)g : ffrag;  // the record's bytes start in fragment src
    const bool src_here = src >= c0 && src < c0 + 64;
    const uint32_t sw0 = (uint32_t)__shfl((int)f.blk, src_here ? (int)(src - c0) : (int)lane, 64);
    const uint32_t sw1 = (uint32_t)__shfl((int)((uint32_t)f.start | ((uint32_t)f.len << 16)),
                                          src_here ? (int)(src - c0) : (int)lane, 64);
    if (isE) {
      const uint64_t size = full ? (uint64_t)len : acc_before + len;
      const uint64_t r = rec + __builtin_popcountll(E & below);
      Frag fs = f;
      if (!full) {
        if (src_here) { fs.blk = sw0; fs.start = (uint16_t)sw1; fs.len = (uint16_t)(sw1 >> 16); }
        else fs = frags[src];
      }
      RegReader rd;
      const uint64_t a0 = (uint64_t)start_off + (uint64_t)fs.blk * kBlock + fs.start;
      uint64_t want = size < 64u ? size : 64u;
      if (want > fs.len) want = fs.len;
      rd.nhead = (uint32_t)want;
      if (ABL & 8192) {
#pragma unroll
        for (int k = 0; k < kHeadWords; ++k) rd.h[k] = 0;
      } else {
        load_words(A.seg, A.seg_len, a0, rd.h);
      }
      rd.tstart = ~0ull;
      if (hint) {  // the last bytes: HintRecord.Decode reads fid, offset and size after the key
        uint64_t nt = size < 32u ? size : 32u;
        if (nt > len) nt = len;
        rd.tstart = size - nt;
        load_words(A.seg, A.seg_len, D + len - nt, rd.t);  // this lane's (Full/Last) fragment ends the record
      } else {
#pragma unroll
        for (int k = 0; k < kTailWords; ++k) rd.t[k] = 0;
      }
      rd.seg = A.seg; rd.frags = frags; rd.start_off = start_off;
      rd.f_first = src; rd.f_last = (uint32_t)g;
      uint8_t status, hdr, flags, etag_off;
      uint64_t key_len, val_len, meta_len, expire, aux0, aux1;
      if (ABL & (4096 | 8192)) {
        status = (uint8_t)(rd.h[0] == 0x12345u);
        hdr = flags = etag_off = 0;
        key_len = val_len = meta_len = expire = aux0 = aux1 = rd.h[1];
      } else {
        parse_record(A.p, rd, size, status, hdr, flags, etag_off, key_len, val_len, meta_len, expire, aux0, aux1);
      }
      const bcw_record_table& tab = A.tab;
      if (r < tab.capacity) {
        tab.foff[r] = foff;
        tab.size[r] = size;
        tab.expire[r] = expire;
        if (tab.aux0) tab.aux0[r] = aux0;
        if (tab.aux1) tab.aux1[r] = aux1;
        tab.key_len[r] = (uint32_t)key_len;
        tab.val_len[r] = (uint32_t)val_len;
        tab.meta_len[r] = (uint32_t)meta_len;
        tab.first_frag[r] = src;
        tab.emit_frag[r] = (uint32_t)g;
        tab.hdr_size[r] = hdr;
        tab.flags[r] = flags;
        tab.etag_off[r] = etag_off;
        tab.status[r] = status;
      }
      if (status != BCW_ST_OK) atomicMin((unsigned long long*)&A.misc[M_FIRST_BAD], (unsigned long long)r);
    }
    rec += __builtin_popcountll(E);
    acc = acc2;
    off = off2;
    first = first2;
  }
}

// Emission work item `it`: the records completed by the fragments of blocks [it * bpw, (it + 1) * bpw) (about 64
// fragments), by whichever k_crc wave takes it from its XCD's queue once its own CRC passes are done -- the waves
// that finish early emit for the whole segment, so the last wave to finish its CRC seldom finds work left.
struct ItemMeta {
  uint64_t bb;
  uint2 s;  // emit_prefetch of block bb
  uint32_t f0, f1, rec;
};
// item `it` of a chunk [cb0, cb1) of the segment's blocks: blocks [cb0 + it bpw, + bpw), cut at cb1
__device__ __forceinline__ ItemMeta item_meta(const EmitArgs& A, uint64_t it, uint64_t bpw, uint64_t cb0, uint64_t cb1,
                                              uint32_t lane) {
  ItemMeta m;
  m.bb = cb0 + it * bpw < cb1 ? cb0 + it * bpw : cb1 - 1;  // a clamped (unconditional) load for an exhausted queue
  const uint64_t be = m.bb + bpw < cb1 ? m.bb + bpw : cb1;
  m.s = emit_prefetch(A, m.bb, lane);
  m.f0 = A.fbase[m.bb];
  m.f1 = A.fbase[be];
  m.rec = A.rbase[m.bb];
  return m;
}

// The segment result, by one wave once every k_crc wave has verified and emitted: the first failing fragment
// is the earlier of the first CRC mismatch and the first unknown type (at the same fragment the CRC is
// checked first, wal_iterator.go:79-95), and the records before it are the Full/Last fragments before it.
__device__ __forceinline__ void finalize(const EmitArgs& A, uint64_t nblocks, uint64_t frag_cap, uint32_t tail_panic, uint64_t gen,
                         bcw_decode_result* __restrict__ res, uint32_t lane) {
  uint64_t* misc = A.misc;
  const uint64_t bad_crc = __hip_atomic_load(&misc[M_BAD_CRC], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t bad_type = __hip_atomic_load(&misc[M_BAD_TYPE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t fb = __hip_atomic_load(&misc[M_FIRST_BAD], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t nfr = __hip_atomic_load(&misc[M_NFRAGS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t err = bad_crc < bad_type ? bad_crc : bad_type;
  // records before fragment `lim` (the first failing one, or the fragment capacity of a decode to be retried)
  uint64_t lim = err < frag_cap ? err : frag_cap;
  uint64_t nrec = __hip_atomic_load(&misc[M_NE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // k_scan wrote the block bases and the fragment table inside this launch, on other CUs: every workgroup has
  // completed (its written word preceded its completion), so one agent acquire makes them readable here
  if (lim < nfr || err != ~0ull) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (lim < nfr) {
    // the block holding fragment lim: the last b with fbase[b] <= lim (64-ary search)
    uint64_t lo = 0, hi = nblocks;
    while (hi - lo > 1) {
      const uint64_t step = (hi - lo + 63) / 64;
      const uint64_t q = lo + (uint64_t)lane * step;
      const bool le = q < hi && A.fbase[q] <= lim;
      const uint64_t m = __ballot(le);
      const uint32_t L = m ? 63u - __builtin_clzll(m) : 0u;
      lo = lo + (uint64_t)L * step;
      hi = lo + step < hi ? lo + step : hi;
    }
    uint64_t cnt = 0;
    for (uint64_t c0 = A.fbase[lo]; c0 < lim; c0 += 64) {
      const uint64_t g = c0 + lane;
      const uint32_t ty = g < lim ? A.frags[g].type : 0u;
      cnt += (uint64_t)__builtin_popcountll(__ballot(ty == BCW_RECORD_FULL || ty == BCW_RECORD_LAST));
    }
    nrec = (uint64_t)A.rbase[lo] + cnt;
  }
  if (lane != 0) return;
  bcw_decode_result r{};
  r.n_records = nrec;
  r.n_records_total = nrec;
  r.err_frag = err;
  r.err_class = err == ~0ull ? BCW_ERR_NONE : (bad_crc <= bad_type ? BCW_ERR_CRC : BCW_ERR_TYPE);
  r.n_frags = err != ~0ull ? err + 1 : nfr;
  // a last block of 1..6 bytes makes the reference iterator panic after every earlier record
  // (wal_iterator.go:62-76 re-slices a header from its stale buffer, then buf[7:7+negative])
  if (r.err_class == BCW_ERR_NONE && tail_panic) r.err_class = BCW_ERR_PANIC;
  if (__hip_atomic_load(&misc[M_ABORT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0ull) {
    r.err_class = BCW_ERR_INTERNAL;
    r.err_frag = __hip_atomic_load(&misc[M_ABORT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the wait site
  }
  r.err_file_off = 0;
  if (err != ~0ull && err < frag_cap) {
    const Frag f = A.frags[err];
    r.err_file_off = (uint64_t)A.p.start_off + (uint64_t)f.blk * kBlock + f.start - kHdr;
  }
  r.first_bad_record = fb < nrec ? (int32_t)(fb < 0x7fffffffull ? fb : 0x7fffffffull) : -1;
  r.n_blocks = nblocks;
  r.retry_frag_capacity = nfr > frag_cap ? nfr : 0;
  r.generation = gen;
  *res = r;
  // for the next decode (both paths rely on these; the scratch setup sets them first)
  misc[M_DONE_CRC] = 0;
  misc[M_BAD_CRC] = ~0ull;
  misc[M_FIRST_BAD] = ~0ull;
  misc[M_BAD_TYPE] = ~0ull;
  misc[M_ABORT] = 0;
}

// ABL: ablation bits for tools/kbench only (0 in the product): 1 no CRC chain, 2 no window loads,
// 4 no lane-operator / scan combine, 8 no record-state tail, 16 phase stamps, 128 no first-window mask, 256 no last-window fix,
// 512 per-wave wall-clock stamps (entry, tables loaded, loop done) into the expire column as u64[4] per wave, 1024 no
// priority balancing, 32768 no CRC passes (the emission alone)
template <int ABL = 0>
__global__ __launch_bounds__(kCrcThreads) void k_crc(const uint8_t* __restrict__ seg, uint64_t seg_len,
                                                     uint32_t start_off, uint64_t nblocks,
                                                     const uint32_t* __restrict__ fbase, Frag* __restrict__ frags,
                                                     uint64_t frag_cap, Tables tabs, EmitArgs ea,
                                                     uint32_t tail_panic, uint64_t gen,
                                                     bcw_decode_result* __restrict__ res,
                                                     uint64_t* __restrict__ misc, uint64_t cb0, uint64_t cb1,
                                                     uint32_t nwg_total) {
  // [cb0, cb1): the chunk of the segment's blocks this launch verifies and emits (the whole segment, or one of the
  // chunks launched as their chase ends); nwg_total: the workgroups of every chunk's launch, the last of which
  // writes the segment result
  __shared__ __attribute__((aligned(16))) uint32_t lds[kCrcLds / 4];
  const uint64_t t_entry = (ABL & 512) ? wall_clock64() : 0;
  uint32_t* s_slice = lds;
  uint32_t* s_fwd = lds + kLdsSlice;
  uint32_t* s_carry = s_fwd + kLdsFwd;
  uint32_t* s_half = s_carry + 128;
  uint32_t* s_wave_all = s_carry + kLdsOps;
  const uint32_t tid = threadIdx.x;
  __shared__ uint32_t s_wdone;      // waves of this workgroup done
  __shared__ uint32_t s_eq;         // the workgroup's emission items taken
  __shared__ uint32_t s_rem[kCrcWaves];  // windows each wave has left (balance)
  if (tid == 0) { s_wdone = 0; s_eq = 0; }
  const uint32_t lane = tid & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // ABL & 65536: the workgroup's last wave is a dedicated record emitter (no CRC passes) from the kernel's start
  constexpr bool kEm = (ABL & 65536) != 0;
  constexpr uint32_t kNCrc = kEm ? kCrcWaves - 1 : kCrcWaves;  // CRC waves per workgroup
  const bool emitter = kEm && wave == kCrcWaves - 1;
  const uint64_t nw = (uint64_t)gridDim.x * kNCrc;
  const uint64_t gw = (uint64_t)blockIdx.x * kNCrc + (emitter ? kNCrc - 1 : wave);
  const uint64_t cn = cb1 - cb0;
  const uint64_t b0 = cb0 + (emitter ? cn * (gw + 1) / nw : cn * gw / nw), b1 = cb0 + cn * (gw + 1) / nw;
  // the wave's fragment range and its first descriptors are loaded while the table image crosses into LDS
  // (that chain of dependent loads no longer follows the image copy)
  const uint64_t f0 = fbase[b0];
  uint64_t f1 = fbase[b1];
  // the emission work items (blocks per item for ~64 fragments each of the chunk; see emit_item)
  const uint64_t fc0 = fbase[cb0], fc1 = fbase[cb1];
  const uint64_t nf_all = fc1 > fc0 ? (fc1 - fc0 < frag_cap ? fc1 - fc0 : frag_cap) : 0;
  uint64_t bpw = nf_all ? (64 * cn) / nf_all : cn;
  if (bpw < 1) bpw = 1;
  uint4 pf = make_uint4(0, 0, 0, 0);  // the next group's 64 fragment descriptors (raw; see load_win)
  {  // table image -> LDS: all 16 B loads in flight before the first store
    constexpr uint32_t kVec = kLdsImage / 4;
    constexpr int kFull = (int)(kVec / kCrcThreads);
    const uint4* src = reinterpret_cast<const uint4*>(tabs.lds_image);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    uint4 v[kFull];
#pragma unroll
    for (int k2 = 0; k2 < kFull; ++k2) v[k2] = src[tid + k2 * kCrcThreads];
    const uint32_t tail = tid + kFull * kCrcThreads;
    uint4 vt = make_uint4(0, 0, 0, 0);
    if (tail < kVec) vt = src[tail];
    if (f1 > frag_cap) f1 = frag_cap;
    if (f0 + lane < f1) pf = reinterpret_cast<const uint4*>(frags)[f0 + lane];
    if (tail < kVec) dst[tail] = vt;
#pragma unroll
    for (int k2 = 0; k2 < kFull; ++k2) dst[tid + k2 * kCrcThreads] = v[k2];
  }
  __syncthreads();

  if (blockIdx.x == 0 && tid == 0) misc[M_T_CRC0] = wall_clock64();
  const uint64_t t_tables = (ABL & 512) ? wall_clock64() : 0;
  const SliceLane sl = slice_lane(lane);  // slice-table lookup constants
  uint32_t* r_cpre = s_wave_all + wave * kWaveLds;  // ring of fragments: first window (wave-relative)
  uint32_t* r_cend = r_cpre + kRing;                 //   end of its windows
  uint4* r_ent = reinterpret_cast<uint4*>(r_cend + kRing);  // {window end (GE) - wbase, C | last window's hi << 16
                                                             //  | first window's lo << 24, J, fragment index}
  const int64_t wbase = (int64_t)start_off + (int64_t)b0 * kBlock - 128;  // below every window of the wave
  const uint32_t nfr = f1 > f0 ? (uint32_t)(f1 - f0) : 0u;
  const uint32_t nwin = (nfr + 63u) / 64u;

  uint32_t r_head = 0, r_tail = 0;  // absolute ring positions (wave-uniform)
  uint32_t cbase = 0;               // windows appended so far
  uint32_t kwin = 0;                // next group of 64 fragments to append
  // pf: the next group's fragment descriptor, loaded one group ahead as a raw 16 B vector (decoded only when the
  // group is appended, so the load does not make the compiler wait for it -- and the window loads -- early)

  // Group kwin (64 fragments, one per lane): every fragment is appended to the ring with its C windows
  // (GE tiling, see above); the group after it is prefetched. No window is loaded here: the first window
  // of a fragment is an ordinary pass window with the bytes before the data masked off.
  auto load_win = [&]() {
    const uint32_t fi = kwin * 64u + lane;
    ++kwin;
    const bool valid = fi < nfr;
    Frag f;
    __builtin_memcpy(&f, &pf, sizeof f);
    // unconditional (a clamped index; lanes past the end reload the last descriptor): a branch would merge
    // the old and new values right after the load, waiting for it
    pf = reinterpret_cast<const uint4*>(frags)[f0 + (fi + 64u < nfr ? fi + 64u : nfr - 1u)];
    FragGeo geo{0, 0, 0};
    uint32_t e = 0;
    if (valid) {
      e = (uint32_t)f.start + f.len;
      geo = frag_geo(start_off, f.blk, f.start, e);
    }
    const uint32_t cb = geo.C;
    const uint64_t vm = __ballot(valid);
    const uint32_t below = lane == 0 ? 0u : (uint32_t)__builtin_popcountll(vm & (~0ull >> (64 - lane)));
    const uint32_t incl = wave_add_scan(cb, lane);
    const uint32_t tot = __shfl(incl, 63, 64);
    if (valid) {
      const uint32_t a = (r_tail + below) & (kRing - 1);
      const int64_t ge = geo.gs + (int64_t)(e - f.start);
      const uint32_t lo = (uint32_t)(geo.gs - (geo.GE - 128 * (int64_t)geo.C));  // bytes before the data
      r_cpre[a] = cbase + incl - cb;
      r_cend[a] = cbase + incl;
      r_ent[a] = make_uint4((uint32_t)(geo.GE - wbase), geo.C | ((uint32_t)(ge - (geo.GE - 128)) << 16) | (lo << 24),
                            f.chk, fi);
    }
    r_tail += (uint32_t)__builtin_popcountll(vm);
    cbase += __builtin_amdgcn_readfirstlane(tot);
    wave_sync();
  };

  // make the ring hold every fragment owning a chunk of [pass, pass+64): drop entries ending at or
  // before `pass` (chunk ends increase along the ring, so the dead entries are a ballot prefix)
  auto advance = [&](uint32_t pass) {
    auto evict = [&]() {
      for (;;) {
        const uint32_t a = r_head + lane;
        const bool dead = a < r_tail && r_cend[a & (kRing - 1)] <= pass;
        const uint32_t n = (uint32_t)__builtin_popcountll(__ballot(dead));
        r_head += n;
        if (n < 64u) break;
      }
    };
    evict();
    while (kwin < nwin && cbase < pass + 64u) {
      load_win();
      evict();
    }
  };

  // lane l's chunk pass + l belongs to the last ring entry whose first chunk is <= pass + l: entries
  // starting inside the pass set bits of a 64-bit mask (OR over the wave), a popcount of the mask up
  // to the lane counts them, and the ring head continues any fragment carried into the pass
  auto describe = [&](uint32_t pass) -> BodyDesc {
    BodyDesc d{};
    const uint32_t j = pass + lane;
    const uint32_t a0 = r_head + lane, a1 = a0 + 64u;
    const uint32_t c0 = a0 < r_tail ? r_cpre[a0 & (kRing - 1)] : 0xffffffffu;
    const uint32_t c1 = a1 < r_tail ? r_cpre[a1 & (kRing - 1)] : 0xffffffffu;
    uint64_t bits = 0;
    if (c0 >= pass && c0 - pass < 64u) bits |= 1ull << (c0 - pass);
    if (c1 >= pass && c1 - pass < 64u) bits |= 1ull << (c1 - pass);
    const uint32_t mlo = __builtin_amdgcn_readlane(wave_or_scan(( uint32_t)bits, lane), 63);
    const uint32_t mhi = __builtin_amdgcn_readlane(wave_or_scan((uint32_t)(bits >> 32), lane), 63);
    const uint64_t M = (uint64_t)mlo | ((uint64_t)mhi << 32);
    const uint32_t carried = (r_head < r_tail && (uint32_t)__builtin_amdgcn_readfirstlane(c0) < pass) ? 1u : 0u;
    const uint64_t upto = lane == 63u ? ~0ull : ((2ull << lane) - 1ull);
    const uint32_t cnt = carried + (uint32_t)__builtin_popcountll(M & upto);
    const uint32_t a = r_head + cnt - 1u;
    if (!(cnt > 0u && j < cbase && a < r_tail)) return d;  // inactive (meta = 0)
    const uint32_t slot = a & (kRing - 1);
    const uint4 e0 = r_ent[slot];
    const uint32_t chl = e0.y;
    const uint32_t cfb = j - r_cpre[slot];
    const uint32_t c = (chl & 0xffffu) - 1u - cfb;  // windows from the end (0 = last)
    d.woff = e0.x - 128u * (c + 1u);
    d.meta = (c == 0u ? ((chl >> 16) & 0xffu) : 0u) | (cfb << 8) | ((c == 0u ? 1u : 0u) << 17) | (1u << 18) |
             ((cfb == 0u ? (chl >> 24) : 0u) << 19);
    d.J = c == 0u ? e0.z : 0u;  // J = ~unmask(stored) ^ A_{8L}(~0) (see above), from the fragment table
    d.fi = e0.w;
    return d;
  };

  // gsafe: an in-bounds window (the wave's first block, clamped to the segment); safe_win: 128 B every lane may
  // load without a bounds check -- that window, or the table image for segments shorter than 128 B
  const int64_t gblk = wbase + 128 > 0 ? wbase + 128 : 0;  // the wave's first block
  const int64_t gsafe = seg_len < 128 ? -1 : (gblk < (int64_t)seg_len - 128 ? gblk : (int64_t)seg_len - 128);
  const uint8_t* safe_win = seg_len >= 128 ? seg + gsafe : reinterpret_cast<const uint8_t*>(tabs.lds_image);

  uint32_t carry = 0;  // fragment state at the end of the previous pass (lane 63)
  // chain pass d in w, and load pass dn into w as the chains free its registers (the next pass's loads overlap
  // the chain's second half and everything up to the next pass's chain, with no second window buffer); a pass
  // whose windows touch the segment's ends takes bounds-checked loads after the chain instead
  auto window_goff = [&](const BodyDesc& d) -> int64_t { return d.active() ? wbase + d.woff : gsafe; };
  auto inbounds = [&](int64_t goff) { return __all(goff >= 0 && (uint64_t)goff + 128 <= seg_len); };
  auto compute = [&](const BodyDesc& d, uint32_t (&w)[32], const BodyDesc& dn) {
    // this pass's loads (issued at the end of the previous compute) have landed
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
    // the prefetched fragment descriptor has landed too: make it a plain value here, so that decoding it later
    // (load_win) waits for nothing -- a wait there would be vmcnt(0) and also wait for the window loads in flight
    asm volatile("" : "+v"(pf.x), "+v"(pf.y), "+v"(pf.z), "+v"(pf.w));
    {  // a pass touching the segment's ends was loaded from safe_win: bounds-checked loads now
      const int64_t goff = window_goff(d);
      if (!(ABL & 2) && !inbounds(goff) && d.active()) load_window(seg, seg_len, goff, false, w);
    }
    const int64_t ngoff = window_goff(dn);
    const bool nfast = inbounds(ngoff);
    // unconditional loads (a pass touching the segment's ends reads safe_win here and is
    // reloaded at the top of its compute): a branch around them makes the compiler copy each landed tuple into the
    // loop's registers right away, waiting for it
    const uint4* nq = reinterpret_cast<const uint4*>(nfast ? seg + ngoff : safe_win);
    uint32_t v = 0;
    if (d.active()) {
      if (!(ABL & 128) && d.cfb() == 0u) mask_first(w, d.lo());  // zero the bytes before the data
      if (!(ABL & 256) && d.last()) fix_last(w, d.hi(), d.J);
    }
    // a fragment continuing from the previous pass: its state so far seeds lane 0's chain
    const uint32_t seed = (d.active() && lane == 0u && d.cfb() > 0u) ? carry : 0u;
    if (!(ABL & 1)) {
      v = crc_window(s_slice, s_half, sl, seed, w);
    } else {
      v = seed ^ w[0] ^ w[31];
    }
    if (!d.active()) v = 0u;
    // U-domain: lane l holds A_{1024(63-l)} of its window state
    if (!(ABL & 4)) v = apply_fwd(s_fwd, lane, v);
    uint32_t U = v;
    if (!(ABL & 4)) {
      // segment sum = prefix XOR at this lane ^ prefix XOR just before the segment's first lane (one
      // zero-filled DPP scan and one ds_bpermute instead of a segmented scan's per-step lane conditions)
      const uint32_t segl = d.active() ? (d.cfb() > lane ? 0u : lane - d.cfb()) : lane;
      const uint32_t P = wave_scan_z(v, [](uint32_t x, uint32_t y) { return x ^ y; });
      const uint32_t Pb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((segl > 0u ? segl - 1u : 0u) << 2), (int)P);
      U = segl > 0u ? P ^ Pb : P;
    }
    // pass dn's loads: issued here, once the window is dead, so they stay in flight through the ring upkeep
    // and the descriptor build of the pass after. Issued progressively inside the chains instead (into the
    // registers each step frees) k_crc took 275 vs 235 us (kbench, one process): a load instruction that
    // finds the texture addresser's queue full stalls the issuing wave, and inside the chain that stall
    // lands on its latency-bound critical path.
    if (!(ABL & 2)) {
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        const uint4 q = nq[g];
        w[4 * g + 0] = q.x; w[4 * g + 1] = q.y; w[4 * g + 2] = q.z; w[4 * g + 3] = q.w;
      }
    }
    if (d.active() && d.last()) {
      frags[f0 + d.fi].ok = (U == 0u) ? 1 : 0;
      if (U != 0u && !(ABL & 7)) atomicMin(reinterpret_cast<unsigned long long*>(&misc[M_BAD_CRC]), (unsigned long long)(f0 + d.fi));
    }
    carry = __builtin_amdgcn_readlane(U, 63);
  };

  // software pipeline: a pass's windows are in flight while the ring upkeep and descriptor build run
  // (ABL & 16: per-phase cycle stamps for tools/kbench, summed into misc[7..9]: describe = ring upkeep +
  // descriptor + load issue, issue = unused, compute = the chain, including any wait for its loads)
  uint64_t t_desc = 0, t_issue = 0, t_comp = 0, tq = 0;
  auto stamp = [&](uint64_t& acc) {
    if (ABL & 16) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      acc += t - tq;
      tq = t;
    }
  };
  if (ABL & 16) tq = __builtin_amdgcn_s_memtime();
  // Balance within the workgroup: the SIMD arbiter favours older waves, so with equal shares the workgroup's
  // last four waves would finish ~15 % after its first four. Each wave publishes its remaining windows (an
  // estimate: 256 per block + one per fragment, less the windows done) and takes issue priority while it has
  // (nearly) the most left.
  const uint32_t est = (uint32_t)(b1 - b0) * 256u + nfr;
  if (lane == 0) s_rem[wave] = est;
  auto balance = [&](uint32_t done) {
    if (ABL & 1024) return;
    const uint32_t rem = est > done ? est - done : 0u;
    if (lane == 0) s_rem[wave] = rem;
    const uint32_t v = lane < (uint32_t)kCrcWaves ? s_rem[lane] : 0u;
    const uint32_t mx = __builtin_amdgcn_readlane(wave_max_scan(v, lane), 63);
    if (rem + 128u >= mx) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(0);
  };
  auto pipeline = [&]() {
    // One window buffer: pass p chains in w, then pass p+64's loads are issued into it and stay in flight while
    // the ring upkeep and the describe of pass p+128 run. One copy of the loop body (instruction-cache
    // footprint).
    uint32_t w[32];
    advance(0u);
    BodyDesc dc = describe(0u);
    if (!(ABL & 2)) {  // the first pass (compute reloads it bounds-checked when it touches the segment's ends)
      const int64_t goff = window_goff(dc);
      const uint4* q = reinterpret_cast<const uint4*>(inbounds(goff) ? seg + goff : safe_win);
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        const uint4 v = q[g];
        w[4 * g + 0] = v.x; w[4 * g + 1] = v.y; w[4 * g + 2] = v.z; w[4 * g + 3] = v.w;
      }
    }
    advance(64u);
    BodyDesc dn = describe(64u);
    for (uint32_t p = 0;;) {
      stamp(t_desc);
      compute(dc, w, dn);
      balance(p + 64u);
      stamp(t_comp);
      p += 64u;
      if (p >= cbase) break;
      dc = dn;
      advance(p + 64u);
      dn = describe(p + 64u);
    }
  };
  if (nfr > 0u && !(ABL & 32768)) pipeline();
  stamp(t_comp);
  if ((ABL & 16) && lane == 0) {
    atomicAdd(reinterpret_cast<unsigned long long*>(&misc[7]), (unsigned long long)t_desc);
    atomicAdd(reinterpret_cast<unsigned long long*>(&misc[8]), (unsigned long long)t_issue);
    atomicAdd(reinterpret_cast<unsigned long long*>(&misc[9]), (unsigned long long)t_comp);
  }

  __builtin_amdgcn_s_setprio(0);
  if ((ABL & 512) && lane == 0) {
    uint64_t* q = ea.tab.expire + 4 * gw;  // kbench only (the table is overwritten by the emission unless ABL & 8)
    q[0] = t_entry; q[1] = t_tables; q[2] = wall_clock64(); q[3] = nfr;
  }
  // ---- record emission: the workgroup's work items (those starting in its blocks), taken from an LDS counter by
  // its waves as they finish their CRC passes, so the early finishers emit for the late ones (ItemMeta). The next
  // item is taken and its block data requested while this item's fragment descriptors are in flight, so an item
  // costs two dependent round trips (descriptors, record prefixes) ----
  if (!(ABL & 8) && !(ea.kb_flags & 1u)) {
    const uint64_t B0 = cn * ((uint64_t)blockIdx.x * kNCrc) / nw;  // chunk-relative
    const uint64_t B1 = cn * ((uint64_t)(blockIdx.x + 1) * kNCrc) / nw;
    const uint64_t i0 = (B0 + bpw - 1) / bpw, nitems = (!kEm || emitter) ? (B1 + bpw - 1) / bpw : 0;
    uint32_t taken = 0;  // the dedicated emitter takes every item in order
    auto deq = [&]() -> uint64_t {
      uint32_t j = 0;
      if (kEm) {
        j = taken++;
      } else {
        if (lane == 0) j = atomicAdd(&s_eq, 1u);
        j = __builtin_amdgcn_readfirstlane(j);
      }
      return i0 + j;
    };
    const uint64_t t_crc = ea.kb_stamps ? wall_clock64() : 0;
    uint64_t n_items = 0;
    uint64_t it = deq();
    ItemMeta m = item_meta(ea, it, bpw, cb0, cb1, lane);
    PredSync ps;  // k_chase's tables: nothing to acquire
    while (it < nitems) {
      ++n_items;
      const EmitState es = emit_state(ea, m.bb, lane, m.s, m.rec, ps);
      const uint64_t f1 = m.f1 < frag_cap ? m.f1 : frag_cap;
      uint64_t nx = 0;
      ItemMeta mn;
      emit_chunks<ABL & (4096 | 8192)>(ea, es, m.f0, f1, lane, [&]() {
        nx = deq();
        mn = item_meta(ea, nx, bpw, cb0, cb1, lane);
      });
      it = nx;
      m = mn;
    }
    if (ea.kb_stamps && lane == 0) {
      uint64_t* q = ea.kb_stamps + 4 * ((uint64_t)blockIdx.x * kCrcWaves + wave);
      q[0] = t_crc; q[1] = wall_clock64(); q[2] = n_items; q[3] = nfr;
    }
  }
  // ---- completion: each wave's stores and atomics are done (vmcnt(0)) before it counts itself done in LDS;
  // the last wave of a workgroup adds the workgroup to the agent-scope counter, and the last workgroup's
  // last wave writes the segment result from the agent-scope minima (MI355X_MICROARCH.md, inter-workgroup
  // visibility, row 1) ----
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  uint32_t order = 0;
  if (lane == 0) order = atomicAdd(&s_wdone, 1u);
  order = __builtin_amdgcn_readlane(order, 0);
  if (order != kCrcWaves - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  uint64_t gorder = 0;
  if (lane == 0)
    gorder = __hip_atomic_fetch_add(&misc[M_DONE_CRC], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  gorder = (uint64_t)__shfl((long long)gorder, 0, 64);
  if (gorder != nwg_total - 1u) return;
  if (lane == 0) misc[M_T_FIN] = wall_clock64();
  finalize(ea, nblocks, frag_cap, tail_panic, gen, res, lane);
}

// ------------------------------------------------------------------------------------------
// k_scan: the whole decode of a segment in ONE launch, so the header chase no longer runs as a
// launch of its own in front of the CRC stream. One 1024-thread workgroup per CU; workgroups take tickets and own
// consecutive block ranges [B0, B1) in ticket order (so a workgroup only ever waits on running ones).
//
// The CRC work is made independent of the fragment geometry. Windows are the absolute 128 B windows of the segment
// (m: bytes [128m, 128m + 128)); workgroup w owns the windows m0 <= m < m1 whose first byte lies in its blocks. A
// unit is 64 consecutive windows of the workgroup from m0 + 64u; lane l computes v = R(window) (raw CRC-32C, init
// 0), maps it to the unit's end with F_l = A_{1024(63-l)} and the wave stores the prefix XOR
//     P[m] = XOR_{i <= l} F_i(v_{m0 + 64u + i})           (the unit-end frame; pwin, 4 B per window).
// A fragment with data [GS, GE) and check word J passes iff R(data || J) = 0 (J = the raw CRC its stored CRC
// implies, see k_crc); with a = GS >> 7, j0 = GE >> 7 and j1 = (GE + 3) >> 7 that is
//     T = XOR_{m = a..j1} A_{1024(F - m)}(z_m) = 0       (any frame F >= j1: the shift is invertible)
// where z_m = R(window m with the bytes outside [GS, GE) zeroed and J written at [GE, GE + 4)). Every window
// strictly between a and j0 lies inside the data (z_m = v_m) and inside the workgroup's own windows, so per unit
// its sum is P[hi] ^ P[lo - 1]; the edge windows a, j0, j1 are recomputed masked (at most three per fragment).
// Horner over the units a..j1 spans (A_{8*8192} between units) gives T in the frame of j1's unit end.
//
// Phases of a workgroup:
//   chase   waves 0..nch-1 (nch = ceil((B1 - B0) / 64)) chase one block per lane (chase_block, the first headers
//           held in LDS), the last of them publishes the workgroup's fragment / Full-Last counts and sums its
//           predecessors' (direct: at most one word per CU), then every chaser writes its blocks' fragment table
//           entries, fbase, rbase and summaries, and the last one publishes "written" behind an agent release.
//   windows the other waves start at once (the chasers once done): units from an LDS counter, software-pipelined
//           like k_crc (the next unit's loads issued right after the chain).
//   verify  after a workgroup barrier: items of 64 of the workgroup's fragments, one lane per fragment.
//   emit    k_crc's emission items over the workgroup's blocks; a walk-back that crosses B0 acquires the
//           predecessors' writes first (PredSync).
constexpr int kScanHoldWords = kCrcWaves * kWaveLds;  // the chasers' held headers (48 KiB, k_crc's ring space)

// Quad-coalesced unit loads: load g (g = 4 p2 + 2 w1 + w0) gives the 4 lanes of quad a the 16 B pieces 4 p2 .. 4 p2 + 3
// of window 4a + (g & 3) -- 64 contiguous bytes per quad, 1 KiB per instruction in 16 runs, instead of one 16 B piece
// of 64 different lines (the texture addresser's tag lookups per instruction drop 4x). Two lane-bit <-> register-bit
// exchanges (DPP quad_perm) then leave piece p of window W in w[4p..4p+3] of lane W (kbench: loads + chain of a
// 1 GiB segment at 12 waves 186 us, lane-per-window 210 us). k_scan's units are contiguous 8 KiB, so they can.
__device__ __forceinline__ void load_unit_quad(const uint8_t* __restrict__ base, uint32_t lane, uint32_t (&w)[32]) {
  const uint32_t qb = 16u * (lane & 3u) + 512u * (lane >> 2);  // quad a's 512 B, this lane's 16 B column
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const uint4 v = *reinterpret_cast<const uint4*>(base + qb + 128u * (g & 3) + 64u * (g >> 2));
    w[4 * g + 0] = v.x; w[4 * g + 1] = v.y; w[4 * g + 2] = v.z; w[4 * g + 3] = v.w;
  }
}
template <int K>
__device__ __forceinline__ void swap_lane_reg_bit(uint32_t (&w)[32], uint32_t lane) {
  constexpr int CTRL = K == 0 ? 0xB1 : 0x4E;  // quad_perm partner lane ^ 1 / lane ^ 2
  const bool hi = (lane >> K) & 1u;
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    if (x & (1 << K)) continue;
    const int y = x | (1 << K);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t rx = w[4 * x + d], ry = w[4 * y + d];
      const uint32_t px = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)rx, CTRL, 0xf, 0xf, true);
      const uint32_t py = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ry, CTRL, 0xf, 0xf, true);
      w[4 * x + d] = hi ? py : rx;
      w[4 * y + d] = hi ? ry : px;
    }
  }
}
// after load_unit_quad: register group g = 4 p2 + 2 w1 + w0 of lane 4a + l holds piece 4 p2 + l of window 4a + 2 w1 + w0;
// exchanging lane bit 0 with register bit 0 and lane bit 1 with register bit 1 leaves piece 4 p2 + 2 w1' + w0' of
// window 4a + l in group g of lane 4a + l, i.e. the lane's own window in order
__device__ __forceinline__ void unit_quad_transpose(uint32_t (&w)[32], uint32_t lane) {
  swap_lane_reg_bit<0>(w, lane);
  swap_lane_reg_bit<1>(w, lane);
}

// window bytes of a fragment for its zero test: data outside [gs, ge) zeroed, J at [ge, ge + 4) (window-relative,
// any values). Per word: a kept-byte mask and the J bytes that land in it.
__device__ __forceinline__ void mask_frag_window(uint32_t (&w)[32], int gs, int ge, uint32_t J) {
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int q = 4 * i;
    const int lo = min(max(gs - q, 0), 4), hi = min(max(ge - q, 0), 4);  // kept bytes [lo, hi) of the word
    const uint32_t keep = (uint32_t)((1ull << (8 * hi)) - 1ull) & ~(uint32_t)((1ull << (8 * lo)) - 1ull);
    const int s = ge - q;  // position of J's first byte in the word
    const uint32_t jw = (s > -4 && s < 4) ? (uint32_t)(((uint64_t)J << (8 * (s + 4))) >> 32) : 0u;
    w[i] = (w[i] & keep) | jw;
  }
}

// z_m of a fragment (absolute data [GS, GE), check word J): R of its masked / J-patched window m
__device__ __forceinline__ uint32_t edge_window(const uint8_t* __restrict__ seg, uint64_t seg_len, int64_t m,
                                                int64_t GS, int64_t GE, uint32_t J, const uint32_t* __restrict__ tab,
                                                const uint32_t* __restrict__ half, const SliceLane& sl) {
  const int64_t o = m * (int64_t)kWin;
  uint32_t w[32];
  if (o < GE && o + (int64_t)kWin > GS) {  // the window holds data bytes
    load_window(seg, seg_len, o, (uint64_t)o + kWin <= seg_len, w);
  } else {
#pragma unroll
    for (int i = 0; i < 32; ++i) w[i] = 0u;
  }
  mask_frag_window(w, (int)(GS - o), (int)(GE - o), J);
  return crc_window(tab, half, sl, 0u, w);
}

// ABL: ablation bits for tools/kbench only (0 in the product): 1 no CRC chain in the window units, 2 no verify,
// 4 no window units, 8 no emission, 32 static unit ranges per wave, 512 per-wave wall-clock stamps into ea.kb_stamps
// (8 x u64 per wave: entry, tables in LDS, chase written (chasers), units done, chase seen, verify done, all done)
template <int ABL = 0>
__global__ __launch_bounds__(kScanThreads) void k_scan(const uint8_t* __restrict__ seg, uint64_t seg_len,
                                                      uint32_t start_off, uint64_t nblocks, uint32_t* __restrict__ fbase,
                                                      uint32_t* __restrict__ rbase, uint2* __restrict__ bsum,
                                                      Frag* __restrict__ frags, uint64_t frag_cap,
                                                      uint32_t* __restrict__ pwin, uint32_t ustride,
                                                      uint64_t* __restrict__ lb, uint64_t* __restrict__ lbe,
                                                      uint64_t* __restrict__ lbw, uint64_t ticket_base, uint64_t epoch,
                                                      Tables tabs, EmitArgs ea, uint32_t tail_panic, uint64_t gen,
                                                      bcw_decode_result* __restrict__ res) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsImage + kScanHoldWords];
  __shared__ uint64_t s_base[4];       // workgroup's first fragment, first record row, fragments, Full/Last fragments
  __shared__ uint32_t s_ctot[kScanWaves], s_etot[kScanWaves];  // per chaser wave: fragments, Full/Last fragments
  __shared__ uint32_t s_chn, s_chw, s_ready, s_unit, s_vq, s_eq, s_wdone;
  __shared__ uint64_t s_wg;
  __shared__ uint32_t s_udone[(kScanMaxBlocks * (kBlock / 8192) + 2 + 31) / 32];  // window units done (bit per unit)
  __shared__ uint64_t s_em[4];  // emission items: B0, B1, blocks per item, the workgroup's fragment end
  constexpr uint32_t kVItems = 256;  // verify items whose unit range the chasers record (later ones: from descriptors)
  __shared__ uint32_t s_vlo[kVItems], s_vhi[kVItems];  // first / last window unit a verify item's interiors need
  // prefix rows on their way to HBM: the streaming waves put a unit's 64 prefixes here and the writer wave stores them
  // (vmcnt retires in order per wave, so a streaming wave's own store would hold up the waits for its later loads
  // until the store is acknowledged -- slow under a read-saturated load: 35-50 us of a config-B decode, kbench)
  constexpr uint32_t kRing = 32;
  __shared__ __attribute__((aligned(16))) uint32_t s_ring[kRing * 64];
  __shared__ uint32_t s_rstate[kRing];  // 0: free, else the unit + 1 whose row the slot holds
  constexpr uint32_t kWDepth = 16;  // each writer's stores in flight (vmcnt(8) below; 56 in flight: 309 vs 303 us, B)
  __shared__ uint32_t s_rhead, s_wunit[kScanWriters][kWDepth];
  uint32_t* s_slice = lds;
  uint32_t* s_fwd = lds + kLdsSlice;
  uint32_t* s_carry = s_fwd + kLdsFwd;  // A_{8*8192}: one unit
  uint32_t* s_half = s_carry + 128;
  uint32_t* s_hold = lds + kLdsImage;
  uint64_t* misc = ea.misc;
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  auto stamp = [&](int k) {
    if ((ABL & 512) && lane == 0) ea.kb_stamps[((uint64_t)blockIdx.x * kScanWaves + wave) * 8 + k] = wall_clock64();
  };
  stamp(0);
  if (tid == 0) {
    s_wg = atomicAdd(reinterpret_cast<unsigned long long*>(&misc[M_TICKET]), 1ull) - ticket_base;
    s_chn = s_chw = s_ready = s_unit = s_vq = s_eq = s_wdone = 0;
  }
  for (uint32_t i = tid; i < sizeof(s_udone) / 4; i += kScanThreads) s_udone[i] = 0u;
  for (uint32_t i = tid; i < kVItems; i += kScanThreads) { s_vlo[i] = 0xffffffffu; s_vhi[i] = 0u; }
  for (uint32_t i = tid; i < kRing; i += kScanThreads) s_rstate[i] = 0u;
  if (tid == 0) s_rhead = 0u;
  {  // table image -> LDS: all 16 B loads in flight before the first store
    constexpr uint32_t kVec = kLdsImage / 4;
    constexpr int kFull = (int)(kVec / kScanThreads);
    const uint4* src = reinterpret_cast<const uint4*>(tabs.lds_image);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    uint4 v[kFull];
#pragma unroll
    for (int k2 = 0; k2 < kFull; ++k2) v[k2] = src[tid + k2 * kScanThreads];
    const uint32_t tail = tid + kFull * kScanThreads;
    uint4 vt = make_uint4(0, 0, 0, 0);
    if (tail < kVec) vt = src[tail];
    if (tail < kVec) dst[tail] = vt;
#pragma unroll
    for (int k2 = 0; k2 < kFull; ++k2) dst[tid + k2 * kScanThreads] = v[k2];
  }
  __syncthreads();
  stamp(1);
  stamp(2);
  const uint64_t G = gridDim.x;
  const uint64_t wg = s_wg;
  const uint64_t B0 = nblocks * wg / G, B1 = nblocks * (wg + 1) / G;
  const uint32_t nch = (uint32_t)((B1 - B0 + 63) / 64) > 0u ? (uint32_t)((B1 - B0 + 63) / 64) : 1u;
  const uint64_t tag = epoch << 40;
  // the workgroup's windows [m0, m1): those whose first byte lies in its blocks and in the segment (a window past the
  // segment's end is never interior to a fragment). Only the last unit can then be partial or touch the segment's
  // end -- at most one slow ("deferred") unit per workgroup, which the unit loop relies on.
  const uint64_t mseg = (seg_len + kWin - 1) / kWin;
  const uint64_t m0 = ((uint64_t)start_off + B0 * kBlock + kWin - 1) / kWin;
  uint64_t m1 = ((uint64_t)start_off + B1 * kBlock + kWin - 1) / kWin;
  if (m1 > mseg) m1 = mseg;
  if (m1 < m0) m1 = m0;
  const uint32_t nunits = (uint32_t)((m1 - m0 + 63) / 64);
  // the workgroup's prefix rows: unit u's 64 prefixes are one aligned 256 B row at pw + 64 u (rows indexed from the
  // workgroup's first window, not by absolute window: a row straddling 128 B lines made every store a partial-line
  // write, ~35 us of a config-B decode)
  uint32_t* const pw = pwin + (uint64_t)wg * ustride * 64u;
  const SliceLane sl = slice_lane(lane);

  // ---- chase (waves 0..nch-1): k_chase's per-block walk, one block per lane ----
  if (wave < nch) {
    const uint32_t NL = nch * 64u, L = wave * 64u + lane;
    const uint32_t H = (uint32_t)kScanHoldWords / (3u * NL);  // held headers per lane
    const uint64_t b = B0 + L;
    uint32_t bufsize = 0;
    uint64_t boff = 0;
    if (b < B1) {
      boff = (uint64_t)start_off + b * kBlock;
      bufsize = (uint32_t)((seg_len - boff) < kBlock ? (seg_len - boff) : kBlock);
    }
    uint32_t ne = 0, tacc = 0, tnz = 0xffffu, tst = 0, badk = 0xffffffffu;
    uint32_t hres = 0;  // where the first header past the held ones starts (the table pass resumes there)
    const uint32_t n = chase_block(seg, seg_len, boff, (ABL & 4096) ? 0u : bufsize,
                                   [&](uint32_t k, uint32_t start, uint32_t len, uint32_t crc, uint32_t type) {
                                     if (k < H) {
                                       uint32_t* e = s_hold + (k * NL + L) * 3u;
                                       e[0] = crc;
                                       e[1] = start | (len << 16);
                                       e[2] = type;
                                     }
                                     if (k == H - 1u) hres = start + len;
                                     if (type == BCW_RECORD_FULL || type == BCW_RECORD_LAST) {
                                       ++ne;
                                       tacc = 0;
                                       tnz = 0xffffu;
                                     } else {
                                       if (len > 0 && tnz == 0xffffu) { tnz = k; tst = start; }
                                       tacc += len;
                                       if ((type < BCW_RECORD_FULL || type > BCW_RECORD_LAST) && badk == 0xffffffffu)
                                         badk = k;
                                     }
                                   });
    const uint32_t incl = wave_add_scan(n, lane);
    const uint32_t incl_e = wave_add_scan(ne, lane);
    if (lane == 63) { s_ctot[wave] = incl; s_etot[wave] = incl_e; }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    uint32_t ord = 0;
    if (lane == 0) ord = atomicAdd(&s_chn, 1u);
    ord = __builtin_amdgcn_readfirstlane(ord);
    if (ord == nch - 1u) {  // the last chaser wave: publish the workgroup's counts, sum the predecessors'
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      uint64_t wt = 0, wte = 0;
      for (uint32_t c = 0; c < nch; ++c) { wt += s_ctot[c]; wte += s_etot[c]; }
      if (lane == 0) {
        __hip_atomic_store(&lb[wg], tag | (kLbAgg << 38) | (wt & kLbMask), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&lbe[wg], tag | (kLbAgg << 38) | (wte & kLbMask), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
      uint64_t c = 0, ce = 0;
      for (uint64_t q0 = 0; q0 < wg; q0 += 64) {
        const uint64_t q = q0 + lane;
        if (q < wg) {
          uint64_t v, ve;
          Spin sp;
          while (((v = __hip_atomic_load(&lb[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 40) != epoch)
            if (!sp.go(misc, 1)) break;
          while (((ve = __hip_atomic_load(&lbe[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 40) != epoch)
            if (!sp.go(misc, 2)) break;
          c += v & kLbMask;
          ce += ve & kLbMask;
        }
      }
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {
        c += (uint64_t)__shfl_xor((long long)c, d, 64);
        ce += (uint64_t)__shfl_xor((long long)ce, d, 64);
      }
      if (lane == 0) {
        s_base[0] = c; s_base[1] = ce; s_base[2] = wt; s_base[3] = wte;
        const uint64_t bpw = wt ? (64 * (B1 - B0)) / wt : (B1 - B0);
        s_em[0] = B0; s_em[1] = B1; s_em[2] = bpw < 1 ? 1 : bpw;
        s_em[3] = c + wt < 0xffffffffull ? c + wt : 0xffffffffull;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __hip_atomic_store(&s_ready, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    {
      Spin sp;
      while (__hip_atomic_load(&s_ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
        if (!sp.go(misc, 3)) break;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    uint64_t wpre = 0, wpre_e = 0;
    for (uint32_t c = 0; c < wave; ++c) { wpre += s_ctot[c]; wpre_e += s_etot[c]; }
    const uint64_t g0 = s_base[0] + wpre + incl - n;
    const uint64_t r0 = s_base[1] + wpre_e + incl_e - ne;
    if (b < B1) {
      fbase[b] = (uint32_t)(g0 < 0xffffffffull ? g0 : 0xffffffffull);
      rbase[b] = (uint32_t)(r0 < 0xffffffffull ? r0 : 0xffffffffull);
      bsum[b] = make_uint2(tacc | (tnz << 16), tst | (ne ? kSumHasE : 0u));
      if (badk != 0xffffffffu)  // the first unknown-type fragment of the segment (reset by the previous finalize)
        atomicMin(reinterpret_cast<unsigned long long*>(&misc[M_BAD_TYPE]), (unsigned long long)(g0 + badk));
      // the window units a verify item's interior windows lie in (min over its fragments, max over them), for the
      // verify items taken between units (each item: 64 consecutive fragments of the workgroup)
      const uint64_t Fw = s_base[0];
      auto vrange = [&](uint64_t g, uint32_t start, uint32_t len) {
        const int64_t GS = (int64_t)boff + start, GE = GS + len;
        const int64_t a = GS >> 7, j0 = GE >> 7;
        if (j0 - 1 <= a) return;
        const uint64_t it = (g - Fw) / 64;
        if (it >= kVItems) return;
        atomicMin(&s_vlo[it], (uint32_t)((a + 1 - (int64_t)m0) >> 6));
        atomicMax(&s_vhi[it], (uint32_t)((j0 - 1 - (int64_t)m0) >> 6));
      };
      const uint32_t nh = n < H ? n : H;
      for (uint32_t k = 0; k < nh; ++k) {
        const uint32_t* e = s_hold + (k * NL + L) * 3u;
        put_frag(frags, g0 + k, frag_cap, (uint32_t)b, e[1] & 0xffffu, e[1] >> 16, e[0], e[2], tabs.initc);
        vrange(g0 + k, e[1] & 0xffffu, e[1] >> 16);
      }
      if (n > H)  // the tail of a block with more headers than held, chased again from the first of them
        chase_block(seg, seg_len, boff, bufsize, [&](uint32_t k, uint32_t start, uint32_t len, uint32_t crc, uint32_t type) {
          put_frag(frags, g0 + k, frag_cap, (uint32_t)b, start, len, crc, type, tabs.initc);
          vrange(g0 + k, start, len);
        }, hres, H);
    }
    if (wg == G - 1u && wave == 0u && lane == 0u) {  // the segment totals
      const uint64_t total = s_base[0] + s_base[2], total_e = s_base[1] + s_base[3];
      fbase[nblocks] = (uint32_t)(total < 0xffffffffull ? total : 0xffffffffull);
      rbase[nblocks] = (uint32_t)(total_e < 0xffffffffull ? total_e : 0xffffffffull);
      __hip_atomic_store(&misc[M_NFRAGS], total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&misc[M_NE], total_e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // every chaser wave's stores are done before it counts itself; the last one releases them all (agent) and
    // publishes the workgroup's written word
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    uint32_t ordw = 0;
    if (lane == 0) ordw = atomicAdd(&s_chw, 1u);
    ordw = __builtin_amdgcn_readfirstlane(ordw);
    if (ordw == nch - 1u && lane == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&lbw[wg], tag | 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    stamp(2);
  }

  // the chasers' writes are visible to this workgroup's waves (they wait for it before verify and emission)
  auto wait_chase = [&]() {
    Spin sp;
    while (__hip_atomic_load(&s_chw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < nch)
      if (!sp.go(misc, 4)) break;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };
  const bool chaser = wave < nch;
  const int64_t M0 = (int64_t)m0;
  auto frag_range = [&](uint64_t& fa, uint64_t& fb) {  // the workgroup's fragments (after wait_chase)
    const uint64_t F0 = s_base[0], NF = s_base[2];
    fa = F0 < frag_cap ? F0 : frag_cap;
    fb = F0 + NF < frag_cap ? F0 + NF : frag_cap;
  };
  auto units_done = [&](uint32_t mn, uint32_t mx) -> bool {  // every unit in [mn, mx] stored (wave-uniform)
    if (mn > mx) return true;
    for (uint32_t wd = mn >> 5; wd <= (mx >> 5); ++wd) {
      const uint32_t blo = wd == (mn >> 5) ? (mn & 31u) : 0u, bhi = wd == (mx >> 5) ? (mx & 31u) : 31u;
      const uint32_t need = (uint32_t)((2ull << bhi) - 1ull) & ~((1u << blo) - 1u);
      if ((__hip_atomic_load(&s_udone[wd], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & need) != need)
        return false;
    }
    return true;
  };
  // Steps of a wave. A chaser, its fragment table written: record emission (a latency-bound chain that needs no CRC
  // result), then verify items as the window units they need get stored -- it trails the unit frontier, so little
  // verify work is left when the streaming ends. Every other wave: window units, then the verify and emission
  // items left.
  enum { ST_UNITS = 0, ST_VERIFY = 1, ST_EMIT = 2, ST_WRITE = 3 };
  const bool writer = wave >= kScanWaves - kScanWriters;  // never a chaser (kScanMaxBlocks)
  const uint32_t wid = writer ? wave - (kScanWaves - kScanWriters) : 0u;
  const int nsteps = chaser ? 2 : 3;
  for (int st = 0; st < nsteps; ++st) {
    const int kind = chaser ? (st == 0 ? ST_EMIT : ST_VERIFY)
                            : (st == 0 ? (writer ? ST_WRITE : ST_UNITS) : (st == 1 ? ST_VERIFY : ST_EMIT));
    if (kind == ST_WRITE) {
      // ---- the writers: the prefix rows to HBM, kWB ring slots (one batch) at a time in ticket order, batches dealt
      // round-robin to the kScanWriters writer waves. One wave-wide poll and kWB independent row reads per batch (a
      // row at a time was a chain of LDS round trips); kWDepth stores in flight per writer (the writers hardly ever
      // wait on their stores: kbench measures ~0.1 us of ack waits per writer). A unit is marked done once its store
      // has retired, kWDepth rows later or at the end (a shorter lag leaves fewer verify items for the tail) ----
      constexpr uint32_t kWB = 8;
      // (ABL & 512, kbench: the writer's wait time in stamp slot 7)
      constexpr uint32_t kD = kWDepth;
      uint64_t kb_wait = 0;
      uint32_t nrow = 0;  // rows this writer has issued
      for (uint32_t t = wid * kWB; t < nunits; t += kScanWriters * kWB) {
        const uint32_t nb = nunits - t < kWB ? nunits - t : kWB;
        {  // every slot of the batch filled (lanes 0..nb-1 poll one slot each)
          Spin sp;
          for (;;) {
            const uint32_t st = lane < nb ? __hip_atomic_load(&s_rstate[(t + lane) % kRing], __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_WORKGROUP)
                                          : 1u;
            if (__ballot(st == 0u) == 0ull) break;
            if (!sp.go(misc, 6)) break;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        uint32_t P[kWB], U[kWB];
#pragma unroll
        for (uint32_t j = 0; j < kWB; ++j) {
          const uint32_t slot = (t + j) % kRing;
          P[j] = j < nb ? s_ring[slot * 64 + lane] : 0u;
          U[j] = j < nb ? s_rstate[slot] - 1u : nunits;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // the rows are read before their slots are freed
        if (lane < nb) __hip_atomic_store(&s_rstate[(t + lane) % kRing], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (nrow >= kD) {  // this writer's rows nrow - kD .. + kWB have retired once kD - kWB remain
          const uint64_t tw = (ABL & 512) ? wall_clock64() : 0;
          static_assert(kWDepth == 16 && kWB == 8, "vmcnt below");
          asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          if (ABL & 512) kb_wait += wall_clock64() - tw;
#pragma unroll
          for (uint32_t j = 0; j < kWB; ++j) {
            const uint32_t ud = s_wunit[wid][(nrow + j) % kD];
            if (ud < nunits && lane == 0) atomicOr(&s_udone[ud >> 5], 1u << (ud & 31u));
          }
        }
        // (one 256 B row per store: 1 KiB stores of four rows each were slower, 338 vs 309 us at config B)
#pragma unroll
        for (uint32_t j = 0; j < kWB; ++j) {
          if (j < nb && !(ABL & 2048) && m0 + 64ull * U[j] + lane < m1) pw[64ull * U[j] + lane] = P[j];
          if (lane == 0) s_wunit[wid][(nrow + j) % kD] = U[j];
        }
        nrow += kWB;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stamp(3);
      for (uint32_t r = nrow > kD ? nrow - kD : 0; r < nrow; ++r) {
        const uint32_t ud = s_wunit[wid][r % kD];
        if (ud < nunits && lane == 0) atomicOr(&s_udone[ud >> 5], 1u << (ud & 31u));
      }
      if ((ABL & 512) && lane == 0) ea.kb_stamps[((uint64_t)blockIdx.x * kScanWaves + wave) * 8 + 7] = kb_wait;
    } else if (kind == ST_UNITS) {
      // ---- windows: units of 64 windows from the LDS counter ----
      const uint8_t* safe_win = seg_len >= kWin ? seg : reinterpret_cast<const uint8_t*>(tabs.lds_image);
      // ABL & 32: static contiguous unit ranges per wave instead of the LDS counter (kbench)
      const uint32_t su0 = nunits * wave / kScanWaves, su1 = nunits * (wave + 1) / kScanWaves;
      uint32_t snext = su0;
      auto take = [&]() -> uint32_t {
        if (ABL & 32) { const uint32_t r = snext < su1 ? snext : nunits; ++snext; return r; }
        uint32_t u = 0;
        if (lane == 0) u = atomicAdd(&s_unit, 1u);
        return __builtin_amdgcn_readfirstlane(u);
      };
      auto win_of = [&](uint32_t u) -> uint64_t { return m0 + 64ull * u + lane; };
      auto fast = [&](uint32_t u) {  // every lane's window is in the segment (and the workgroup's)
        return u < nunits && m0 + 64ull * u + 64 <= m1 && (m0 + 64ull * u + 64) * kWin <= seg_len;
      };
      // Two window buffers: a unit's loads are issued one unit ahead, so they fly through the other buffer's chain.
      // Every lane loads (an invalid unit reads a safe address) so the loads are one straight-line group, and no
      // load sits in a branch of the loop (the compiler then waits for every load in flight, both buffers'): the
      // unit that is not "fast" -- the workgroup's partial last unit, or one at the segment's end -- is set aside
      // and done after the loop with bounds-checked loads.
      // ABL & 8192 (kbench): lane-per-window loads instead of the quad-coalesced ones
      // 8 KiB every lane may read: the segment's start, or the table image (97 KiB) for a segment shorter than that
      // (whose units are then all slow ones)
      const uint8_t* safe_unit =
          seg_len >= 64 * kWin ? seg : reinterpret_cast<const uint8_t*>(tabs.lds_image);
      auto issue = [&](uint32_t u, uint32_t (&w)[32]) {
        if (!(ABL & 8192)) {
          load_unit_quad(fast(u) ? seg + (m0 + 64ull * u) * kWin : safe_unit, lane, w);
          return;
        }
        const uint4* q = reinterpret_cast<const uint4*>(fast(u) ? seg + win_of(u) * kWin : safe_win);
#pragma unroll
        for (int g = 0; g < 8; ++g) {
          const uint4 v = q[g];
          w[4 * g + 0] = v.x; w[4 * g + 1] = v.y; w[4 * g + 2] = v.z; w[4 * g + 3] = v.w;
        }
      };
      uint32_t kb_acc = 0;  // kbench (ABL & 2048): the prefixes folded here instead of stored
      uint64_t kb_ring_waits = 0;  // kbench (ABL & 512): spins on a full ring
      auto prefix = [&](uint32_t (&w)[32], bool valid) -> uint32_t {
        uint32_t v = (ABL & 1) ? (w[0] ^ w[31]) : crc_window(s_slice, s_half, sl, 0u, w);
        if (!valid) v = 0u;
        if (ABL & 1024) return v;
        v = apply_fwd(s_fwd, lane, v);
        return wave_scan_z(v, [](uint32_t x, uint32_t y) { return x ^ y; });
      };
      auto store = [&](uint32_t u, uint32_t P, bool valid) {  // the row into the writer's ring (every unit, once)
        if (ABL & 2048) kb_acc ^= P;
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(&s_rhead, 1u);
        const uint32_t slot = __builtin_amdgcn_readfirstlane(t) % kRing;
        Spin sp;
        while (__hip_atomic_load(&s_rstate[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u) {
          if (ABL & 512) ++kb_ring_waits;
          if (!sp.go(misc, 5)) break;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        s_ring[slot * 64 + lane] = P;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(&s_rstate[slot], u + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        (void)valid;
      };
      uint32_t deferred = nunits;  // this wave's slow unit, if it took one
      // a unit's prefixes, stored right away (fast units); a slow unit is only noted
      auto process = [&](uint32_t u, uint32_t (&w)[32]) {
        if (u < nunits) {
          if (fast(u)) {
            if (!(ABL & 8192)) unit_quad_transpose(w, lane);
            store(u, prefix(w, true), true);
          } else {
            deferred = u;
          }
        }
      };
      uint32_t wa[32], wb[32];
      // kbench: ABL & 128 -- only waves 2..9 take units
      const bool no_units = (ABL & 4) || ((ABL & 128) && (wave < 2 || wave > 9));
      uint32_t ua = no_units ? nunits : take();
      issue(ua, wa);
      uint32_t ub = no_units ? nunits : take();
      issue(ub, wb);
      // Per half: process the buffer (its prefixes into the writer's ring), then its next unit's 8 loads; the
      // compiler waits for the other buffer's loads (vmcnt(8): this half's loads stay in flight).
      // No exit between the halves (an exit there made the compiler wait for both buffers' loads): ub > ua, so a
      // half whose unit is past the end only skips its compute.
      while (ua < nunits) {
        process(ua, wa);
        ua = take();
        issue(ua, wa);
        process(ub, wb);
        ub = take();
        issue(ub, wb);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (deferred < nunits) {
        const uint64_t m = win_of(deferred);
        load_window(seg, seg_len, (int64_t)(m * kWin), false, wa);
        store(deferred, prefix(wa, m < m1), m < m1);
      }
      if ((ABL & 2048) && kb_acc == 0x9e3779b9u) pw[0] = kb_acc;
      stamp(3);
      if ((ABL & 512) && lane == 0) ea.kb_stamps[((uint64_t)blockIdx.x * kScanWaves + wave) * 8 + 7] = kb_ring_waits;
    } else if (kind == ST_VERIFY) {
      // ---- verify items (one lane per fragment, 64 consecutive fragments of the workgroup), each once its units
      // are stored ----
      wait_chase();
      stamp(4);
      uint64_t Fa, Fb;
      frag_range(Fa, Fb);
      for (; !(ABL & 2);) {
        uint32_t it = 0;
        if (lane == 0) it = atomicAdd(&s_vq, 1u);
        it = __builtin_amdgcn_readfirstlane(it);
        if (Fa + 64ull * it >= Fb) break;
        const uint64_t g = Fa + 64ull * it + lane;
        Frag f{};
        if (g < Fb) {
          const uint4 raw = reinterpret_cast<const uint4*>(frags)[g];
          __builtin_memcpy(&f, &raw, sizeof f);
        }
        const int64_t GS = (int64_t)start_off + (int64_t)f.blk * kBlock + f.start, GE = GS + f.len;
        const int64_t a = GS >> 7, j0 = GE >> 7, j1 = (GE + 3) >> 7;
        uint32_t mn, mx;
        if (it < kVItems) {
          mn = s_vlo[it];
          mx = s_vhi[it];
        } else {  // from the descriptors
          const bool has = g < Fb && j0 - 1 > a;
          mn = has ? (uint32_t)((a + 1 - M0) >> 6) : 0xffffffffu;
          mx = has ? (uint32_t)((j0 - 1 - M0) >> 6) : 0u;
#pragma unroll
          for (int d = 32; d >= 1; d >>= 1) {
            mn = min(mn, (uint32_t)__shfl_xor((int)mn, d, 64));
            mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
          }
          mn = __builtin_amdgcn_readfirstlane(mn);
          mx = __builtin_amdgcn_readfirstlane(mx);
        }
        {
          Spin sp;
          while (!units_done(mn, mx))
            if (!sp.go(misc, 7)) break;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (g < Fb) {
          // the edge windows one at a time (one window of registers)
          uint32_t z[3] = {0u, 0u, 0u};
#pragma unroll 1
          for (int e = 0; e < 3; ++e) {
            const int64_t m = e == 0 ? a : (e == 1 ? j0 : j1);
            if (e == 1 && j0 == a) continue;
            if (e == 2 && (j1 == j0 || j1 == a)) continue;
            const uint32_t v = edge_window(seg, seg_len, m, GS, GE, f.chk, s_slice, s_half, sl);
            z[0] = e == 0 ? v : z[0];
            z[1] = e == 1 ? v : z[1];
            z[2] = e == 2 ? v : z[2];
          }
          const int64_t pa = (a - M0) >> 6, pf = (j1 - M0) >> 6;
          uint32_t T = 0;
          for (int64_t p = pa; p <= pf; ++p) {
            if (p > pa) T = apply_op(s_carry, T);
            const int64_t wlo = M0 + 64 * p, whi = wlo + 63;
            const int64_t lo = a + 1 > wlo ? a + 1 : wlo, hi = j0 - 1 < whi ? j0 - 1 : whi;
            if (lo <= hi) T ^= pw[hi - M0] ^ (lo > wlo ? pw[lo - 1 - M0] : 0u);
            if (((a - M0) >> 6) == p) T ^= apply_fwd(s_fwd, (uint32_t)((a - M0) & 63), z[0]);
            if (j0 != a && ((j0 - M0) >> 6) == p) T ^= apply_fwd(s_fwd, (uint32_t)((j0 - M0) & 63), z[1]);
            if (j1 != j0 && j1 != a && ((j1 - M0) >> 6) == p) T ^= apply_fwd(s_fwd, (uint32_t)((j1 - M0) & 63), z[2]);
          }
          frags[g].ok = T == 0u ? 1 : 0;
          if (T != 0u) atomicMin(reinterpret_cast<unsigned long long*>(&misc[M_BAD_CRC]), (unsigned long long)g);
        }
      }
      stamp(5);
    } else if (!(ABL & 8)) {
      // ---- record emission: items of ~64 fragments over the workgroup's blocks (k_crc's emit_chunks) ----
      wait_chase();
      const uint64_t nitems = (s_em[1] - s_em[0] + s_em[2] - 1) / s_em[2];
      PredSync ps;
      ps.B0 = B0; ps.lbw = lbw; ps.wg = wg; ps.epoch = epoch; ps.misc = misc; ps.acq = (wg == 0);
      // the item geometry lives in LDS and is re-read per item: the emission runs at the register limit
      auto meta = [&](uint64_t it) -> ItemMeta {
        const uint64_t b0 = s_em[0], b1 = s_em[1], bpw = s_em[2];
        ItemMeta mm;
        mm.bb = b0 + it * bpw;
        if (mm.bb >= b1) mm.bb = b1 - 1;  // an exhausted queue: a clamped (unconditional) load
        const uint64_t be = mm.bb + bpw < b1 ? mm.bb + bpw : b1;
        mm.s = emit_prefetch(ea, mm.bb, lane);
        mm.f0 = ea.fbase[mm.bb];
        mm.f1 = be < b1 ? ea.fbase[be] : (uint32_t)s_em[3];
        mm.rec = ea.rbase[mm.bb];
        return mm;
      };
      auto deq = [&]() -> uint64_t {
        uint32_t j = 0;
        if (lane == 0) j = atomicAdd(&s_eq, 1u);
        return __builtin_amdgcn_readfirstlane(j);
      };
      uint64_t it = deq();
      ItemMeta m = meta(it);
      while (it < nitems) {
        const EmitState es = emit_state(ea, m.bb, lane, m.s, m.rec, ps);
        const uint64_t f1 = m.f1 < frag_cap ? m.f1 : frag_cap;
        uint64_t nx = 0;
        ItemMeta mn;
        emit_chunks<0>(ea, es, m.f0, f1, lane, [&]() {
          nx = deq();
          mn = meta(nx);
        });
        it = nx;
        m = mn;
      }
    }
  }

  stamp(6);
  // ---- completion (k_crc's protocol) ----
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  uint32_t order = 0;
  if (lane == 0) order = atomicAdd(&s_wdone, 1u);
  order = __builtin_amdgcn_readlane(order, 0);
  if (order != kScanWaves - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  uint64_t gorder = 0;
  if (lane == 0)
    gorder = __hip_atomic_fetch_add(&misc[M_DONE_CRC], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  gorder = (uint64_t)__shfl((long long)gorder, 0, 64);
  if (gorder != gridDim.x - 1u) return;
  finalize(ea, nblocks, frag_cap, tail_panic, gen, res, lane);
}

__global__ void k_export_frags(const Frag* __restrict__ frags, const uint64_t* __restrict__ misc, uint64_t cap,
                               uint32_t start_off, bcw_frag_table out, const uint32_t* __restrict__ initc) {
  const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t n = misc[M_NFRAGS];
  if (g >= n || g >= cap || g >= out.capacity) return;
  const Frag f = frags[g];
  out.data_off[g] = (uint64_t)start_off + (uint64_t)f.blk * kBlock + f.start;
  out.len[g] = f.len;
  const uint32_t u = ~(f.chk ^ initc[f.len]);  // unmask(stored), from J
  out.stored_crc[g] = ((u >> 15) | (u << 17)) + 0xa282ead8u;
  out.type[g] = f.type;
  out.crc_ok[g] = f.ok;
}



// ------------------------------------------------------------------------------------------
hipError_t launch_decode(const uint8_t* d_seg, const bcw_decode_params& p, const bcw_record_table& t,
                         bcw_decode_result* d_result, const Tables& tabs, Scratch& s, uint64_t nblocks,
                         uint64_t gen, hipStream_t stream, int num_cus, Prof* prof) {
  Prof dummy;
  Prof& pr = prof ? *prof : dummy;
  hipEvent_t ev = nullptr;
  const uint64_t tail = (p.seg_len - p.start_off) % kBlock;
  const uint32_t tail_panic = (tail > 0 && tail < kHdr) ? 1u : 0u;
  auto next_epoch = [&]() {
    if ((++s.epoch & 0xffffffull) == 0) {  // 24-bit look-back epochs: clear the words before reuse
      (void)hipMemsetAsync(s.lb, 0, s.nlb * sizeof(uint64_t), stream);
      (void)hipMemsetAsync(s.lbe, 0, s.nlb * sizeof(uint64_t), stream);
      (void)hipMemsetAsync(s.lbw, 0, s.nlb * sizeof(uint64_t), stream);
      s.epoch = 1;
    }
  };
  if (s.scan && nblocks <= (uint64_t)kScanMaxBlocks * (uint64_t)num_cus) {  // one launch (k_scan)
    const uint32_t grid = (uint32_t)(nblocks < (uint64_t)num_cus ? nblocks : (uint64_t)num_cus);
    const EmitArgs ea{d_seg, p.seg_len, p, s.frags, s.fbase, s.rbase, s.bsum, t, s.misc, s.equeue, 0u, nullptr};
    pr.begin(K_SCAN, stream, ev);
    k_scan<0><<<grid, kScanThreads, 0, stream>>>(d_seg, p.seg_len, p.start_off, nblocks, s.fbase, s.rbase, s.bsum,
                                                s.frags, s.frag_cap, s.pwin, scan_unit_stride(nblocks, grid), s.lb,
                                                s.lbe, s.lbw, s.tickets, s.epoch, tabs, ea, tail_panic, gen, d_result);
    pr.end(K_SCAN, stream, ev);
    s.tickets += grid;
    next_epoch();
    return hipGetLastError();
  }
  const uint32_t nb_grid = (uint32_t)((nblocks + 63) / 64);
  const EmitArgs ea{d_seg, p.seg_len, p, s.frags, s.fbase, s.rbase, s.bsum, t, s.misc, s.equeue, 0u, nullptr};
  // Two chunks for a segment of at least 128 blocks per CU: k_chase over the second chunk runs beside k_crc over the
  // first, and the second k_crc's workgroups take the CUs the first one's finishing workgroups free (each k_crc on a
  // stream of its own; the call's stream waits for both). The chunks split at a multiple of 64 blocks, a k_chase
  // workgroup's range, whose end bases that workgroup writes. A k_crc's emission items stay inside its chunk; a
  // record that began in an earlier chunk reads that chunk's (finished) tables.
  const bool two = (s.chunks == 2 && nblocks >= 128ull * (uint64_t)num_cus) || (s.chunks == 3 && nblocks >= 128);
  if (two && !s.cs[0]) {
    for (auto& c : s.cs)
      if (hipStreamCreateWithFlags(&c, hipStreamNonBlocking) != hipSuccess) return hipErrorOutOfMemory;
    for (auto& e : s.cev)
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return hipErrorOutOfMemory;
  }
  const uint64_t cut = two ? (nblocks / 2 + 63) / 64 * 64 : nblocks;  // blocks of the first chunk
  const uint32_t g0n = (uint32_t)((cut + 63) / 64);
  pr.begin(K_CHASE, stream, ev);
  k_chase<0><<<g0n, 64, 0, stream>>>(d_seg, p.seg_len, p.start_off, nblocks, s.fbase, s.rbase, s.bsum, s.frags,
                                    s.frag_cap, s.lb, s.lbe, s.misc, s.tickets, s.epoch, tabs.initc, s.chase_direct,
                                    s.equeue);
  if (!two) {
    pr.end(K_CHASE, stream, ev);
    s.tickets += nb_grid;
    next_epoch();
    pr.begin(K_CRC, stream, ev);
    k_crc<0><<<(uint32_t)num_cus, kCrcThreads, 0, stream>>>(d_seg, p.seg_len, p.start_off, nblocks, s.fbase, s.frags,
                                                           s.frag_cap, tabs, ea, tail_panic, gen, d_result, s.misc,
                                                           0ull, nblocks, (uint32_t)num_cus);
    pr.end(K_CRC, stream, ev);
    return hipGetLastError();
  }
  (void)hipEventRecord(s.cev[0], stream);
  // (the second chase continues the first one's tickets: its workgroups are g0n.. of the segment's)
  k_chase<0><<<nb_grid - g0n, 64, 0, stream>>>(d_seg, p.seg_len, p.start_off, nblocks, s.fbase, s.rbase, s.bsum,
                                              s.frags, s.frag_cap, s.lb, s.lbe, s.misc, s.tickets, s.epoch,
                                              tabs.initc, s.chase_direct, s.equeue);
  pr.end(K_CHASE, stream, ev);
  (void)hipEventRecord(s.cev[1], stream);
  s.tickets += nb_grid;
  next_epoch();
  // profiling: one K_CRC interval from the first chunk's k_crc start to the second's end (events on both streams)
  (void)hipStreamWaitEvent(s.cs[0], s.cev[0], 0);
  (void)hipStreamWaitEvent(s.cs[1], s.cev[1], 0);
  pr.begin(K_CRC, s.cs[0], ev);
  k_crc<0><<<(uint32_t)num_cus, kCrcThreads, 0, s.cs[0]>>>(d_seg, p.seg_len, p.start_off, nblocks, s.fbase, s.frags,
                                                          s.frag_cap, tabs, ea, tail_panic, gen, d_result, s.misc,
                                                          0ull, cut, 2u * (uint32_t)num_cus);
  k_crc<0><<<(uint32_t)num_cus, kCrcThreads, 0, s.cs[1]>>>(d_seg, p.seg_len, p.start_off, nblocks, s.fbase, s.frags,
                                                          s.frag_cap, tabs, ea, tail_panic, gen, d_result, s.misc,
                                                          cut, nblocks, 2u * (uint32_t)num_cus);
  (void)hipEventRecord(s.cev[2], s.cs[0]);
  (void)hipStreamWaitEvent(s.cs[1], s.cev[2], 0);  // the interval's end (and the join) after both
  pr.end(K_CRC, s.cs[1], ev);
  (void)hipEventRecord(s.cev[3], s.cs[1]);
  (void)hipStreamWaitEvent(stream, s.cev[3], 0);
  return hipGetLastError();
}

hipError_t launch_export_frags(const Scratch& s, const bcw_frag_table& out, uint32_t start_off, hipStream_t stream,
                               uint64_t n, const uint32_t* initc) {
  if (n == 0) return hipSuccess;
  k_export_frags<<<(uint32_t)((n + 255) / 256), 256, 0, stream>>>(s.frags, s.misc, s.frag_cap, start_off, out,
                                                                    initc);
  return hipGetLastError();
}

}  // namespace bcw
