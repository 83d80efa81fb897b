// bcw_decode.hip -- MI355X (gfx950) kernels for bitcaskDB WAL segment decode + CRC verify.
//
// Pipeline (one HIP stream, no host synchronisation inside):
//   k_chase    one lane per 32 KiB block: header chase (wal_iterator.go:45-77), workgroup scan of the
//              fragment counts, predecessor sums / decoupled look-back over workgroups, fragment table, block
//              bases and record-state summaries
//   k_crc      one workgroup per CU: per-fragment masked CRC-32C verify as a zero test (wal_iterator.go:79 /
//              utils.go:24-29) streamed over absolute 1 KiB chunks (stream_verify), then record emission +
//              RecordFromBytes (record.go:140-239) / HintRecord.Decode (hint.go:50-84) from the chase alone
//              (emit_chunks); the last workgroup writes bcw_decode_result (finalize)
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
       M_ABORT = 12,     // k_chase: the wait site that timed out (0: none); reported as BCW_ERR_INTERNAL
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
// cache-resident by then). A workgroup only waits on lower workgroup ids (dispatched before it). Look-back words:
// epoch << 40 | flag << 38 | count (flag 1: aggregate, 2: inclusive prefix). One wave per workgroup spreads the blocks over every CU: the chase is a chain
// of scattered header reads, bound by latency and by each CU's address-processing rate.
//
// The chase is the iterator's header loop (wal_iterator.go:45-77: the block's buffer is
// min(32768, Size - fileOff) bytes, a header is parsed while bufOff + 7 <= bufSize, the data length is
// clamped to the buffer), a dependent chain of header reads (chase_block).
// A bounded wait (k_chase's predecessor waits): every spin gives up after 200 ms (a correct wait lasts microseconds)
// or once another wave has given up, records its site in misc[M_ABORT] and lets the kernel run to its end; the decode
// then reports BCW_ERR_INTERNAL instead of hanging the device. k_crc skips its CRC pass and emission over the
// unreliable bases, and the finalizer delivers no row. A wait that gave up counts its word as 0. (BCW_OPT_TEST_ABORT_WAIT
// makes one workgroup's Spin give up at its first step, with lim = 0.)
struct Spin {
  uint64_t t0 = 0;
  uint64_t lim = 20000000ull;  // 200 ms of the 100 MHz wall clock
  __device__ __forceinline__ bool go(uint64_t* misc, uint32_t site) {  // true: keep waiting
    const uint64_t t = wall_clock64();
    if (t0 == 0) t0 = t;
    if (t - t0 < lim &&
        __hip_atomic_load(&misc[M_ABORT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0ull) {
      __builtin_amdgcn_s_sleep(1);
      return true;
    }
    atomicMax(reinterpret_cast<unsigned long long*>(&misc[M_ABORT]), (unsigned long long)site);
    return false;
  }
};

constexpr int kChaseHold = 64;
constexpr uint64_t kLbAgg = 1, kLbInc = 2, kLbMask = (1ull << 38) - 1;
constexpr int kDirect = BCW_CHASE_DIRECT_MAX;  // k_chase workgroups up to which each sums all predecessors' aggregates

// visit(k, start, len, crc, type) for every header of the block from header n at block offset h on; returns the
// fragment count. One header per round: speculative stride reads (several predicted headers per round once two
// consecutive Full fragments had equal lengths) cost more than they saved (config C k_chase 60 -> 29 us without
// them, round 4).
template <typename V>
__device__ __forceinline__ uint32_t chase_block(const uint8_t* __restrict__ seg, uint64_t seg_len, uint64_t boff,
                                                uint32_t bufsize, V&& visit, uint32_t h = 0, uint32_t n = 0) {
  while (h + kHdr <= bufsize) {
    uint32_t crc, len, type;
    read_header(seg, seg_len, boff + h, crc, len, type);
    const uint32_t start = h + kHdr;
    if (len > bufsize - start) len = bufsize - start;  // wal_iterator.go:75
    visit(n, start, len, crc, type);
    ++n;
    h = start + len;
  }
  return n;
}

// The fragment table entry, one 16 B store (Frag: blk | start, len | chk | type, ok 0, pad 0; the stored CRC is kept as
// the check word J, see Frag; ic = initc[len]), and the fragment's stream record (k_crc's stream verify reads only
// these): x = end chunk ce = ge / 1024, y = begin chunk cb = gs / 1024 (absolute 1 KiB chunks of the segment; gs, ge
// the data's absolute byte range), z = J, w = pb | pa << 10 | kRecUsual | kRecAdj with pb = ge % 1024, pa = gs % 1024.
// kRecAdj: the next fragment's data starts at ge + 7 (a header follows at once: the next header of the block, or the
// next block's first when the data ends exactly at this full block's end). kRecUsual: kRecAdj, the fragment began in an
// earlier chunk and pb <= 1016 (its J and the next fragment's start lie in chunk ce) -- chunk ce then needs one
// gap mask and one close, provided the next fragment's data runs past it (k_crc checks that on the next record).
// Bits 22-28: Lfull, the lanes [0, Lfull) whose 16 B piece of chunk ce holds only the fragment's bytes (and J); bits
// 29-31: K, the fragment's J ends in word K of lane Lfull's piece (0 or 4: no lane is split), as stream_verify's
// close derives them from pb.
constexpr uint32_t kRecUsual = 1u << 20, kRecAdj = 1u << 21;
__device__ __forceinline__ uint32_t check_word(uint32_t crc, uint32_t ic) { return ~rotl32(crc - 0xa282ead8u, 15) ^ ic; }
__device__ __forceinline__ void put_frag_J(Frag* __restrict__ frags, uint4* __restrict__ srec, uint64_t g,
                                           uint64_t frag_cap, uint32_t b, uint64_t boff, uint32_t start_len,
                                           uint32_t J, uint32_t type, bool adj) {
  if (g >= frag_cap) return;
  *reinterpret_cast<uint4*>(frags + g) = make_uint4(b, start_len, J, type & 0xffu);
  const uint64_t gs = boff + (start_len & 0xffffu), ge = gs + (start_len >> 16);
  const uint32_t cb = (uint32_t)(gs / kSChunk), ce = (uint32_t)(ge / kSChunk);
  const uint32_t pa = (uint32_t)(gs % kSChunk), pb = (uint32_t)(ge % kSChunk);
  const bool usual = adj && cb < ce && pb <= (uint32_t)kSChunk - 8u;
  const uint32_t e = pb + 4u, K = ((e % kSPiece) + 3u) >> 2, Lfull = e / kSPiece + (K == (uint32_t)kSPW ? 1u : 0u);
  srec[g] = make_uint4(ce, cb, J, pb | pa << 10 | (usual ? kRecUsual : 0u) | (adj ? kRecAdj : 0u) | Lfull << 22 |
                                      (K & 3u) << 29);
}
__device__ __forceinline__ void put_frag(Frag* __restrict__ frags, uint4* __restrict__ srec, uint64_t g,
                                         uint64_t frag_cap, uint32_t b, uint64_t boff, uint32_t start, uint32_t len,
                                         uint32_t crc, uint32_t type, const uint32_t* __restrict__ initc, bool adj) {
  put_frag_J(frags, srec, g, frag_cap, b, boff, start | (len << 16), check_word(crc, initc[len]), type, adj);
}

// Block summary for the record state machine (wal_iterator.go:69-96), written by k_chase from the headers alone:
// the state of the iterator after a block depends only on the fragment types and lengths before it (a CRC
// failure or unknown type ends the iteration, and nothing after the first failing fragment is emitted), so
// record emission needs no CRC verdict. x = tail length | tail first non-empty fragment (block-local index,
// 0xffff: none) << 16; y = that fragment's block-relative start | has-Full/Last << 16. The tail is the part
// after the block's last Full/Last fragment (the whole block when it has none).
constexpr uint32_t kSumHasE = 1u << 16;

// The 8 class weights of XBal (lane k of xw holds class k's: 65536 + 256 d_k, |d_k| < 128) as uniform scalars: the
// d_k packed in bytes, their prefix sums in 16-bit fields. A class is picked by shifts (selects or an indexed array
// became a lookup table in scratch memory, which cost k_chase ~20 us).
struct ClassW {
  uint64_t pw;        // byte k: d_k
  uint64_t pp0, pp1;  // 16-bit field k (of pp0 for k < 4, of pp1 for k >= 4): d_0 + ... + d_{k-1}
  uint64_t p8;        // all weights
  __device__ __forceinline__ uint64_t weight(uint32_t y) const {
    return (uint64_t)(65536 + 256 * (int64_t)(int8_t)(uint8_t)(pw >> (8u * y)));
  }
  __device__ __forceinline__ uint64_t prefix(uint32_t y) const {
    const uint64_t f = (y < 4u ? pp0 : pp1) >> (16u * (y & 3u));
    return (uint64_t)(65536 * (int64_t)y + 256 * (int64_t)(int16_t)(uint16_t)f);
  }
  // the classes k >= 1 whose prefix lies at or below x
  __device__ __forceinline__ uint32_t classes_below(double x) const {
    uint32_t n = 0;
#pragma unroll
    for (uint32_t k = 1; k < 8; ++k) n += (double)prefix(k) <= x ? 1u : 0u;
    return n;
  }
};
// k_crc's wave boundaries: range r (workgroup r, class r % 8) has its class's weight; wave v = 16 r + j starts at
// the fraction num16(v) / den16 of the segment after start_off, num16(v) = 16 x (weights of ranges < r) +
// weight(r % 8) j, rounded down to 1 KiB: P(v) = 1024 floor(num16(v) C / den16), C = floor(L / 1024) (exact in 64 bits
// up to 512 GiB). Its inverse is exact too: the first v with P(v) >= x is the first with num16(v) >= N =
// ceil(ceil(x / 1024) den16 / C).
// floor(a / b) for a < 2^62, 0 < b < 2^32, from a floating-point estimate (rb = 1 / b) and exact steps: a 64-bit
// integer division is a ~100-instruction sequence, and k_chase's table pass ran 8 k cycles longer with four of them
__device__ __forceinline__ uint64_t div_floor(uint64_t a, uint64_t b, double rb) {
  uint64_t q = (uint64_t)((double)a * rb);
  while (q * b > a) --q;
  while ((q + 1) * b <= a) ++q;
  return q;
}
struct WavePart {
  ClassW cw;
  uint64_t L, nwaves, round16, den16, C;
  double rden, rC;
  __device__ __forceinline__ WavePart(const ClassW& c, uint64_t L_, uint64_t nwaves_) : cw(c), L(L_), nwaves(nwaves_) {
    const uint32_t G = (uint32_t)(nwaves / kCrcWaves);
    round16 = 16ull * cw.p8;
    den16 = round16 * (G / 8u) + 16ull * cw.prefix(G % 8u);
    C = L / 1024u;
    rden = 1.0 / (double)den16;
    rC = C ? 1.0 / (double)C : 0.0;
  }
  __device__ __forceinline__ uint64_t P(uint64_t v) const {
    if (v >= nwaves) return L;
    const uint64_t r = v / kCrcWaves;
    const uint32_t y = (uint32_t)(r % 8u);
    const uint64_t num16 = round16 * (r / 8u) + 16ull * cw.prefix(y) + cw.weight(y) * (v % kCrcWaves);
    return 1024u * div_floor(num16 * C, den16, rden);
  }
  __device__ __forceinline__ uint64_t first_at(uint64_t x) const {
    if (C == 0) return x == 0 ? 0 : nwaves;  // (a segment under 1 KiB: every boundary but the last at 0)
    const uint64_t X = (x + 1023u) / 1024u, N = div_floor(X * den16 + C - 1, C, rC);
    const uint32_t q = (uint32_t)N / (uint32_t)round16;  // (N <= den16 + 1 < 2^32)
    const uint64_t rem = N - (uint64_t)q * round16;
    uint32_t y = 0;
#pragma unroll
    for (uint32_t k = 1; k < 8; ++k) y += 16ull * cw.prefix(k) <= rem ? 1u : 0u;
    const uint64_t wy = cw.weight(y), base = 16ull * cw.prefix(y);
    const uint32_t jj = (uint32_t)(rem - base + wy - 1) / (uint32_t)wy;  // 0..16 (16: the next range's first wave)
    const uint64_t v = ((uint64_t)q * 8u + y) * kCrcWaves + jj;
    return v < nwaves ? v : nwaves;
  }
};

__device__ __forceinline__ ClassW class_weights(uint32_t xw) {
  ClassW c{0, 0, 0, 0};
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t d = ((int64_t)__builtin_amdgcn_readlane(xw, k) - 65536) / 256;
    c.pw |= (uint64_t)(uint8_t)(int8_t)d << (8 * k);
    if (k < 4) c.pp0 |= (uint64_t)(uint16_t)(int16_t)acc << (16 * k);
    else c.pp1 |= (uint64_t)(uint16_t)(int16_t)acc << (16 * (k - 4));
    acc += d;
  }
  c.p8 = (uint64_t)(65536 * 8 + 256 * acc);
  return c;
}

// ABL: ablation bits for tools/kbench only (0 in the product): 1 no predecessor sum, 2 no table writes,
// 16 phase cycles (chase, sum, writes; s_memtime) summed into misc[7..9], 32 per-workgroup wall-clock stamps (entry,
// chase end, sum end, end) into lbe[4 wg ..] (kbench passes a buffer of its own; direct-sum sizes only)
template <int ABL = 0>
__global__ __launch_bounds__(64) void k_chase(const uint8_t* __restrict__ seg, uint64_t seg_len, uint32_t start_off,
                                              uint64_t nblocks, uint32_t* __restrict__ fbase,
                                              uint32_t* __restrict__ rbase, uint2* __restrict__ bsum,
                                              Frag* __restrict__ frags, uint4* __restrict__ srec, uint64_t frag_cap,
                                              uint64_t* __restrict__ lb,
                                              uint64_t* __restrict__ lbe, uint64_t* __restrict__ misc,
                                              uint64_t epoch, const uint32_t* __restrict__ initc,
                                              uint32_t direct_max, uint64_t test_abort_wg,
                                              uint32_t* __restrict__ wstart, uint32_t nwaves,
                                              XBal* __restrict__ xb, uint32_t xb_on) {
  // {crc, start | len << 16} and type of each lane's first 64 headers: 36 KiB, so a k_chase workgroup still fits beside
  // a k_crc workgroup (which leaves 44 KiB of the CU's LDS since round 4) when another segment's decode is in flight.
  // A block with more headers is chased a second time from the 65th on when its table entries are written (16 held
  // headers, round 3: config C k_chase 69.5 vs 58.9 us with 64, kbench)
  // (ABL & 256, kbench: 16 held headers per lane, the round-3 size)
  constexpr int kHold = (ABL & 256) ? 16 : kChaseHold;
  __shared__ uint32_t s_hold[kHold][2][64];
  __shared__ uint8_t s_type[kHold][64];
  const uint32_t lane = threadIdx.x;
  // k_crc's per-XCD split (XBal): the range weight of each class, requested now, used after the chase
  const uint32_t xw = lane < 8u ? (xb_on ? xb->w[lane] : 65536u) : 0u;
  const uint64_t tc0 = (ABL & 16) ? __builtin_amdgcn_s_memtime() : 0;
  if ((ABL & 32) && threadIdx.x == 0) lbe[4 * blockIdx.x] = wall_clock64();
  // the workgroup id orders the look-back: workgroups are dispatched in id order (within each XCD), so one only waits
  // on ids already running; the bounded waits (Spin) turn any other schedule into BCW_ERR_INTERNAL, never a hang.
  // (Round 4 took tickets from one atomic counter: its 512 returning atomics on one word ended 5-7 us apart, and the
  // last ticket's chase gated every base: k_chase B 22.1 -> 16.8 us, C 31.3 -> 24.3 us without them, kbench.)
  const uint64_t wg = blockIdx.x;
  if (wg >= (nblocks + 63) / 64) return;  // (the grid is padded to a multiple of 8 workgroups, see launch_decode)
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
  if ((ABL & 32) && lane == 0) lbe[4 * wg + 1] = wall_clock64();
  if (wg == 0 && lane == 0) xb->on = xb_on;
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
  const bool force = wg + 1 == test_abort_wg;  // BCW_OPT_TEST_ABORT_WAIT (wave-uniform)
  uint64_t excl = 0, excl_e = 0;
  const uint32_t nh = n < (uint32_t)kHold ? n : (uint32_t)kHold;
  // the held headers' check words J (their initc[len] loads issued 16 at a time), computed while the predecessors'
  // counts are awaited: only the stores are left for after the sum (s_hold[k][0] holds J from here on)
  auto held_checks = [&]() {
    if (ABL & 2) return;
    constexpr uint32_t kWb = 16;
    static_assert(kHold % kWb == 0, "held-header batches stay inside s_hold");
    for (uint32_t k0 = 0; k0 < nh; k0 += kWb) {
      uint32_t ic[kWb];
#pragma unroll
      for (uint32_t q = 0; q < kWb; ++q) ic[q] = initc[k0 + q < nh ? s_hold[k0 + q][1][lane] >> 16 : 0u];
#pragma unroll
      for (uint32_t q = 0; q < kWb; ++q)
        if (k0 + q < nh) s_hold[k0 + q][0][lane] = check_word(s_hold[k0 + q][0][lane], ic[q]);
    }
  };
  if (ABL & 1) {
    held_checks();
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
    held_checks();
    // the words not yet published are polled again all together (one round trip per poll, not one per word: polled
    // one word at a time, the sum ended ~5 us after the last chase on B, kbench k_chase stamps)
    Spin sp;  // bounded (BCW_ERR_INTERNAL)
    if (force) sp.lim = 0;
    for (;;) {
      bool wait = force;
#pragma unroll
      for (int k = 0; k < kDirect / 64; ++k) wait |= (v[k] >> 40) != epoch;
      if (!__builtin_amdgcn_readfirstlane((uint32_t)(__ballot(wait) != 0ull))) break;
      if (!sp.go(misc, 9)) {
#pragma unroll
        for (int k = 0; k < kDirect / 64; ++k)
          if ((v[k] >> 40) != epoch) v[k] = 0;
        break;
      }
#pragma unroll
      for (int k = 0; k < kDirect / 64; ++k) {
        const uint64_t q = lane + 64u * k;
        if ((v[k] >> 40) != epoch) v[k] = __hip_atomic_load(&lb[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    uint64_t c = 0, ce = 0;
#pragma unroll
    for (int k = 0; k < kDirect / 64; ++k) {
      const uint64_t q = lane + 64u * k;
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
    held_checks();
    // both counts walk back together; each stops at its own nearest inclusive prefix (the two words of a
    // predecessor turn inclusive one after the other)
    bool dn = false, de = false;
    for (uint64_t top = wg; top > 0 && !(dn && de);) {  // predecessors [top - 64, top)
      const uint64_t q = top - 1 - lane;  // lane 0: the nearest
      uint64_t vn = 0, ve = 0;
      if (top > lane) {
        Spin sp;
        if (force) sp.lim = 0;
        if (!dn)
          while (((vn = __hip_atomic_load(&lb[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 40) != epoch || force)
            if (!sp.go(misc, 10)) { vn = 0; break; }
        if (!de)
          while (((ve = __hip_atomic_load(&lbe[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 40) != epoch || force)
            if (!sp.go(misc, 11)) { ve = 0; break; }
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
  if ((ABL & 32) && lane == 0) lbe[4 * wg + 2] = wall_clock64();
  if (b < nblocks && !(ABL & 2)) {
    fbase[b] = (uint32_t)(g0 < 0xffffffffull ? g0 : 0xffffffffull);
    const uint64_t r0 = excl_e + incl_e - ne;
    rbase[b] = (uint32_t)(r0 < 0xffffffffull ? r0 : 0xffffffffull);
    bsum[b] = make_uint2(tacc | (tnz << 16), tst | (ne ? kSumHasE : 0u));
    if (badk != 0xffffffffu)  // the first unknown-type fragment of the segment (reset by the previous finalize)
      atomicMin(reinterpret_cast<unsigned long long*>(&misc[M_BAD_TYPE]), (unsigned long long)(g0 + badk));
    // the held headers' entries (their J computed during the wait, held_checks). The block's last fragment is
    // adjacent to the next block's first when it ends exactly at this full block's end and the next block holds a
    // header.
    const bool next_hdr = b + 1 < nblocks && seg_len - (boff + kBlock) >= kHdr;
    auto adj = [&](uint32_t k, uint32_t sl_k) { return k + 1u < n || (next_hdr && (sl_k & 0xffffu) + (sl_k >> 16) == kBlock); };
    // k_crc's wave ranges, balanced by bytes: wave w streams the fragments whose header lies in [P_w, P_w+1)
    // (positions after start_off), so wstart[w] = the first fragment whose header is at or after P_w. This lane writes the boundaries that fall in its block, walking its headers in order.
    // (Whole blocks per wave left 7 of config B's 4096 waves with 9 blocks instead of 8: they ended ~20 us after the
    // median wave, kbench timelines.)
    // Range r (k_crc's workgroup r, class r % 8) has its class's weight (WavePart). This lane writes the boundaries
    // that lie in its block: from the first at or after its start while they lie before its end (the segment's last
    // block: every one left, up to P_nwaves = L, which lies at its span's end when L is a multiple of 32 KiB). (A
    // second first_at for the block's end cost ~1 us of k_chase's table pass.)
    const uint64_t L = seg_len - start_off, rel = boff - start_off;
    const WavePart wp(class_weights(xw), L, nwaves);
    const uint64_t span = b + 1 == nblocks ? ~0ull : (uint64_t)kBlock - 1;  // the last position it owns
    uint64_t w = wp.first_at(rel);
    uint64_t bw = wp.P(w) - rel;  // boundary w, block-relative
    auto bounds_upto = [&](uint64_t hp, uint64_t idx) __attribute__((always_inline)) {  // boundaries at or before hp: idx
      const uint64_t h = hp < span ? hp : span;
      while (w <= nwaves && bw <= h) {
        wstart[w] = (uint32_t)(idx < 0xffffffffull ? idx : 0xffffffffull);
        ++w;
        bw = wp.P(w) - rel;
      }
    };
    for (uint32_t k = 0; k < nh; ++k) {
      const uint32_t sl = s_hold[k][1][lane];
      put_frag_J(frags, srec, g0 + k, frag_cap, (uint32_t)b, boff, sl, s_hold[k][0][lane], s_type[k][lane],
                 adj(k, sl));
      bounds_upto((sl & 0xffffu) - kHdr, g0 + k);
    }
    if (n > (uint32_t)kHold)  // the tail of a block with more headers than held, chased again from the first of them
      chase_block(seg, seg_len, boff, bufsize, [&](uint32_t k, uint32_t start, uint32_t len, uint32_t crc, uint32_t type) {
        put_frag(frags, srec, g0 + k, frag_cap, (uint32_t)b, boff, start, len, crc, type, initc,
                 adj(k, start | (len << 16)));
        bounds_upto(start - kHdr, g0 + k);
      }, hres, (uint32_t)kHold);
    bounds_upto(~0ull, g0 + n);  // boundaries after the block's last header: the next block's first fragment
  }
  if (ABL & 32) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) lbe[4 * wg + 3] = wall_clock64();
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
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// F_l(x): lane-replicated nibble images, lane l reads its own copy (bank = l % 32). Byte offsets: nibble image i of
// value v at i * 4096 + v * 256 + 4 l, so each address is one shift and one v_and_or_b32 (the lane's 4 l never
// overlaps the 0xf00 field) and the image offset i * 4096 is the ds_read immediate (the operators lie first in LDS).
__device__ __forceinline__ uint32_t apply_fwd(const uint32_t* __restrict__ fwd, uint32_t lane, uint32_t x) {
  const uint8_t* b = reinterpret_cast<const uint8_t*>(fwd);
  const uint32_t lane4 = 4u * lane;
  auto at = [&](int i) -> uint32_t {
    const uint32_t sh = 4 * i >= 8 ? (x >> (4 * i - 8)) : (x << (8 - 4 * i));
    return *reinterpret_cast<const uint32_t*>(b + (((sh & 0xf00u) | lane4) + 4096u * (uint32_t)i));
  };
  const uint32_t r0 = at(0), r1 = at(1), r2 = at(2), r3 = at(3), r4 = at(4), r5 = at(5), r6 = at(6), r7 = at(7);
  return xor3(xor3(r0, r1, r2), xor3(r3, r4, r5), r6) ^ r7;
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
  uint64_t tend;         // and the byte after its last
  const uint8_t* seg;
  const Frag* frags;
  uint32_t start_off;
  uint32_t f_first, f_last;
  __device__ __forceinline__ uint32_t operator()(uint64_t pos) {
    if (pos < nhead) return reg_byte(h, (uint32_t)pos);
    if (pos >= tstart && pos < tend) return reg_byte(t, (uint32_t)(pos - tstart));
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
  uint32_t kb_flags; // tools/kbench only (0 in the product): 1 = skip the emission at run time
  uint64_t* kb_stamps;  // tools/kbench only (null in the product): 8 words per wave {CRC done, emission done, items,
                        // fragments, entry (real time), entry (shader cycles), emission done (shader cycles),
                        // XCC id << 32 | HW_ID}
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

// walk back over the block summaries, 64 blocks a step, to the nearest block with a Full/Last fragment (before
// block 0: an empty state); s = emit_prefetch(A, b0, lane)
__device__ __forceinline__ EmitState emit_state(const EmitArgs& A, uint64_t b0, uint32_t lane, uint2 s, uint32_t rec) {
  EmitState st{0, -1, 0, 0, rec};
  uint64_t acc = 0;
  for (uint64_t top = b0; top > 0;) {
    if (top != b0) {
      const uint64_t q = top - 1 - lane;
      s = top > lane ? A.bsum[q] : make_uint2(0xffff0000u, kSumHasE);
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
// NOSTORE (tools/kbench only): the rows are computed but not stored
template <bool NOSTORE = false, bool NOPARSE = false, typename Hook>
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
    // the fragment after src (a record head that runs past its first fragment continues there)
    const bool nx_here = src + 1u >= c0 && src + 1u < c0 + 64;
    const uint32_t sx0 = (uint32_t)__shfl((int)f.blk, nx_here ? (int)(src + 1u - c0) : (int)lane, 64);
    const uint32_t sx1 = (uint32_t)__shfl((int)((uint32_t)f.start | ((uint32_t)f.len << 16)),
                                          nx_here ? (int)(src + 1u - c0) : (int)lane, 64);
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
      load_words(A.seg, A.seg_len, a0, rd.h);
      rd.tstart = rd.tend = ~0ull;
      if (hint) {  // the last bytes: HintRecord.Decode reads fid, offset and size after the key
        uint64_t nt = size < 32u ? size : 32u;
        if (nt > len) nt = len;
        rd.tstart = size - nt;
        load_words(A.seg, A.seg_len, D + len - nt, rd.t);  // this lane's (Full/Last) fragment ends the record
      } else if (want < (size < 64u ? size : 64u)) {
        // RecordFromBytes reads past the first fragment (a record that starts in the last bytes of a block): the next
        // fragment's first 32 B, loaded beside the head, instead of a fragment walk per byte (two dependent loads
        // each: one such record held its whole work item ~20 us)
        Frag f2;
        if (nx_here) { f2.blk = sx0; f2.start = (uint16_t)sx1; f2.len = (uint16_t)(sx1 >> 16); }
        else f2 = frags[src + 1u];
        load_words(A.seg, A.seg_len, (uint64_t)start_off + (uint64_t)f2.blk * kBlock + f2.start, rd.t);
        uint64_t n2 = f2.len < 32u ? f2.len : 32u;
        if (n2 > size - want) n2 = size - want;
        rd.tstart = want;
        rd.tend = want + n2;
      } else {
#pragma unroll
        for (int k = 0; k < kTailWords; ++k) rd.t[k] = 0;
      }
      rd.seg = A.seg; rd.frags = frags; rd.start_off = start_off;
      rd.f_first = src; rd.f_last = (uint32_t)g;
      uint8_t status, hdr, flags, etag_off;
      uint64_t key_len, val_len, meta_len, expire, aux0, aux1;
      if (NOPARSE) {  // (kbench: the head's words folded instead of parsed)
        status = 0; hdr = (uint8_t)rd.h[0]; flags = (uint8_t)rd.h[5]; etag_off = 0;
        key_len = rd.h[6] ^ rd.h[9]; val_len = rd.h[7] ^ rd.h[12]; meta_len = rd.h[8] ^ rd.h[15]; expire = rd.h[10];
        aux0 = rd.t[0]; aux1 = rd.t[1];
      } else {
        parse_record(A.p, rd, size, status, hdr, flags, etag_off, key_len, val_len, meta_len, expire, aux0, aux1);
      }
      const bcw_record_table& tab = A.tab;
      if (NOSTORE) {
        if (status == 0xeeu) tab.foff[r] = foff ^ size ^ expire ^ aux0 ^ aux1 ^ key_len ^ val_len ^ meta_len ^ hdr ^ flags ^ etag_off;
      } else if (r < tab.capacity) {
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
// a wave-uniform load of a table k_chase wrote (read-only in k_crc) through the constant address space: a scalar
// load, although the table pointer was reloaded from LDS (as a generic pointer it was a flat load from a VGPR address)
__device__ __forceinline__ uint32_t ld_const(const uint32_t* p, uint64_t i) {
  return ((const __attribute__((address_space(4))) uint32_t*)p)[i];
}
// item `it` of a chunk [cb0, cb1) of the segment's blocks: blocks [cb0 + it bpw, + bpw), cut at cb1
__device__ __forceinline__ ItemMeta item_meta(const EmitArgs& A, uint64_t it, uint64_t bpw, uint64_t cb0, uint64_t cb1,
                                              uint32_t lane) {
  ItemMeta m;
  m.bb = cb0 + it * bpw < cb1 ? cb0 + it * bpw : cb1 - 1;  // a clamped (unconditional) load for an exhausted queue
  const uint64_t be = m.bb + bpw < cb1 ? m.bb + bpw : cb1;
  m.s = emit_prefetch(A, m.bb, lane);
  m.f0 = ld_const(A.fbase, m.bb);
  m.f1 = ld_const(A.fbase, be);
  m.rec = ld_const(A.rbase, m.bb);
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
  const uint64_t abort_site = __hip_atomic_load(&misc[M_ABORT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t err = bad_crc < bad_type ? bad_crc : bad_type;
  // records before fragment `lim` (the first failing one, or the fragment capacity of a decode to be retried)
  uint64_t lim = err < frag_cap ? err : frag_cap;
  uint64_t nrec = __hip_atomic_load(&misc[M_NE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lim < nfr && abort_site == 0ull) {
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
  if (abort_site != 0ull) {
    // a wait gave up: the bases (and so every row) may come from stale look-back words. Deliver no row at all, so
    // that no consumer (the index puts, the compaction filter and encode, the host replay) applies one.
    r.err_class = BCW_ERR_INTERNAL;
    r.err_frag = abort_site;  // the wait site
    r.n_records = r.n_records_total = 0;
    nrec = 0;
  }
  r.err_file_off = 0;
  if (err != ~0ull && err < frag_cap && abort_site == 0ull) {
    const Frag f = A.frags[err];
    r.err_file_off = (uint64_t)A.p.start_off + (uint64_t)f.blk * kBlock + f.start - kHdr;
  }
  r.first_bad_record = fb < nrec ? (int32_t)(fb < 0x7fffffffull ? fb : 0x7fffffffull) : -1;
  r.n_blocks = nblocks;
  r.retry_frag_capacity = (nfr > frag_cap && abort_site == 0ull) ? nfr : 0;  // (a stale count is no capacity)
  r.generation = gen;
  *res = r;
  // after a give-up the fragment table and verdicts are stale (aborted waves verify nothing): the fragment export
  // (k_export_frags, bcw_decode_fragments) delivers no row for this decode
  if (abort_site != 0ull) misc[M_NFRAGS] = 0;
  // for the next decode (the scratch setup sets them first)
  misc[M_DONE_CRC] = 0;
  misc[M_BAD_CRC] = ~0ull;
  misc[M_FIRST_BAD] = ~0ull;
  misc[M_BAD_TYPE] = ~0ull;
  misc[M_ABORT] = 0;
}

// ------------------------------------------------------------------------------------------
// Stream verify: the CRC zero tests of a wave's fragments over absolute 1 KiB chunks of the segment. Lane l reads
// bytes [16l, 16l + 16) of a chunk: one fully contiguous non-temporal 1 KiB load per chunk and wave, independent of
// the fragment geometry (kbench spat: 160 us for a 1 GiB segment, against 164 us for a grid-stride stream and 176 us
// for the lane-per-window loads of the round-3 passes).
//
// Each lane runs a Horner chain over its 16 B pieces. Its state H_l is the raw CRC-32C of the current fragment's
// bytes up to its piece of the last chunk, shifted on by 1008 bytes: the frame of its piece in the next chunk, whose
// chain it seeds directly. The shift costs nothing: the last of a piece's 4 slice-by-4 steps looks up tables of
// "byte followed by k + 1008 zero bytes" (T'_k) instead of T_k. A chunk inside one fragment's data (the usual case)
// is that chain and nothing else. A chunk holding a fragment's end runs the chain over the piece masked to the
// fragment's data, its check word J written at [ge, ge + 4) (k_crc's zero test: R(data || J) = 0 iff
// ComputeCRC32(data) matches), and the next fragment's first bytes when that one's data runs past the chunk. With
// e = ge + 4 - C0 the lanes l < floor(e / 16) hold only the closing fragment's bytes (their part A_l = s_4); the lane
// L = floor(e / 16) (when e % 16 != 0) holds both, split at word K = ceil((e % 16) / 4) (3 header bytes lie between J
// and the next data): A_L = A_{8(4(4-K) + 1008)}(s_K), s_K its chain state after word K; the lanes after it hold
// only the next fragment's: A_l = A_{8(16 + 1008)}(seed). The next fragment's part is s_4 ^ A_l. The closing
// fragment's total, in the chunk-end frame (+1008), is the XOR over the lanes of G_l(A_l), G_l = A_{8*16*(63-l)}:
// it passes iff that is 0. A chunk with several fragment ends repeats this per fragment (a chain each).
struct StreamFrag {
  int64_t gs, ge;  // absolute data range
  uint32_t J;      // check word
};

// slice-by-4 lookups of the stream layout (kS2Slice): 256-B rows e = {T3, T2, T1, T0} x 8 copies, then the shifted
// tables {T3', T2', T1', T0'} x 8 copies. Lane l uses copy l % 8 and looks up the four tables in the rotated order
// starting at (l / 8) % 4, so the 8-lane groups of each 32-lane bank group read four different tables: every
// ds_read_b32 is conflict-free. One v_perm_b32 per lookup: byte 0 from the lane's base word, byte 1 from the state.
struct SliceLane2 {
  uint32_t base;    // byte k: (slot of lookup k) * 32 + copy * 4
  uint32_t sel[4];  // perm selectors of lookups 0..3
};
__device__ __forceinline__ SliceLane2 slice_lane2(uint32_t lane) {
  SliceLane2 s;
  const uint32_t g = (lane >> 3) & 3u, copy = lane & 7u;
  s.base = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    const uint32_t slot = (k + g) & 3u;  // lookup k reads state byte `slot` in table T_{3 - slot}
    s.base |= (slot * 32u + copy * 4u) << (8u * k);
    s.sel[k] = 0x0c0c0000u | ((4u + slot) << 8) | k;
  }
  return s;
}
// A_32(x) (or, SH, A_{8*1012}(x)) ^ next
template <bool SH>
__device__ __forceinline__ uint32_t slice4_step2(const uint8_t* __restrict__ tb, const SliceLane2& sl, uint32_t x,
                                                 uint32_t next) {
  constexpr uint32_t o = SH ? 128u : 0u;
  const uint32_t a0 = *reinterpret_cast<const uint32_t*>(tb + __builtin_amdgcn_perm(x, sl.base, sl.sel[0]) + o);
  const uint32_t a1 = *reinterpret_cast<const uint32_t*>(tb + __builtin_amdgcn_perm(x, sl.base, sl.sel[1]) + o);
  const uint32_t a2 = *reinterpret_cast<const uint32_t*>(tb + __builtin_amdgcn_perm(x, sl.base, sl.sel[2]) + o);
  const uint32_t a3 = *reinterpret_cast<const uint32_t*>(tb + __builtin_amdgcn_perm(x, sl.base, sl.sel[3]) + o);
  return xor3(xor3(a0, a1, a2), a3, next);
}
// A_{8*1008}(A_128(seed) ^ R(piece)); CAP: also the unshifted state after word K (1 <= K < kSPW, wave-uniform)
template <bool CAP>
__device__ __forceinline__ uint32_t chain_piece2(const uint8_t* __restrict__ tb, const SliceLane2& sl, uint32_t seed,
                                                 const uint32_t (&w)[kSPW], uint32_t K = 0, uint32_t* cap = nullptr) {
  uint32_t x = seed ^ w[0];
  uint32_t st[kSPW - 1];
#pragma unroll
  for (int q = 0; q < kSPW - 1; ++q) {
    x = slice4_step2<false>(tb, sl, x, w[q + 1]);
    if (CAP) st[q] = x ^ w[q + 1];
  }
  if (CAP) *cap = K == 1u ? st[0] : (K == 2u ? st[1] : st[2]);  // (uniform K: two selects, no branch)
  return slice4_step2<true>(tb, sl, x, 0u);
}

// chunks that can hold a fragment's data or check word: every byte of them lies before seg_len + 4
__device__ __forceinline__ uint64_t c_safe_bound(uint64_t seg_len) { return (seg_len + 4u + kSChunk - 1u) / kSChunk; }

// the 16 B select entry of lane l for a boundary at chunk-relative byte P (table of n entries, index clamped)
__device__ __forceinline__ uint4 lds_entry(const uint32_t* __restrict__ tab, uint32_t idx) {
  return *reinterpret_cast<const uint4*>(tab + 4u * idx);
}
// Fragment-end masks: x_j = v_perm(J, w_j, S_j), byte selectors S from LDS tables indexed by the boundary's offset in
// the lane's piece (no lane compares, no branches). The usual end: data on both sides of the 7 bytes [pb, pb + 7)
// (J over the next header's CRC field, its length and type bytes zeroed).
__device__ __forceinline__ void mask_gap(uint32_t (&x)[kSPW], const uint32_t (&w)[kSPW], int32_t pb, uint32_t J,
                                         uint32_t lane, const uint32_t* __restrict__ lds) {
  const uint32_t g = min((uint32_t)(pb - (int32_t)(kSPiece * lane) + 6), (uint32_t)(kS2GapN - 1));
  const uint4 S = lds_entry(lds + kS2Gap, g);
  x[0] = __builtin_amdgcn_perm(J, w[0], S.x);
  x[1] = __builtin_amdgcn_perm(J, w[1], S.y);
  x[2] = __builtin_amdgcn_perm(J, w[2], S.z);
  x[3] = __builtin_amdgcn_perm(J, w[3], S.w);
}
// The general end: only the bytes of [pa, pb) and [pc, kSChunk) kept and J written at [pb, pb + 4) (chunk-relative,
// wave-uniform, clamped to [-64, 4096]): keep = (GE[pa] & ~GE[pb]) | GE[pc], the others J's bytes or 0 (JSEL).
__device__ __forceinline__ void mask_chunk(uint32_t (&x)[kSPW], const uint32_t (&w)[kSPW], int32_t pa, int32_t pb,
                                           int32_t pc, uint32_t J, uint32_t lane, const uint32_t* __restrict__ lds) {
  const int32_t q = (int32_t)(kSPiece * lane);
  const uint4 A = lds_entry(lds + kS2Ge, (uint32_t)min(max(pa - q, 0), kS2GeN - 1));
  const uint4 B = lds_entry(lds + kS2Ge, (uint32_t)min(max(pb - q, 0), kS2GeN - 1));
  const uint4 C = lds_entry(lds + kS2Ge, (uint32_t)min(max(pc - q, 0), kS2GeN - 1));
  const uint4 Js = lds_entry(lds + kS2Jsel, min((uint32_t)(pb - q + 3), (uint32_t)(kS2JselN - 1)));
  auto one = [&](uint32_t wj, uint32_t a, uint32_t b, uint32_t c, uint32_t js) {
    const uint32_t keep = __builtin_amdgcn_bitop3_b32(a, b, c, 0xBA);               // (a & ~b) | c
    const uint32_t sel = __builtin_amdgcn_bitop3_b32(keep, 0x03020100u, js, 0xCA);  // keep ? identity : js
    return __builtin_amdgcn_perm(J, wj, sel);
  };
  x[0] = one(w[0], A.x, B.x, C.x, Js.x);
  x[1] = one(w[1], A.y, B.y, C.y, Js.y);
  x[2] = one(w[2], A.z, B.z, C.z, Js.z);
  x[3] = one(w[3], A.w, B.w, C.w, Js.w);
}
// a split operator of the byte tables (kS2Kop): 4 lookups
__device__ __forceinline__ uint32_t apply_op_b(const uint32_t* __restrict__ t, uint32_t x) {
  const uint32_t a0 = t[x & 0xffu], a1 = t[256 + ((x >> 8) & 0xffu)];
  const uint32_t a2 = t[512 + ((x >> 16) & 0xffu)], a3 = t[768 + (x >> 24)];
  return xor3(a0, a1, a2) ^ a3;
}

// Verify fragments [f0, f0 + nfr) (one wave) from their stream records (k_chase, kRecUsual), read with scalar loads
// (s_load, counted in lgkmcnt) one fragment ahead. lds: the kS2Image tables. The verdicts collect in a 64-bit mask
// and reach the dense verdict array (fok) every 64 fragments.
//
// Positions are 32-bit and relative to the wave's first chunk. The loop carries little uniform state -- the current
// fragment's record, the next one's (raw: its load is first waited for at the next fragment end, so the fast chunks
// in between hide its latency), the fragment index, the verdict mask and `ev`, the next chunk that needs more than the
// fast chain -- so that the unrolled ring keeps it in SGPRs without spills: a chunk c != ev lies inside the open
// fragment's data (one compare, then the chain). At chunk ev the usual end (kRecUsual, and the next fragment's data
// runs past the chunk) is one gap mask and one close straight from the records; anything else runs the general loop
// over the fragments touching the chunk. (Round 4's loop derived every position from the fragment table per end,
// kept per-fragment fast-range bounds and stale-table clamps: it spilled 57 SGPRs and its fragment end cost ~160 VALU
// + ~150 SALU instructions, SQ counters in profiles/r05_clock.)
// FASTONLY (tools/kbench only): every chunk takes the fast chain (verdicts meaningless).
template <bool FASTONLY = false>
__device__ __forceinline__ void stream_verify(const uint8_t* __restrict__ seg, uint64_t seg_len,
                                              uint8_t* __restrict__ fok, const uint4* __restrict__ srec, uint64_t f0,
                                              uint32_t nfr, const uint32_t* __restrict__ lds, uint32_t lane,
                                              uint64_t* __restrict__ misc, uint32_t* __restrict__ s_rem,
                                              uint32_t wslot, const uint8_t* __restrict__ dummy) {
  constexpr int D = 8;  // chunks in flight per wave (kbench, round 4: 12 within noise of 8, 4 and 6 slower)
  if (nfr == 0) return;
  const uint8_t* tb = reinterpret_cast<const uint8_t*>(lds + kS2SliceOff);
  const uint32_t* s_lop = lds + kS2LopOff;
  const uint32_t* s_kop = lds + kS2KopOff;
  const SliceLane2 sl = slice_lane2(lane);
  const uint4* rd = srec + f0;
  const uint4 r0 = rd[0], r1 = rd[nfr - 1u];
  // the wave's chunks: [cf, cf + nch), absolute chunk indices (the first fragment begins in chunk cf; the last one's J
  // ends in the last)
  const uint32_t cf = r0.y;
  uint64_t c_end = ((uint64_t)r1.x * kSChunk + (r1.w & 1023u) + 4u + kSChunk - 1u) / kSChunk;
  if (c_end > c_safe_bound(seg_len)) c_end = c_safe_bound(seg_len);  // (a table bug: reported below, never silent)
  if (c_end < cf || c_end - cf > (1u << 20)) c_end = cf;               // (ditto: no real wave spans 1 GiB)
  const uint32_t nch = (uint32_t)(c_end - cf);
  struct G32 { int32_t gs, ge; uint32_t J; };  // wave-relative data range, check word
  constexpr int32_t kFar = 0x40000000;
  auto geo = [&](uint4 r) -> G32 {
    return G32{(int32_t)(((r.y - cf) << 10) + ((r.w >> 10) & 1023u)), (int32_t)(((r.x - cf) << 10) + (r.w & 1023u)),
               r.z};
  };
  uint32_t i = 0;   // the current fragment (wave-relative)
  uint4 rc = r0;    // its record
  uint4 rn = rd[1];  // the next fragment's (4 entries of slack after the last: an unconditional load)
  uint32_t ev = 0;  // the next chunk that is not inside the open fragment's data (fragment 0 begins in chunk 0)
  uint32_t H = 0;
  uint64_t okm = 0;            // verdicts of fragments (i & ~63) + j, bit j
  uint32_t bad = 0xffffffffu;  // first failing fragment (wave-relative), found at the flushes
  auto flush = [&](uint32_t from, uint32_t n) {  // verdicts of fragments [from, from + n) (n <= 64)
    if (lane < n) fok[f0 + from + lane] = (uint8_t)((okm >> lane) & 1u);
    const uint64_t fail = ~okm & (n == 64u ? ~0ull : (1ull << n) - 1ull);
    if (fail != 0ull && bad == 0xffffffffu) bad = from + (uint32_t)__builtin_ctzll(fail);
  };
  // the closing fragment's zero test over the masked chunk words x (its data and J end at pb + 4, chunk-relative),
  // its verdict, the next fragment's chain state; then the next fragment becomes current
  // (the closing fragment's bytes end at e = pb + 4, 1 <= e <= kSChunk: lanes < Lfull hold only its bytes; lane Lfull
  // is split at word K = 1..3 of its piece when K3 = K & 3 != 0, else no lane is)
  auto close = [&](const uint32_t (&x)[kSPW], uint32_t Lfull, uint32_t K3) {
    uint32_t cap = 0;
    const uint32_t s8 = chain_piece2<true>(tb, sl, H, x, K3, &cap);
    const uint32_t Lsplit = K3 != 0u ? Lfull : 64u;
    const uint32_t K = K3;
    const bool full = lane < Lfull, split = lane == Lsplit;
    // split lane: its captured state shifted by A_{8(4(4-K)+1008)}; lanes after it: the carried H shifted by
    // A_{8*1024} (table 0); then each lane's share G_l(A_l) = A_{8*16*(63-l)}(A_l), XOR-reduced over the wave
    const uint32_t A = full ? s8 : apply_op_b(s_kop + (split ? K : 0u) * 1024u, split ? cap : H);
    const uint32_t T = wave_scan_z(apply_fwd(s_lop, lane, A), [](uint32_t a, uint32_t b) { return a ^ b; });
    if (__builtin_amdgcn_readlane(T, 63) == 0u) okm |= 1ull << (i & 63u);
    H = s8 ^ A;
    ++i;
    if ((i & 63u) == 0u) {
      flush(i - 64u, 64u);
      okm = 0;
    }
    rc = rn;
    rn = rd[i + 1u];  // (indexed from the wave's base: a pointer carried through the loop became a vector load)
  };
  auto close_pb = [&](const uint32_t (&x)[kSPW], int32_t pb) {
    const uint32_t e = (uint32_t)(pb + 4), K = ((e % kSPiece) + 3u) >> 2;
    close(x, e / kSPiece + (K == (uint32_t)kSPW ? 1u : 0u), K & 3u);
  };
  // chunk c == ev: the fragment ends (and beginnings) inside it, one close per end; then the next `ev`
  auto slow = [&](uint32_t c, const uint32_t (&w)[kSPW]) {
    const int32_t C0 = (int32_t)(c * kSChunk), C1 = C0 + kSChunk;
    uint32_t nev;
    // (evaluated without short-circuits: a value computed on one path only became an SGPR phi whose undefined side the
    // compiler filled with a readfirstlane of a ring register, waiting for that chunk's load)
    // (ev is also the chunk a fragment begins in when it was not open: the wave's first one, or one after a header
    // straddling two chunks)
    const bool usual = ((rc.w & kRecUsual) != 0u) & (rc.x - cf == c) & (rn.x - cf > c) & (i + 1u < nfr);
    if (usual) {
      uint32_t x[kSPW];
      mask_gap(x, w, (int32_t)(rc.w & 1023u), rc.z, lane, lds);
      close(x, (rc.w >> 22) & 127u, rc.w >> 29);
      nev = rc.x - cf;  // the next fragment (now current, open) ends in a later chunk
    } else {
      auto rel = [&](int32_t p) -> int32_t { return min(max(p - C0, -64), 4096); };
      G32 fc = i < nfr ? geo(rc) : G32{kFar, kFar, 0u};
      for (;;) {
        if (fc.gs >= C1) break;  // not begun here (also once every fragment is done: fc.gs = kFar)
        const G32 fn = i + 1u < nfr ? geo(rn) : G32{kFar, kFar, 0u};
        const bool closes = fc.ge + 4 <= C1;
        // the next fragment shares the chain when its data runs to the chunk's end (bytes [gs, C1) all data, no J)
        const bool next_in = closes && fn.gs < C1 && fn.ge >= C1;
        uint32_t x[kSPW];
        const int32_t pa = rel(fc.gs), pb = rel(fc.ge);
        if (next_in && pa <= 0 && fn.gs - fc.ge == (int32_t)kHdr)  // a header between two data runs
          mask_gap(x, w, pb, fc.J, lane, lds);
        else
          mask_chunk(x, w, pa, pb, next_in ? rel(fn.gs) : 4096, fc.J, lane, lds);
        if (!closes) {  // the data (or J) runs on into the next chunk
          H = chain_piece2<false>(tb, sl, H, x);
          break;
        }
        close_pb(x, pb);
        fc = fn;
        if (next_in) break;
      }
      // open: fc's bytes so far are in H; its data ends in chunk fc.ge / kSChunk (its J may straddle into the next)
      nev = fc.gs < C1 ? max((uint32_t)fc.ge / (uint32_t)kSChunk, c + 1u) : c + 1u;
    }
    ev = nev;
  };
  auto step = [&](uint32_t c, const uint32_t (&w)[kSPW]) {
    if (FASTONLY || c != ev) H = chain_piece2<false>(tb, sl, H, w);
    else slow(c, w);
  };
  const uint64_t c_safe = seg_len / kSChunk;  // chunks [0, c_safe) lie inside the segment
  const uint32_t nl = c_safe > cf ? (uint32_t)min(c_safe - cf, (uint64_t)nch) : 0u;  // pipelined chunks
  if (nl > 0u) {
    const uint8_t* wseg = seg + (uint64_t)cf * kSChunk;
    const uint32_t lane16 = lane * kSPiece;
    // The ring of D chunk loads is issued and waited for by hand: the compiler's in-order vmcnt accounting, at every
    // fragment end, either drained the whole ring or waited for the newest chunk (an undefined SGPR phi filled by a
    // readfirstlane of a ring register). Each slot waits with vmcnt(D - 1): the D - 1 later chunks' loads (a verdict
    // store in between only makes that wait longer, never short). Every ring register stays live until the final
    // vmcnt(0), so none is reused while a load into it is in flight.
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    v4u buf[D];
    // unconditional (no branch around a load); the loads issued past the last chunk read 1 KiB of the table image
    // instead, which every workgroup has just read (an L2 hit). Non-temporal: the segment is read once (kbench spat:
    // 185 -> 160 us for the whole segment).
    auto issue = [&](uint32_t c, v4u& w) {
      const uint8_t* p = c < nl ? wseg + (size_t)c * kSChunk : dummy;  // uniform: the lane offset is the VGPR part
      asm volatile("global_load_dwordx4 %0, %1, %2 nt" : "=v"(w) : "v"(lane16), "s"(p) : "memory");
    };
#pragma unroll
    for (int k = 0; k < D; ++k) issue((uint32_t)k, buf[k]);
    for (uint32_t c = 0; c < nl; c += D) {
      // issue-priority balancing: a SIMD's issue arbiter serves its oldest wave first, so with equal shares the four
      // waves of a SIMD finished up to 50 us apart and the last of them streamed alone. Each wave publishes its
      // chunks left (s_rem[simd][age]) and runs at priority 2 while it has (nearly) the most left on its SIMD.
      const uint32_t left = nl - c;
      if (lane == 0) s_rem[wslot] = left;
      const uint4 r = *reinterpret_cast<const uint4*>(s_rem + (wslot & ~3u));
      const uint32_t mx = max(max(r.x, r.y), max(r.z, r.w));
      if (left + (uint32_t)D >= mx) __builtin_amdgcn_s_setprio(2);
      else __builtin_amdgcn_s_setprio(0);
#pragma unroll
      for (int k = 0; k < D; ++k) {
        // chunk c + k, then its register takes chunk c + k + D
        if (c + k < nl) {
          asm volatile("s_waitcnt vmcnt(%1)" : "+v"(buf[k]) : "n"(D - 1));
          const uint32_t w[kSPW] = {buf[k].x, buf[k].y, buf[k].z, buf[k].w};
          step(c + k, w);
        }
        issue(c + k + D, buf[k]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(buf[0]), "v"(buf[1]), "v"(buf[2]), "v"(buf[3]), "v"(buf[4]), "v"(buf[5]),
                 "v"(buf[6]), "v"(buf[7]));
    static_assert(D == 8, "the final wait names every ring register");
  }
  for (uint32_t c = nl; c < nch; ++c) {  // chunks touching the segment's end
    uint32_t w[kSPW];
    const uint4 A = load16_safe(seg, seg_len, (int64_t)(((uint64_t)cf + c) * kSChunk) + lane * kSPiece);
    w[0] = A.x; w[1] = A.y; w[2] = A.z; w[3] = A.w;
    step(c, w);
  }
  flush(i & ~63u, i & 63u);
  if (FASTONLY && H == 0x9e3779b9u) misc[7] = H;  // (kbench: keep the chains alive)
  if (lane == 0) {
    if (bad != 0xffffffffu)
      atomicMin(reinterpret_cast<unsigned long long*>(&misc[M_BAD_CRC]), (unsigned long long)(f0 + bad));
    // every fragment of the wave is closed by its chunks; one that is not means the fragment table and the chunk range
    // disagree (a bug): report the decode as failed (BCW_ERR_INTERNAL) instead of passing the fragment unverified
    if (!FASTONLY && i < nfr) atomicMax(reinterpret_cast<unsigned long long*>(&misc[M_ABORT]), 20ull);
  }
}

// The arguments of k_crc's record emission and completion, parked in LDS during the CRC pass: kept in SGPRs they
// would be live across the whole stream loop (the kernel spilled 58 SGPRs, and kept uniform loop state in VGPRs).
struct CrcTail {
  EmitArgs ea;
  bcw_decode_result* res;
  uint64_t* misc;
  uint64_t nblocks, frag_cap, gen, cb0, cb1;
  uint32_t tail_panic, nwg_total;
};

// The next decode's split (XBal), by the last wave of k_crc: every workgroup's stream times are in (the completion
// counter orders them). Class y's mean stream time T_y against the mean over the classes T: its range weight moves
// half way to w_y T / T_y (kept within 0.8-1.25 of equal), when k_chase used the weights: a fresh context converges
// within the driver's warmup decodes. The times are reset for the next launch.
struct XBalIn {  // class y = lane % 8: its summed stream times, their count, its weight; whether k_chase used them
  uint64_t t, n;
  uint32_t w, on;
};
// (requested before the finalize's loads, so that the two round trips overlap)
__device__ __forceinline__ XBalIn xbal_load(const XBal* __restrict__ xb, uint32_t lane) {
  const uint32_t y = lane & 7u;
  XBalIn v;
  v.t = __hip_atomic_load(&xb->t[y], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  v.n = __hip_atomic_load(&xb->n[y], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  v.w = xb->w[y];
  v.on = xb->on;
  return v;
}
__device__ __forceinline__ void xbal_update(XBal* __restrict__ xb, uint32_t lane, const XBalIn& in) {
  const uint32_t y = lane & 7u;
  const uint64_t t = in.t, n = in.n;
  const float Ty = n && t ? (float)t / (float)n : 0.0f;
  const bool all = __ballot(lane < 8u && Ty > 0.0f) == 0xffull && in.on != 0u;  // every XCD measured
  float sT = lane < 8u ? Ty : 0.0f;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) sT += __shfl_xor(sT, d, 64);
  if (lane < 8u) {
    if (all) {
      const float wy = (float)in.w * (1.0f + 0.5f * ((sT / 8.0f) / Ty - 1.0f));
      const float d = fminf(fmaxf(rintf((wy - 65536.0f) / 256.0f), -51.0f), 64.0f);  // (k_chase's ClassW: 256 steps)
      xb->w[y] = (uint32_t)(65536 + 256 * (int32_t)d);
    }
    xb->t[y] = 0;
    xb->n[y] = 0;
  }
}

// k_crc: one 1024-thread workgroup per CU. Each wave verifies the fragments of its share of the blocks (stream_verify),
// then takes record-emission items of its workgroup's blocks (emit_chunks); the last wave of the last workgroup
// writes the segment result (finalize).
// ABL: tools/kbench ablations (0 in the product): 8 no emission, 32768 no CRC pass (the emission alone), 8388608 every
// chunk on the fast chain (stream_verify<true>), 4096 emission without the row stores
template <int ABL = 0>
__global__ __launch_bounds__(kCrcThreads) void k_crc(const uint8_t* __restrict__ seg, uint64_t seg_len,
                                                     uint32_t start_off, uint64_t nblocks,
                                                     const uint32_t* __restrict__ fbase, uint8_t* __restrict__ fok,
                                                     const uint4* __restrict__ srec,
                                                     uint64_t frag_cap, Tables tabs, EmitArgs ea,
                                                     uint32_t tail_panic, uint64_t gen,
                                                     bcw_decode_result* __restrict__ res,
                                                     uint64_t* __restrict__ misc, uint64_t cb0, uint64_t cb1,
                                                     uint32_t nwg_total, const uint32_t* __restrict__ wstart,
                                                     XBal* __restrict__ xb) {
  // [cb0, cb1): the blocks this launch emits (the whole segment); nwg_total: the workgroups that count towards
  // completion; wstart: each wave's first fragment (k_chase, gridDim.x x kCrcWaves + 1 entries)
  __shared__ __attribute__((aligned(16))) uint32_t lds[kS2Image];
  __shared__ CrcTail s_tail;
  __shared__ uint32_t s_wdone;  // waves of this workgroup done
  __shared__ uint32_t s_eq;     // the workgroup's emission items taken
  __shared__ __attribute__((aligned(16))) uint32_t s_rem[kCrcWaves];  // chunks left per wave [simd][age] (stream_verify)
  __shared__ uint32_t s_sdone;              // waves of this workgroup whose stream is done
  __shared__ unsigned long long s_tsum;     // their summed stream times
  __shared__ uint64_t s_t0;                 // the workgroup's start (wall_clock64)
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid < (uint32_t)kCrcWaves) s_rem[tid] = 0;
  if (ea.kb_stamps && lane == 0) {  // (kbench: the in-kernel clock = shader cycles / real time between entry and end)
    uint64_t* q = ea.kb_stamps + 8 * ((uint64_t)blockIdx.x * kCrcWaves + wave);
    q[4] = wall_clock64();
    q[5] = __builtin_amdgcn_s_memtime();
    // the XCC (HW_REG_XCC_ID, 20) and HW_ID (4: wave / SIMD / CU / SH / SE) this wave runs on
    q[7] = ((uint64_t)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32) | __builtin_amdgcn_s_getreg(4 | (31 << 11));
  }
  if (tid == 0) {
    s_wdone = 0;
    s_eq = 0;
    s_sdone = 0;
    s_tsum = 0;
    s_t0 = wall_clock64();
    s_tail = CrcTail{ea, res, misc, nblocks, frag_cap, gen, cb0, cb1, tail_panic, nwg_total};
  }
  {  // table image -> LDS, all loads in flight before the first store. The slice rows hold every table dword 8 times
     // (the bank-conflict-free copies, kS2Image): their 8 KiB of distinct dwords are read and replicated here, the
     // rest copied as it is -- 57 of the image's 113 KiB read per workgroup
    const uint4* src4 = reinterpret_cast<const uint4*>(tabs.lds_image2);
    uint4* dst4 = reinterpret_cast<uint4*>(lds);
    constexpr uint32_t kLop4 = kS2SliceOff / 4, kKop4 = kS2KopOff / 4, kEnd4 = kS2Image / 4;
    constexpr uint32_t kN4 = kLop4 + (kEnd4 - kKop4);  // uint4s copied as they are
    constexpr int kPer = (int)((kN4 + kCrcThreads - 1) / kCrcThreads);
    static_assert(kS2Slice == 256 * 64 && kCrcThreads * 2 == 256 * 8, "slice rows: 256 x 8 distinct dwords");
    auto at = [](uint32_t i) { return i < kLop4 ? i : i - kLop4 + kKop4; };
    uint4 v[kPer];
#pragma unroll
    for (int k2 = 0; k2 < kPer; ++k2) {
      const uint32_t i = tid + k2 * kCrcThreads;
      v[k2] = i < kN4 ? src4[at(i)] : make_uint4(0, 0, 0, 0);
    }
    const uint32_t* src1 = tabs.lds_image2 + kS2SliceOff;
    uint32_t sv[2];
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {  // row e = t / 8, distinct dword t % 8 (its 8 copies are consecutive)
      const uint32_t t = tid + k2 * kCrcThreads;
      sv[k2] = src1[(t >> 3) * 64u + (t & 7u) * 8u];
    }
#pragma unroll
    for (int k2 = 0; k2 < kPer; ++k2) {
      const uint32_t i = tid + k2 * kCrcThreads;
      if (i < kN4) dst4[at(i)] = v[k2];
    }
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const uint32_t t = tid + k2 * kCrcThreads;
      uint4* d = reinterpret_cast<uint4*>(lds + kS2SliceOff + (t >> 3) * 64u + (t & 7u) * 8u);
      d[0] = make_uint4(sv[k2], sv[k2], sv[k2], sv[k2]);
      d[1] = make_uint4(sv[k2], sv[k2], sv[k2], sv[k2]);
    }
  }
  __syncthreads();
  // every wave streams the fragments of its share of the segment's bytes: 1 / (16 x CUs), weighted by its
  // workgroup's class (XBal; k_chase's wstart; dedicated emission waves measured slower)
  const uint64_t gw = (uint64_t)blockIdx.x * kCrcWaves + wave;
  const uint64_t f0 = wstart[gw];
  uint64_t f1 = wstart[gw + 1];
  if (f1 > frag_cap) f1 = frag_cap;
  if (f0 > f1) f1 = f0;
  // a k_chase wait gave up (Spin): the bases are unreliable, so no fragment is read and no row written
  const bool aborted = __builtin_amdgcn_readfirstlane(
                           (uint32_t)__hip_atomic_load(&misc[M_ABORT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0u;
  if (aborted) f1 = f0;
  if (blockIdx.x == 0 && tid == 0) misc[M_T_CRC0] = wall_clock64();
  const uint32_t nfr = f1 > f0 ? (uint32_t)(f1 - f0) : 0u;
  // ---- record emission: the workgroup's work items (those starting in its blocks), taken from an LDS counter by
  // its waves as they finish their CRC streams (ItemMeta). The next item is taken and its block data requested while
  // this item's fragment descriptors are in flight, so an item costs two dependent round trips (descriptors, record
  // prefixes). The arguments are reloaded from LDS (CrcTail). (One item per wave part of the way through its stream,
  // staggered by wave, measured slower: 261-271 vs 209 us on B.)
  uint64_t n_items = 0;
  auto emit_items = [&](uint64_t max_items) {
    asm volatile("" ::: "memory");
    CrcTail T;
    {  // wave-uniform: into SGPRs
      static_assert(sizeof(CrcTail) % 4 == 0, "CrcTail words");
      const uint32_t* src = reinterpret_cast<const uint32_t*>(&s_tail);
      uint32_t* dst = reinterpret_cast<uint32_t*>(&T);
#pragma unroll
      for (int k = 0; k < (int)(sizeof(CrcTail) / 4); ++k) dst[k] = __builtin_amdgcn_readfirstlane(src[k]);
    }
    const EmitArgs& A = T.ea;
    if ((ABL & 8) || (A.kb_flags & 1u) ||
        __builtin_amdgcn_readfirstlane(
            (uint32_t)__hip_atomic_load(&T.misc[M_ABORT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0u)
      return;
    const uint64_t cb0t = T.cb0, cb1t = T.cb1, fcap = T.frag_cap;
    // blocks per item for ~64 fragments each, and this workgroup's items. 32-bit arithmetic: a segment in HBM has
    // fewer than 2^24 blocks (512 GiB; bcw_decode_segment_async refuses more), and the 64-bit divisions' VGPR
    // temporaries were spilled to scratch across the item loop.
    const uint32_t cnt = (uint32_t)(cb1t - cb0t), G = gridDim.x, wg = blockIdx.x;
    const uint64_t fc0 = A.fbase[cb0t], fc1 = A.fbase[cb1t];
    const uint32_t nf_all = (uint32_t)(fc1 > fc0 ? (fc1 - fc0 < fcap ? fc1 - fc0 : fcap) : 0);
    uint32_t bpw = nf_all ? (64u * cnt) / nf_all : cnt;
    if (bpw < 1u) bpw = 1u;
    bpw = __builtin_amdgcn_readfirstlane(bpw);  // (uniform values the division left in VGPRs: into SGPRs)
    const uint32_t cq = cnt / G, cr = cnt % G;  // B(w) = cnt * w / G without a 64-bit product
    const uint32_t B0 = cq * wg + (cr * wg) / G, B1 = cq * (wg + 1u) + (cr * (wg + 1u)) / G;  // chunk-relative
    const uint64_t i0 = __builtin_amdgcn_readfirstlane((B0 + bpw - 1u) / bpw),
                   nitems = __builtin_amdgcn_readfirstlane((B1 + bpw - 1u) / bpw);
    auto deq = [&]() -> uint64_t {
      uint32_t j = 0;
      if (lane == 0) j = atomicAdd(&s_eq, 1u);
      j = __builtin_amdgcn_readfirstlane(j);
      return i0 + j;
    };
    uint64_t taken = 0;
    uint64_t it = deq();
    ItemMeta m = item_meta(A, it, bpw, cb0t, cb1t, lane);
    while (it < nitems) {
      ++taken;
      const EmitState es = emit_state(A, m.bb, lane, m.s, m.rec);
      const uint64_t mf1 = m.f1 < fcap ? m.f1 : fcap;
      uint64_t nx = ~0ull;
      ItemMeta mn = m;
      emit_chunks<(ABL & 4096) != 0, (ABL & 131072) != 0>(A, es, m.f0, mf1, lane, [&]() {
        if (taken < max_items) {
          nx = deq();
          mn = item_meta(A, nx, bpw, cb0t, cb1t, lane);
        }
      });
      it = nx;
      m = mn;
    }
    n_items += taken;
  };
  if (ABL & 64) emit_items(~0ull);  // (kbench: emission before the stream)
  if (ABL & 16384) {  // (kbench: the wave's range as 4 consecutive stream_verify calls: the cost of a ring restart)
    for (uint32_t q = 0; q < 4u; ++q) {
      const uint32_t a = nfr * q / 4u, b = nfr * (q + 1u) / 4u;
      stream_verify<(ABL & 8388608) != 0>(seg, seg_len, fok, srec, f0 + a, b - a, lds, lane, misc, s_rem,
                                          (wave & 3u) * 4u + (wave >> 2),
                                          reinterpret_cast<const uint8_t*>(tabs.lds_image2));
    }
  } else if (!(ABL & 32768))
    stream_verify<(ABL & 8388608) != 0>(seg, seg_len, fok, srec, f0, nfr, lds, lane, misc, s_rem,
                                        (wave & 3u) * 4u + (wave >> 2),
                                        reinterpret_cast<const uint8_t*>(tabs.lds_image2));
  __builtin_amdgcn_s_setprio(0);
  if (lane == 0) {  // this wave's stream time; the workgroup's last stream adds its workgroup's to its class's (XBal)
    atomicAdd(&s_tsum, (unsigned long long)(wall_clock64() - s_t0));
    if (atomicAdd(&s_sdone, 1u) == kCrcWaves - 1u) {
      const uint32_t c = blockIdx.x & 7u;
      __hip_atomic_fetch_add(&xb->t[c], (uint64_t)s_tsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&xb->n[c], (uint64_t)kCrcWaves, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (ea.kb_stamps && lane == 0) {  // (kbench: this wave's CRC end and fragments, written now so that nothing of it
                                   // stays live across the emission)
    uint64_t* q = ea.kb_stamps + 8 * ((uint64_t)blockIdx.x * kCrcWaves + wave);
    q[0] = wall_clock64();
    q[3] = nfr;
  }
  if (!(ABL & 64)) emit_items(~0ull);
  asm volatile("" ::: "memory");  // (reload the tail arguments from LDS, see CrcTail)
  CrcTail T;
  {  // wave-uniform: into SGPRs
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&s_tail);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&T);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(CrcTail) / 4); ++k) dst[k] = __builtin_amdgcn_readfirstlane(src[k]);
  }
  const EmitArgs& A = T.ea;
  if (A.kb_stamps && lane == 0) {
    uint64_t* q = A.kb_stamps + 8 * ((uint64_t)__builtin_amdgcn_workgroup_id_x() * kCrcWaves + wave);
    q[1] = wall_clock64(); q[2] = n_items;
    q[6] = __builtin_amdgcn_s_memtime();
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
    gorder = __hip_atomic_fetch_add(&T.misc[M_DONE_CRC], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  gorder = (uint64_t)__shfl((long long)gorder, 0, 64);
  if (gorder != T.nwg_total - 1u) return;
  if (lane == 0) T.misc[M_T_FIN] = wall_clock64();
  const XBalIn xin = xbal_load(xb, lane);
  finalize(A, T.nblocks, T.frag_cap, T.tail_panic, T.gen, T.res, lane);
  xbal_update(xb, lane, xin);
}

__global__ void k_export_frags(const Frag* __restrict__ frags, const uint8_t* __restrict__ fok,
                               const uint64_t* __restrict__ misc, uint64_t cap,
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
  out.crc_ok[g] = fok[g];
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
  // k_chase's grid padded to a multiple of 8 workgroups (the extra ones return at once) and k_crc's one per CU: the
  // dispatcher then starts every k_crc on the same XCD, so each workgroup class (blockIdx % 8, XBal) keeps its XCD
  // from decode to decode
  const uint32_t nb_grid = (uint32_t)(((nblocks + 63) / 64 + 7) / 8 * 8);
  const EmitArgs ea{d_seg, p.seg_len, p, s.frags, s.fbase, s.rbase, s.bsum, t, s.misc, 0u, nullptr};
  pr.begin(K_CHASE, stream, ev);
  k_chase<0><<<nb_grid, 64, 0, stream>>>(d_seg, p.seg_len, p.start_off, nblocks, s.fbase, s.rbase, s.bsum, s.frags,
                                        s.srec, s.frag_cap, s.lb, s.lbe, s.misc, s.epoch, tabs.initc, s.chase_direct,
                                        s.test_abort_wg, s.wstart, (uint32_t)num_cus * kCrcWaves, s.xbal, s.xbal_on);
  s.test_abort_wg = 0;
  pr.end(K_CHASE, stream, ev);
  if ((++s.epoch & 0xffffffull) == 0) {  // 24-bit look-back epochs: clear the words before reuse
    (void)hipMemsetAsync(s.lb, 0, s.nlb * sizeof(uint64_t), stream);
    (void)hipMemsetAsync(s.lbe, 0, s.nlb * sizeof(uint64_t), stream);
    s.epoch = 1;
  }
  pr.begin(K_CRC, stream, ev);
  k_crc<0><<<(uint32_t)num_cus, kCrcThreads, 0, stream>>>(d_seg, p.seg_len, p.start_off, nblocks, s.fbase, s.fok,
                                                         s.srec, s.frag_cap, tabs, ea,
                                                         tail_panic, gen, d_result, s.misc, 0ull, nblocks,
                                                         (uint32_t)num_cus, s.wstart, s.xbal);
  pr.end(K_CRC, stream, ev);
  return hipGetLastError();
}

hipError_t launch_export_frags(const Scratch& s, const bcw_frag_table& out, uint32_t start_off, hipStream_t stream,
                               uint64_t n, const uint32_t* initc) {
  if (n == 0) return hipSuccess;
  k_export_frags<<<(uint32_t)((n + 255) / 256), 256, 0, stream>>>(s.frags, s.fok, s.misc, s.frag_cap, start_off, out,
                                                                    initc);
  return hipGetLastError();
}

}  // namespace bcw
