// k_crc ablation harness (not product code): one TU with the codec sources, times the full decode
// pipeline and k_crc variants on a synthetic 1 GiB config-B segment.
#include "../../bitcaskdb_amd/csrc/bcw_api.cpp"
#include "../../bitcaskdb_amd/csrc/bcw_decode.hip"
#include "../../bitcaskdb_amd/csrc/bcw_encode.hip"
#include "../../bitcaskdb_amd/csrc/bcw_index.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x) do { auto e_ = (x); if (e_ != hipSuccess && e_ != 0) { fprintf(stderr, "%s:%d err %d\n", __FILE__, __LINE__, (int)e_); exit(1);} } while (0)

// quad-coalesced window loads + DPP transpose (moved here from k_crc, which no longer uses them)
namespace bcw {
// Quad-coalesced window loads. Loading each lane's own 128 B window (lane l: 8 x 16 B at its
// window) touches 64 windows per load instruction and streams at ~60% of HBM; instead load g
// (g = 4*p2 + 2*w1 + w0) gives the 4 lanes of quad a the 16 B pieces 4*p2 .. 4*p2+3 of window
// 4a + (g & 3): 64 contiguous bytes per quad. Two lane-bit <-> register-bit exchanges (DPP
// quad_perm) then leave piece p of window W in w[4p..4p+3] of lane W.
template <int K>
__device__ __forceinline__ void kb_swap_lane_reg_bit(uint32_t (&w)[32], uint32_t lane) {
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
__device__ __forceinline__ void quad_windows_transpose(uint32_t (&w)[32], uint32_t lane) {
  kb_swap_lane_reg_bit<0>(w, lane);
  kb_swap_lane_reg_bit<1>(w, lane);
}
// loads of the quad layout; woff/act: this lane's window offset (from wbase) and active flag;
// SAFE: bounds-checked 16 B loads (windows touching the segment's ends)
template <bool SAFE>
__device__ __forceinline__ void load_windows_quad(const uint8_t* __restrict__ seg, uint64_t seg_len, int64_t wbase,
                                                  uint32_t woff, bool act, uint32_t lane, uint32_t (&w)[32]) {
  uint32_t wo[4], ac[4];
  const uint32_t a = act ? 1u : 0u;
  wo[0] = dpp_mov<0x00>(woff); wo[1] = dpp_mov<0x55>(woff); wo[2] = dpp_mov<0xAA>(woff); wo[3] = dpp_mov<0xFF>(woff);
  ac[0] = dpp_mov<0x00>(a); ac[1] = dpp_mov<0x55>(a); ac[2] = dpp_mov<0xAA>(a); ac[3] = dpp_mov<0xFF>(a);
  const uint32_t q = 16u * (lane & 3u);
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    if (ac[g & 3]) {
      const uint32_t o = wo[g & 3] + 64u * (g >> 2) + q;
      const uint4 v = SAFE ? bcw::load16_safe(seg, seg_len, wbase + (int64_t)o)
                           : *reinterpret_cast<const uint4*>(seg + wbase + o);
      w[4 * g + 0] = v.x; w[4 * g + 1] = v.y; w[4 * g + 2] = v.z; w[4 * g + 3] = v.w;
    }
  }
}

}  // namespace bcw

// HBM stream-read reference: sum of every 16 B word of the segment
__global__ __launch_bounds__(256) void k_stream(const uint4* __restrict__ p, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// access-pattern probe: each wave reads consecutive 8 KiB pieces = 64 windows x 8 pieces of 16 B;
// G lanes share a window per instruction (G=1: window per lane, G=8: 1 KiB contiguous per instruction)
template <int G, bool REGION = false>
__global__ __launch_bounds__(1024) void k_pattern(const uint8_t* __restrict__ p, uint64_t n, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = (uint64_t)gridDim.x * 16, w0 = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint64_t npiece = n / 8192;
  const uint64_t per = npiece / nw;  // REGION: wave w0 reads pieces [w0*per, (w0+1)*per) in order
  constexpr int S = 64 / G, PG = 8 / G;
  uint32_t acc = 0;
  uint4 v[8];
  for (uint64_t it = 0; it < (REGION ? per : (npiece - w0 + nw - 1) / nw); ++it) {
    const uint64_t q = REGION ? w0 * per + it : w0 + it * nw;
    const uint8_t* b = p + q * 8192;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const uint32_t win = lane / G + S * (g / PG), piece = G * (g % PG) + lane % G;
      v[g] = *reinterpret_cast<const uint4*>(b + 128 * win + 16 * piece);
    }
#pragma unroll
    for (int g = 0; g < 8; ++g) acc ^= v[g].x ^ v[g].y ^ v[g].z ^ v[g].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// core probe: the k_crc pass loop stripped to quad loads (1 pass ahead) + transpose + CRC chain of
// every 128 B window of a contiguous per-wave region; no fragments, descriptors or combine.
// MODE bit 0: skip transpose, bit 1: lane-window (G1) loads instead of quad loads, bit 2: no loads
// (registers seeded from the lane), bit 3: no chain (all 32 words folded with xor)
template <int MODE>
__global__ __launch_bounds__(1024) void k_core(const uint8_t* __restrict__ p, uint64_t n, const uint32_t* img,
                                                uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsImage];
  for (uint32_t i = threadIdx.x; i < (uint32_t)kLdsImage; i += 1024) lds[i] = img[i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, lb = (lane & 31u) * 4u;
  const bcw::SliceLane sl = bcw::slice_lane(lane);
  const uint64_t nw = (uint64_t)gridDim.x * 16, w0 = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint64_t per = n / 8192 / nw;
  const uint8_t* base = p + w0 * per * 8192;
  uint32_t wx[32], wy[32], acc = 0;
  auto issue = [&](uint64_t it, uint32_t (&w)[32]) {
    if (it >= per) return;
    if (MODE & 4) {
#pragma unroll
      for (int k = 0; k < 32; ++k) w[k] = (uint32_t)(it * 2654435761u) ^ (lane * 40503u + k);
      return;
    }
    const uint8_t* b = base + it * 8192;
    if (MODE & 2) {
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        const uint4 v = *reinterpret_cast<const uint4*>(b + 128 * lane + 16 * g);
        w[4 * g] = v.x; w[4 * g + 1] = v.y; w[4 * g + 2] = v.z; w[4 * g + 3] = v.w;
      }
    } else {
      bcw::load_windows_quad<false>(b, ~0ull, 0, 128u * lane, true, lane, w);
    }
  };
  issue(0, wx);
  for (uint64_t it = 0; it < per; ++it) {
    issue(it + 1, wy);
    if (!(MODE & 3)) bcw::quad_windows_transpose(wx, lane);
    if (MODE & 8) {
#pragma unroll
      for (int k = 0; k < 32; ++k) acc ^= wx[k];
    } else {
      acc ^= bcw::crc_window(lds, lds + kLdsSlice + kLdsFwd + 128, sl, acc, wx);
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) wx[k] = wy[k];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// prefetch-depth probe: WAVES waves per CU, loads DEPTH passes ahead (DEPTH+1 window buffers), chain
template <int WAVES, int DEPTH, bool QUAD, int ROT = 0, bool CHAIN = true>
__global__ __launch_bounds__(WAVES * 64) void k_depth(const uint8_t* __restrict__ p, uint64_t n, const uint32_t* img,
                                                       uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsImage];
  for (uint32_t i = threadIdx.x; i < (uint32_t)kLdsImage; i += WAVES * 64) lds[i] = img[i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, lb = (lane & 31u) * 4u;
  const bcw::SliceLane sl = bcw::slice_lane(lane);
  const uint64_t nw = (uint64_t)gridDim.x * WAVES, w0 = (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
  const uint64_t per = n / 8192 / nw;
  const uint8_t* base = p + w0 * per * 8192;
  uint32_t w[DEPTH + 1][32], acc = 0;
  auto issue = [&](uint64_t it, uint32_t (&b)[32]) {
    if (it >= per) return;
    const uint8_t* q = base + ((it + (ROT ? w0 * ROT : 0)) % per) * 8192;
    if (QUAD) {
      bcw::load_windows_quad<false>(q, ~0ull, 0, 128u * lane, true, lane, b);
    } else {
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        const uint4 v = *reinterpret_cast<const uint4*>(q + 128 * lane + 16 * g);
        b[4 * g] = v.x; b[4 * g + 1] = v.y; b[4 * g + 2] = v.z; b[4 * g + 3] = v.w;
      }
    }
  };
#pragma unroll
  for (int k = 0; k < DEPTH; ++k) issue(k, w[k]);
  for (uint64_t it = 0; it < per; ++it) {
    issue(it + DEPTH, w[DEPTH]);
    if (QUAD) bcw::quad_windows_transpose(w[0], lane);
    if (CHAIN) {
      acc ^= bcw::crc_window(lds, lds + kLdsSlice + kLdsFwd + 128, sl, acc, w[0]);
    } else {
#pragma unroll
      for (int k = 0; k < 32; ++k) acc ^= w[0][k];
    }
#pragma unroll
    for (int b = 0; b < DEPTH; ++b)
#pragma unroll
      for (int k = 0; k < 32; ++k) w[b][k] = w[b + 1][k];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <typename F>
static float timeit(F f, int reps, hipStream_t st) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  f();
  hipStreamSynchronize(st);
  hipEventRecord(a, st);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b, st);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main(int argc, char** argv) {
  const uint64_t target = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 30);
  const int mode = argc > 2 ? atoi(argv[2]) : 0;
  bcw_ctx* ctx;
  CK(bcw_ctx_create(0, &ctx));
  uint64_t n, r;
  CK(bcw_synth_segment(target, 0, 42, 20, 100, 4096, mode, 1700000000, nullptr, 0, &n, &r));
  std::vector<uint8_t> h(n);
  CK(bcw_synth_segment(target, 0, 42, 20, 100, 4096, mode, 1700000000, h.data(), n, &n, &r));
  uint8_t* d;
  if (getenv("KB_CONTIG")) CK(hipExtMallocWithFlags((void**)&d, n, hipDeviceMallocContiguous));  // physically contiguous
  else CK(hipMalloc(&d, n));
  CK(hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice));
  bcw_record_table t{};
  void* mem;
  const uint64_t cap = r + 64;
  CK(hipMalloc(&mem, cap * 64));
  uint8_t* m = (uint8_t*)mem;
  t.capacity = cap;
  t.foff = (uint64_t*)m; m += cap * 8; t.size = (uint64_t*)m; m += cap * 8; t.expire = (uint64_t*)m; m += cap * 8;
  t.aux0 = (uint64_t*)m; m += cap * 8; t.aux1 = (uint64_t*)m; m += cap * 8;
  t.key_len = (uint32_t*)m; m += cap * 4; t.val_len = (uint32_t*)m; m += cap * 4; t.meta_len = (uint32_t*)m; m += cap * 4;
  t.first_frag = (uint32_t*)m; m += cap * 4; t.emit_frag = (uint32_t*)m; m += cap * 4;
  t.hdr_size = m; m += cap; t.flags = m; m += cap; t.etag_off = m; m += cap; t.status = m;
  bcw_decode_result* dres;
  CK(hipMalloc(&dres, sizeof(bcw_decode_result)));
  bcw_decode_params p{n, 1700000000, 40, 20, 20, 0};
  hipStream_t st = (hipStream_t)bcw_ctx_stream(ctx);
  CK(bcw_decode_segment_async(ctx, d, &p, &t, dres));
  CK(hipStreamSynchronize((hipStream_t)bcw_ctx_stream(ctx)));
  bcw_decode_result res;
  CK(hipMemcpy(&res, dres, sizeof res, hipMemcpyDeviceToHost));
  printf("seg %lu B, %lu records, decode: n_records=%lu err=%d frags=%lu bad=%d\n", n, r, res.n_records, res.err_class,
         res.n_frags, res.first_bad_record);
  const int reps = 20;
  float full = timeit([&] { bcw_decode_segment_async(ctx, d, &p, &t, dres); }, reps, st);
  printf("full pipeline   %.4f ms  %.1f GB/s\n", full, n / (full * 1e-3) / 1e9);
  bcw_ctx_set_profiling(ctx, -1);
  for (int i = 0; i < reps; ++i) bcw_decode_segment_async(ctx, d, &p, &t, dres);
  double tot[16]; uint64_t cnt[16];
  const int nk = bcw_ctx_kernel_times(ctx, tot, cnt, 16);
  bcw_ctx_set_profiling(ctx, 0);
  for (int k = 0; k < nk; ++k) printf("  %-14s %.4f ms\n", bcw_kernel_name(k), tot[k] / (cnt[k] ? cnt[k] : 1));
  Scratch& s = ctx->s;
  {  // k_crc timeline: wall_clock64 (100 MHz) stamps of WG 0's start and the last workgroup's final scan
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a, st));
      CK(bcw_decode_segment_async(ctx, d, &p, &t, dres));
      CK(hipEventRecord(b, st));
      CK(hipStreamSynchronize(st));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      uint64_t mc[16];
      CK(hipMemcpy(mc, s.misc, sizeof mc, hipMemcpyDeviceToHost));
      printf("timeline: pipeline %.1f us; k_crc WG0 start -> finalize %.1f us\n", ms * 1e3,
             (mc[M_T_FIN] - mc[M_T_CRC0]) / 100.0);
    }
  }
  const uint64_t nblocks = (n - 40 + kBlock - 1) / kBlock;
  const EmitArgs ea{d, n, p, s.frags, s.fbase, s.rbase, s.bsum, t, s.misc, s.equeue, 0u, nullptr};
  EmitArgs ea_off = ea;
  ea_off.kb_flags = 1u;  // the product kernel with its emission skipped at run time
  EmitArgs ea_st = ea;   // ... with per-wave stamps of its CRC end, emission end and items
  CK(hipMalloc(&ea_st.kb_stamps, 4 * 8 * (size_t)ctx->num_cus * kCrcWaves));
  auto stamp_report = [&]() {
    const int nw = ctx->num_cus * kCrcWaves;
    std::vector<uint64_t> q(4 * (size_t)nw);
    CK(hipMemcpy(q.data(), ea_st.kb_stamps, q.size() * 8, hipMemcpyDeviceToHost));
    uint64_t t0 = ~0ull;
    for (int w = 0; w < nw; ++w) t0 = std::min(t0, q[4 * w]);
    std::vector<double> ce(nw), ee(nw);
    std::vector<uint64_t> it(nw);
    uint64_t tot = 0;
    for (int w = 0; w < nw; ++w) { ce[w] = (q[4 * w] - t0) / 100.0; ee[w] = (q[4 * w + 1] - t0) / 100.0; it[w] = q[4 * w + 2]; tot += it[w]; }
    std::vector<double> sc = ce, se = ee; std::sort(sc.begin(), sc.end()); std::sort(se.begin(), se.end());
    std::vector<uint64_t> si = it; std::sort(si.begin(), si.end());
    printf("emission stamps (us after the first wave's CRC end): CRC end p10 %.1f p50 %.1f p90 %.1f max %.1f | "
           "emission end p50 %.1f p90 %.1f max %.1f | items total %lu, per wave p50 %lu p90 %lu max %lu\n",
           sc[nw / 10], sc[nw / 2], sc[nw * 9 / 10], sc[nw - 1], se[nw / 2], se[nw * 9 / 10], se[nw - 1], tot,
           si[nw / 2], si[nw * 9 / 10], si[nw - 1]);
    int last = 0; for (int w = 0; w < nw; ++w) if (ee[w] > ee[last]) last = w;
    printf("  last wave to finish: w%d CRC end %.1f emission end %.1f items %lu\n", last, ce[last], ee[last], it[last]);
  };
  auto run = [&](auto kern, int grid, const EmitArgs& a) {
    return timeit([&] { hipMemsetAsync(s.equeue, 0, 1024, st);  // the emission queues (k_chase resets them)
                        kern<<<grid, kCrcThreads, 0, st>>>(d, n, 40, nblocks, s.fbase, s.frags, s.frag_cap, ctx->tabs, a, 0u, 0ull, dres, s.misc, 0ull, nblocks, grid); },
                  reps, st);
  };
  const int cus = ctx->num_cus;
  auto runv = [&](int v) -> float {
    switch (v) {
      case 1: return run(k_crc<1>, cus, ea);
      case 99: return run(k_crc<0>, cus, ea_off);
      case 32768: return run(k_crc<32768>, cus, ea);
      case 40960: return run(k_crc<32768 | 8192>, cus, ea);
      case 32776: return run(k_crc<32768 | 8>, cus, ea);
      case 65536: return run(k_crc<65536>, cus, ea);
      case 65537: { const float r = run(k_crc<65536>, cus, ea_st); stamp_report(); return r; }
      case 36864: return run(k_crc<32768 | 4096>, cus, ea);
      case 98: { const float r = run(k_crc<0>, cus, ea_st); stamp_report(); return r; }
      case 2: return run(k_crc<2>, cus, ea);
      case 8: return run(k_crc<8>, cus, ea);
      case 128: return run(k_crc<128>, cus, ea);
      case 1024: return run(k_crc<1024>, cus, ea);
      case 4096: return run(k_crc<4096>, cus, ea);
      case 8192: return run(k_crc<8192>, cus, ea);
      default: return run(k_crc<0>, cus, ea);
    }
  };
  if (argc > 4 && std::string(argv[3]) == "scan") {  // k_scan variants (one-launch decode), interleaved
    EmitArgs ea_s = ea;
    CK(hipMalloc(&ea_s.kb_stamps, 8 * 8 * (size_t)ctx->num_cus * kScanWaves));
    const uint32_t grid = (uint32_t)std::min<uint64_t>(nblocks, (uint64_t)cus);
    auto run_scan = [&](auto kern, const EmitArgs& a) {
      return timeit([&] {
        kern<<<grid, kScanThreads, 0, st>>>(d, n, 40, nblocks, s.fbase, s.rbase, s.bsum, s.frags, s.frag_cap, s.pwin,
                                            scan_unit_stride(nblocks, grid), s.lb, s.lbe, s.lbw, s.tickets, s.epoch,
                                            ctx->tabs, a, 0u, 0ull, dres);
        s.tickets += grid;
        if ((++s.epoch & 0xffffffull) == 0) {
          hipMemsetAsync(s.lb, 0, s.nlb * 8, st); hipMemsetAsync(s.lbe, 0, s.nlb * 8, st);
          hipMemsetAsync(s.lbw, 0, s.nlb * 8, st); s.epoch = 1;
        }
      }, reps, st);
    };
    auto scan_report = [&]() {  // phase ends per wave (us after the first wave's entry)
      const int nw = (int)grid * kScanWaves;
      std::vector<uint64_t> q(8 * (size_t)nw);
      CK(hipMemcpy(q.data(), ea_s.kb_stamps, q.size() * 8, hipMemcpyDeviceToHost));
      uint64_t t0 = ~0ull;
      for (int w = 0; w < nw; ++w) t0 = std::min(t0, q[8 * w]);
      const char* nm[7] = {"entry", "tables", "chased", "units", "barrier", "verify", "emit"};
      for (int k = 0; k < 7; ++k) {
        std::vector<double> v;  // waves that stamped this phase in this launch (the writers' "units" is their end)
        for (int w = 0; w < nw; ++w)
          if (q[8 * w + k] >= t0 && !(k == 3 && (w % kScanWaves) >= kScanWaves - kScanWriters))
            v.push_back((q[8 * w + k] - t0) / 100.0);
        if (v.empty()) continue;
        std::sort(v.begin(), v.end());
        const size_t m = v.size();
        printf("  %-8s p0 %6.1f p10 %6.1f p50 %6.1f p90 %6.1f max %6.1f us\n", nm[k], v[0], v[m / 10], v[m / 2],
               v[m * 9 / 10], v[m - 1]);
      }
      {  // producer spins on a full ring, and the writer's end (its "units" stamp)
        uint64_t rw = 0, wmax = 0; double wend = 0, wwait = 0; int nwr = 0;
        for (int w = 0; w < nw; ++w) {
          const bool wr = (w % kScanWaves) >= kScanWaves - kScanWriters;
          if (!wr) { rw += q[8 * w + 7]; wmax = std::max(wmax, q[8 * w + 7]); }
          else { wend = std::max(wend, (q[8 * w + 3] - t0) / 100.0); wwait += q[8 * w + 7] / 100.0; ++nwr; }
        }
        printf("  ring-full spins: total %lu, max per wave %lu | writer done (max) %.1f us, ack waits %.1f us per writer\n",
               rw, wmax, wend, wwait / nwr);
      }
      std::vector<double> ch;  // chasers only (wave 0 of each workgroup)
      for (int w = 0; w < nw; w += kScanWaves) ch.push_back((q[8 * w + 2] - t0) / 100.0);
      std::sort(ch.begin(), ch.end());
      printf("  chaser wave 0 written: p10 %.1f p50 %.1f p90 %.1f max %.1f us\n", ch[ch.size() / 10],
             ch[ch.size() / 2], ch[ch.size() * 9 / 10], ch.back());
    };
    auto runs = [&](int v) -> float {
      switch (v) {
        case 1: return run_scan(k_scan<1>, ea);
        case 2: return run_scan(k_scan<2>, ea);
        case 8: return run_scan(k_scan<8>, ea);
        case 10: return run_scan(k_scan<10>, ea);
        case 2048: return run_scan(k_scan<2048>, ea);
        case 2058: return run_scan(k_scan<2058>, ea);
        case 4106: return run_scan(k_scan<4106>, ea);
        case 512: { const float r = run_scan(k_scan<512>, ea_s); scan_report(); return r; }
        case 522: { const float r = run_scan(k_scan<522>, ea_s); scan_report(); return r; }
        case 2560: { const float r = run_scan(k_scan<2560>, ea_s); scan_report(); return r; }
        case 2570: { const float r = run_scan(k_scan<2570>, ea_s); scan_report(); return r; }
        default: return run_scan(k_scan<0>, ea);
      }
    };
    const int nv = argc - 4;
    std::vector<std::vector<float>> ts(nv);
    for (int r = 0; r < 5; ++r)
      for (int i = 0; i < nv; ++i) ts[i].push_back(runs(atoi(argv[4 + i])));
    for (int i = 0; i < nv; ++i) {
      std::sort(ts[i].begin(), ts[i].end());
      printf("k_scan<%s>: min %.4f  median %.4f  max %.4f ms\n", argv[4 + i], ts[i][0], ts[i][2], ts[i][4]);
    }
    return 0;
  }
  if (argc > 4 && std::string(argv[3]) == "cmp") {  // k_crc variants interleaved in one process (same buffers)
    const int nv = argc - 4;
    std::vector<std::vector<float>> ts(nv);
    for (int r = 0; r < 7; ++r)
      for (int i = 0; i < nv; ++i) ts[i].push_back(runv(atoi(argv[4 + i])));
    for (int i = 0; i < nv; ++i) {
      std::sort(ts[i].begin(), ts[i].end());
      printf("k_crc<%s>: min %.4f  median %.4f  max %.4f ms\n", argv[4 + i], ts[i][0], ts[i][3], ts[i][6]);
    }
    return 0;
  }
  {
    uint32_t* dout;
    CK(hipMalloc(&dout, 4));
    const float ms = timeit([&] { k_stream<<<cus * 16, 256, 0, st>>>((const uint4*)d, n / 16, dout); }, reps, st);
    printf("stream read     %.4f ms  %.1f GB/s\n", ms, n / (ms * 1e-3) / 1e9);
    const float m1 = timeit([&] { k_pattern<1><<<cus, 1024, 0, st>>>(d, n, dout); }, reps, st);
    const float m2 = timeit([&] { k_pattern<2><<<cus, 1024, 0, st>>>(d, n, dout); }, reps, st);
    const float m4 = timeit([&] { k_pattern<4><<<cus, 1024, 0, st>>>(d, n, dout); }, reps, st);
    const float m8 = timeit([&] { k_pattern<8><<<cus, 1024, 0, st>>>(d, n, dout); }, reps, st);
    printf("pattern GB/s by lanes per window per instruction: G1 %.0f  G2 %.0f  G4 %.0f  G8 %.0f\n",
           n / (m1 * 1e-3) / 1e9, n / (m2 * 1e-3) / 1e9, n / (m4 * 1e-3) / 1e9, n / (m8 * 1e-3) / 1e9);
    const float r1 = timeit([&] { k_pattern<1, true><<<cus, 1024, 0, st>>>(d, n, dout); }, reps, st);
    const float r4 = timeit([&] { k_pattern<4, true><<<cus, 1024, 0, st>>>(d, n, dout); }, reps, st);
    const float r8 = timeit([&] { k_pattern<8, true><<<cus, 1024, 0, st>>>(d, n, dout); }, reps, st);
    printf("pattern, contiguous region per wave: G1 %.0f  G4 %.0f  G8 %.0f GB/s\n", n / (r1 * 1e-3) / 1e9,
           n / (r4 * 1e-3) / 1e9, n / (r8 * 1e-3) / 1e9);
    const uint32_t* img = ctx->tabs.lds_image;
    const float c0 = timeit([&] { k_core<0><<<cus, 1024, 0, st>>>(d, n, img, dout); }, reps, st);
    const float c1 = timeit([&] { k_core<1><<<cus, 1024, 0, st>>>(d, n, img, dout); }, reps, st);
    const float c2 = timeit([&] { k_core<2><<<cus, 1024, 0, st>>>(d, n, img, dout); }, reps, st);
    printf("core (loads+chain): quad+transpose %.4f  quad no-transpose %.4f  lane-window %.4f ms\n", c0, c1, c2);
    const float c3 = timeit([&] { k_core<2 | 4><<<cus, 1024, 0, st>>>(d, n, img, dout); }, reps, st);
    const float c4 = timeit([&] { k_core<2 | 8><<<cus, 1024, 0, st>>>(d, n, img, dout); }, reps, st);
    const float c5 = timeit([&] { k_core<1 | 8><<<cus, 1024, 0, st>>>(d, n, img, dout); }, reps, st);
    printf("core parts: chain only %.4f  lane-window loads only %.4f  quad loads only %.4f ms\n", c3, c4, c5);
    const float e1 = timeit([&] { k_depth<16, 1, false><<<cus, 1024, 0, st>>>(d, n, img, dout); }, reps, st);
    const float e2 = timeit([&] { k_depth<12, 2, false><<<cus, 768, 0, st>>>(d, n, img, dout); }, reps, st);
    const float e3 = timeit([&] { k_depth<12, 2, true><<<cus, 768, 0, st>>>(d, n, img, dout); }, reps, st);
    const float e4 = timeit([&] { k_depth<8, 3, false><<<cus, 512, 0, st>>>(d, n, img, dout); }, reps, st);
    const float e5 = timeit([&] { k_depth<12, 1, false><<<cus, 768, 0, st>>>(d, n, img, dout); }, reps, st);
    printf("depth: 16w d1 %.4f  12w d2 %.4f  12w d2 quad %.4f  8w d3 %.4f  12w d1 %.4f ms\n", e1, e2, e3, e4, e5);
    const float f4 = timeit([&] { k_depth<4, 1, false><<<cus, 256, 0, st>>>(d, n, img, dout); }, reps, st);
    const float f6 = timeit([&] { k_depth<6, 1, false><<<cus, 384, 0, st>>>(d, n, img, dout); }, reps, st);
    const float f8 = timeit([&] { k_depth<8, 1, false><<<cus, 512, 0, st>>>(d, n, img, dout); }, reps, st);
    const float f10 = timeit([&] { k_depth<10, 1, false><<<cus, 640, 0, st>>>(d, n, img, dout); }, reps, st);
    const float f14 = timeit([&] { k_depth<14, 1, false><<<cus, 896, 0, st>>>(d, n, img, dout); }, reps, st);
    const float g8 = timeit([&] { k_depth<8, 2, false><<<cus, 512, 0, st>>>(d, n, img, dout); }, reps, st);
    const float g12 = timeit([&] { k_depth<12, 1, true><<<cus, 768, 0, st>>>(d, n, img, dout); }, reps, st);
    printf("d1 by waves: 4 %.4f  6 %.4f  8 %.4f  10 %.4f  14 %.4f | 8w d2 %.4f | 12w d1 quad %.4f ms\n", f4, f6, f8,
           f10, f14, g8, g12);
    const float h1 = timeit([&] { k_depth<16, 1, false, 7><<<cus, 1024, 0, st>>>(d, n, img, dout); }, reps, st);
    const float h2 = timeit([&] { k_depth<16, 1, false, 1><<<cus, 1024, 0, st>>>(d, n, img, dout); }, reps, st);
    const float h3 = timeit([&] { k_depth<12, 1, false, 7><<<cus, 768, 0, st>>>(d, n, img, dout); }, reps, st);
    const float h4 = timeit([&] { k_depth<16, 1, true, 7><<<cus, 1024, 0, st>>>(d, n, img, dout); }, reps, st);
    printf("rotated start: 16w rot7 %.4f  16w rot1 %.4f  12w rot7 %.4f  16w quad rot7 %.4f ms\n", h1, h2, h3, h4);
    const float i1 = timeit([&] { k_depth<16, 1, false, 0, false><<<cus, 1024, 0, st>>>(d, n, img, dout); }, reps, st);
    const float i2 = timeit([&] { k_depth<12, 1, false, 0, false><<<cus, 768, 0, st>>>(d, n, img, dout); }, reps, st);
    const float i3 = timeit([&] { k_depth<16, 1, true, 0, false><<<cus, 1024, 0, st>>>(d, n, img, dout); }, reps, st);
    const float i4 = timeit([&] { k_depth<12, 1, true, 0, false><<<cus, 768, 0, st>>>(d, n, img, dout); }, reps, st);
    printf("loads only d1: 16w %.4f  12w %.4f  16w quad %.4f  12w quad %.4f ms\n", i1, i2, i3, i4);
  }
  if (argc > 3) {  // counter-collection mode: only the product k_crc, a few launches
    const int k = atoi(argv[3]);
    const int v = argc > 4 ? atoi(argv[4]) : 0;  // ablation variant
    float tm = 0;
    for (int i = 0; i < k; ++i) {
      switch (v) {
        case 1: tm = run(k_crc<1>, cus, ea); break;
        case 2: tm = run(k_crc<2>, cus, ea); break;
        case 4: tm = run(k_crc<4>, cus, ea); break;
        case 8: tm = run(k_crc<8>, cus, ea); break;
        case 128: tm = run(k_crc<128>, cus, ea); break;
        case 256: tm = run(k_crc<256>, cus, ea); break;
        case 384: tm = run(k_crc<384>, cus, ea); break;
        case 7: tm = run(k_crc<7>, cus, ea); break;
        case 520: tm = run(k_crc<520>, cus, ea); break;
        case 1544: tm = run(k_crc<1544>, cus, ea); break;
        case 1024: tm = run(k_crc<1024>, cus, ea); break;
        default: tm = run(k_crc<0>, cus, ea);
      }
    }
    CK(hipStreamSynchronize(st));
    printf("k_crc<%d> x%d done, %.4f ms\n", v, k, tm);
    if (v == 520 || v == 1544) {  // per-wave stamps of the last launch: start / tables / loop end, by XCD (blockIdx % 8)
      const int nw = cus * kCrcWaves;
      std::vector<uint64_t> q(4 * (size_t)nw);
      CK(hipMemcpy(q.data(), t.expire, q.size() * 8, hipMemcpyDeviceToHost));
      uint64_t t0 = ~0ull, tmax = 0;
      for (int w = 0; w < nw; ++w) { t0 = std::min(t0, q[4 * w]); tmax = std::max(tmax, q[4 * w + 2]); }
      std::vector<double> ends(nw);
      double xs[8] = {0}, xe[8] = {0}, xm[8] = {0}; int xn[8] = {0};
      for (int w = 0; w < nw; ++w) {
        const int x = (w / kCrcWaves) % 8;
        const double st = (q[4 * w] - t0) / 100.0, en = (q[4 * w + 2] - t0) / 100.0;
        ends[w] = en; xs[x] += st; xe[x] += en; xm[x] = std::max(xm[x], en); ++xn[x];
      }
      std::vector<double> so = ends; std::sort(so.begin(), so.end());
      printf("wave loop end (us from first entry): min %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f\n", so[0], so[nw / 10],
             so[nw / 2], so[nw * 9 / 10], so[nw - 1]);
      for (int x = 0; x < 8; ++x)
        printf("  xcd %d: mean start %.1f  mean end %.1f  max end %.1f us\n", x, xs[x] / xn[x], xe[x] / xn[x], xm[x]);
      double ss[kCrcWaves] = {0};
      for (int w = 0; w < nw; ++w) ss[w % kCrcWaves] += ends[w];
      printf("  mean end by wave slot:");
      for (int k = 0; k < kCrcWaves; ++k) printf(" %.1f", ss[k] / (nw / kCrcWaves));
      printf("\n");
      std::vector<double> cuend(cus), cuspread(cus);
      for (int c = 0; c < cus; ++c) {
        double mx = 0, mn = 1e30, sm = 0;
        for (int k = 0; k < kCrcWaves; ++k) { const double e = ends[c * kCrcWaves + k]; mx = std::max(mx, e); mn = std::min(mn, e); sm += e; }
        cuend[c] = sm / kCrcWaves; cuspread[c] = mx - mn;
      }
      std::sort(cuend.begin(), cuend.end()); std::sort(cuspread.begin(), cuspread.end());
      printf("  per-WG mean end: min %.1f p50 %.1f max %.1f | per-WG spread (max-min): p10 %.1f p50 %.1f p90 %.1f\n",
             cuend[0], cuend[cus / 2], cuend[cus - 1], cuspread[cus / 10], cuspread[cus / 2], cuspread[cus * 9 / 10]);
      {  // slowest waves: their fragment counts
        std::vector<std::pair<double, int>> ew(nw);
        for (int w = 0; w < nw; ++w) ew[w] = {ends[w], w};
        std::sort(ew.begin(), ew.end());
        printf("  fastest/slowest waves (end us, frags):");
        for (int k : {0, 1, 2, nw - 3, nw - 2, nw - 1}) printf(" [w%d %.1f %lu]", ew[k].second, ew[k].first, q[4 * ew[k].second + 3]);
        printf("\n");
      }
      double tl = 0; for (int w = 0; w < nw; ++w) tl += (q[4 * w + 1] - q[4 * w]) / 100.0;
      printf("  mean table-load time %.2f us\n", tl / nw);
    }
    return 0;
  }
  float a0 = run(k_crc<0>, cus, ea), a1 = run(k_crc<1>, cus, ea), a2 = run(k_crc<2>, cus, ea), a4 = run(k_crc<4>, cus, ea),
        a3 = run(k_crc<3>, cus, ea), a7 = run(k_crc<7>, cus, ea), a8 = run(k_crc<8>, cus, ea);
  printf("k_crc full      %.4f ms  %.1f GB/s\n", a0, n / (a0 * 1e-3) / 1e9);
  printf("k_crc no-chain  %.4f ms\n", a1);
  printf("k_crc no-loads  %.4f ms\n", a2);
  printf("k_crc no-comb   %.4f ms\n", a4);
  printf("k_crc loads+comb only (no chain, no loads) %.4f ms\n", a3);
  printf("k_crc skeleton (1|2|4) %.4f ms\n", a7);
  printf("k_crc no emission %.4f ms\n", a8);
  const float as = timeit([&] {
    hipMemsetAsync(&s.misc[M_DONE_CRC], 0, 8, st);  // the last workgroup finalizes
    hipMemsetAsync(s.equeue, 0, 1024, st);
    k_crc<0><<<cus, kCrcThreads, 0, st>>>(d, n, 40, nblocks, s.fbase, s.frags, s.frag_cap, ctx->tabs, ea, 0u, 0ull, dres,
                                          s.misc, 0ull, nblocks, (uint32_t)cus);
  }, reps, st);
  printf("k_crc + finalize %.4f ms\n", as);
  {
    CK(hipMemset(&s.misc[7], 0, 24));
    run(k_crc<16 | 8>, cus, ea);
    uint64_t m[3];
    CK(hipMemcpy(m, &s.misc[7], 24, hipMemcpyDeviceToHost));
    const double w = (double)cus * kCrcWaves * (reps + 1);  // waves x launches
    printf("  phase cycles per wave (s_memtime): describe %.0f  issue %.0f  compute %.0f\n", m[0] / w, m[1] / w,
           m[2] / w);
  }
  {
    CK(bcw_decode_segment_async(ctx, d, &p, &t, dres));
    CK(hipStreamSynchronize(st));
    uint64_t m[16];
    CK(hipMemcpy(m, s.misc, sizeof m, hipMemcpyDeviceToHost));
    int hz = 0;
    CK(hipDeviceGetAttribute(&hz, hipDeviceAttributeWallClockRate, 0));  // kHz
    printf("  stamps: first WG start -> finalize %.1f us (wall clock %d kHz)\n", (m[M_T_FIN] - m[M_T_CRC0]) * 1e3 / hz, hz);
    auto crun = [&](auto kern) {
      return timeit([&] {
        kern<<<(uint32_t)((nblocks + 63) / 64), 64, 0, st>>>(d, n, 40, nblocks, s.fbase, s.rbase, s.bsum, s.frags,
                                                              s.frag_cap, s.lb, s.lbe, s.misc, s.tickets, s.epoch,
                                                              ctx->tabs.initc, s.chase_direct, s.equeue);
        s.tickets += (nblocks + 63) / 64;
        ++s.epoch;
      }, reps, st);
    };
    printf("k_chase alone %.4f  no sum %.4f  no writes %.4f  chase only %.4f ms  hold 64: %.4f ms\n", crun(k_chase<0>),
           crun(k_chase<1>), crun(k_chase<2>), crun(k_chase<3>), crun(k_chase<256>));
    CK(hipMemset(&s.misc[7], 0, 24));
    crun(k_chase<16>);
    uint64_t m3[3];
    CK(hipMemcpy(m3, &s.misc[7], 24, hipMemcpyDeviceToHost));
    const double wl = (double)((nblocks + 63) / 64) * (reps + 1);
    printf("  k_chase phase cycles per workgroup (s_memtime): chase %.0f  sum %.0f  writes %.0f\n", m3[0] / wl,
           m3[1] / wl, m3[2] / wl);
  }
  // verify still OK after variants (re-run the real pipeline)
  CK(bcw_decode_segment_async(ctx, d, &p, &t, dres));
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(&res, dres, sizeof res, hipMemcpyDeviceToHost));
  printf("recheck: n_records=%lu err=%d bad=%d\n", res.n_records, res.err_class, res.first_bad_record);
  return 0;
}
