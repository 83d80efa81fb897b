#include <unistd.h>
#include <time.h>
// k_crc ablation harness (not product code): one TU with the codec sources, times the full decode
// pipeline and k_crc variants on a synthetic 1 GiB config-B segment.
#include "../../bitcaskdb_amd/csrc/bcw_api.cpp"
#include "../../bitcaskdb_amd/csrc/bcw_decode.hip"
#include "../../bitcaskdb_amd/csrc/bcw_encode.hip"
#include "../../bitcaskdb_amd/csrc/bcw_index.hip"

#include <algorithm>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x) do { auto e_ = (x); if (e_ != hipSuccess && e_ != 0) { fprintf(stderr, "%s:%d err %d\n", __FILE__, __LINE__, (int)e_); exit(1);} } while (0)

// HBM stream-read reference: sum of every 16 B word of the segment
__global__ __launch_bounds__(256) void k_stream(const uint4* __restrict__ p, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// the same with per-workgroup clock stamps (8 words per workgroup, the k_crc kb_stamps layout: [1] end real time,
// [4] entry real time, [5] entry shader cycles, [6] end shader cycles)
__global__ __launch_bounds__(256) void k_stream_clk(const uint4* __restrict__ p, uint64_t n, uint32_t* out,
                                                    uint64_t* __restrict__ st) {
  uint64_t t0 = 0, c0 = 0;
  if (threadIdx.x == 0) { t0 = wall_clock64(); c0 = __builtin_amdgcn_s_memtime(); }
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
  if (threadIdx.x == 0) {
    uint64_t* q = st + 8 * (uint64_t)blockIdx.x;
    q[1] = wall_clock64(); q[4] = t0; q[5] = c0; q[6] = __builtin_amdgcn_s_memtime();
  }
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

// stream-verify load probe: each wave streams its contiguous region in 2 KiB chunks, D chunks in flight.
// PAT 0: lane l reads [32l, 32l + 32) (two 16 B loads, 16 lines each); 1: lane l reads [16l, 16l + 16) and
// [1024 + 16l, ...) (two fully contiguous 1 KiB loads); NT: non-temporal loads
template <int WAVES, int D, int PAT, bool NT = false>
__global__ __launch_bounds__(WAVES * 64) void k_spat(const uint8_t* __restrict__ p, uint64_t n, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = (uint64_t)gridDim.x * WAVES, w0 = (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
  const uint64_t per = n / 2048 / nw;
  const uint8_t* base = p + w0 * per * 2048;
  uint32_t buf[D][8], acc = 0;
  auto issue = [&](uint64_t c, uint32_t (&w)[8]) {
    const uint8_t* q = base + (c < per ? c : 0) * 2048;
    const uint4* a = reinterpret_cast<const uint4*>(q + (PAT == 0 ? 32 * lane : 16 * lane));
    const uint4* b = reinterpret_cast<const uint4*>(q + (PAT == 0 ? 32 * lane + 16 : 1024 + 16 * lane));
    uint4 A, B;
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    if (NT) {
      const v4u va = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(a));
      const v4u vb = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(b));
      A = make_uint4(va.x, va.y, va.z, va.w); B = make_uint4(vb.x, vb.y, vb.z, vb.w);
    }
    else { A = *a; B = *b; }
    w[0] = A.x; w[1] = A.y; w[2] = A.z; w[3] = A.w; w[4] = B.x; w[5] = B.y; w[6] = B.z; w[7] = B.w;
  };
#pragma unroll
  for (int k = 0; k < D; ++k) issue(k, buf[k]);
  for (uint64_t c = 0; c < per; c += D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      if (c + k < per) acc ^= buf[k][0] ^ buf[k][1] ^ buf[k][2] ^ buf[k][3] ^ buf[k][4] ^ buf[k][5] ^ buf[k][6] ^ buf[k][7];
      issue(c + k + D, buf[k]);
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// the chase loop alone (no ticket, no LDS hold, no sum, no writes): V 0 chase_block with a count-only visit,
// V 1 a plain one-header-per-round chain
template <int V>
__global__ __launch_bounds__(64) void k_chase_probe(const uint8_t* __restrict__ seg, uint64_t seg_len, uint32_t start_off,
                                                    uint64_t nblocks, uint32_t* __restrict__ out) {
  const uint64_t b = blockIdx.x * 64ull + threadIdx.x;
  uint32_t bufsize = 0;
  uint64_t boff = 0;
  if (b < nblocks) {
    boff = (uint64_t)start_off + b * kBlock;
    bufsize = (uint32_t)((seg_len - boff) < kBlock ? (seg_len - boff) : kBlock);
  }
  uint32_t acc = 0, n = 0;
  if (V == 0) {
    n = chase_block(seg, seg_len, boff, bufsize,
                    [&](uint32_t, uint32_t, uint32_t len, uint32_t crc, uint32_t ty) { acc ^= crc + len + ty; });
  } else {
    uint32_t h = 0;
    while (h + kHdr <= bufsize) {
      uint32_t cr, ln, ty;
      read_header(seg, seg_len, boff + h, cr, ln, ty);
      const uint32_t st = h + kHdr;
      if (ln > bufsize - st) ln = bufsize - st;
      acc ^= cr + ln + ty;
      ++n;
      h = st + ln;
    }
  }
  if (b < nblocks) out[b] = acc + n;
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
  const EmitArgs ea{d, n, p, s.frags, s.fbase, s.rbase, s.bsum, t, s.misc, 0u, nullptr};
  EmitArgs ea_off = ea;
  ea_off.kb_flags = 1u;  // the product kernel with its emission skipped at run time
  EmitArgs ea_st = ea;   // ... with per-wave stamps of its CRC end, emission end and items
  CK(hipMalloc(&ea_st.kb_stamps, 8 * 8 * (size_t)ctx->num_cus * kCrcWaves));
  auto stamp_report = [&]() {
    const int nw = ctx->num_cus * kCrcWaves;
    std::vector<uint64_t> q8(8 * (size_t)nw), q(4 * (size_t)nw);
    CK(hipMemcpy(q8.data(), ea_st.kb_stamps, q8.size() * 8, hipMemcpyDeviceToHost));
    for (int w = 0; w < nw; ++w) for (int k = 0; k < 4; ++k) q[4 * w + k] = q8[8 * w + k];
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
  // KB_CLOCK: every timed launch also writes per-wave stamps; last_mhz = the last launch's in-kernel clock (median
  // over waves of shader cycles / real time), so that a variant's cycles = ms x MHz
  const bool kb_clock = getenv("KB_CLOCK") != nullptr;
  uint64_t* clk_st = nullptr;
  const size_t clk_per = 8 * (size_t)ctx->num_cus * kCrcWaves;
  if (kb_clock) CK(hipMalloc(&clk_st, clk_per * 8));
  double last_mhz = 0;
  static char last_tl[1024] = "";
  auto clock_of = [&](const uint64_t* dq, int nw) {
    std::vector<uint64_t> q(8 * (size_t)nw);
    CK(hipMemcpy(q.data(), dq, q.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> f;
    for (int w = 0; w < nw; ++w) {
      const uint64_t* e = q.data() + 8 * w;
      if (e[1] > e[4]) f.push_back((double)(e[6] - e[5]) / (double)(e[1] - e[4]) * 100.0);
    }
    std::sort(f.begin(), f.end());
    // the last launch's timeline (real time, us from the first wave's entry): entry spread, stream end p50 / max,
    // wave end max, and the median stream duration per wave
    uint64_t t0 = ~0ull;
    for (int w = 0; w < nw; ++w) if (q[8 * w + 4]) t0 = std::min(t0, q[8 * w + 4]);
    std::vector<double> ent, se, we, dur;
    for (int w = 0; w < nw; ++w) {
      const uint64_t* e = q.data() + 8 * w;
      if (!e[4]) continue;
      ent.push_back((e[4] - t0) / 100.0);
      if (e[0]) { se.push_back((e[0] - t0) / 100.0); dur.push_back((e[0] - e[4]) / 100.0); }
      if (e[1]) we.push_back((e[1] - t0) / 100.0);
    }
    std::sort(ent.begin(), ent.end()); std::sort(se.begin(), se.end()); std::sort(we.begin(), we.end());
    std::sort(dur.begin(), dur.end());
    if (!ent.empty() && !se.empty() && !we.empty()) {
      int o = snprintf(last_tl, sizeof last_tl, "entry max %.1f | stream end p10 %.1f p50 %.1f max %.1f | end max %.1f | "
                       "stream dur p50 %.1f", ent.back(), se[se.size() / 10], se[se.size() / 2], se.back(), we.back(),
                       dur[dur.size() / 2]);
      // per XCC (HW_REG_XCC_ID): stream end p50 / max and wave end max; then the last wave's stream end, end, items
      std::vector<double> xs[16], xe[16];
      int last = -1;
      for (int w = 0; w < nw; ++w) {
        const uint64_t* e = q.data() + 8 * w;
        if (!e[4] || !e[0] || !e[1]) continue;
        const int x = (int)((e[7] >> 32) & 15);
        xs[x].push_back((e[0] - t0) / 100.0); xe[x].push_back((e[1] - t0) / 100.0);
        if (last < 0 || e[1] > q[8 * last + 1]) last = w;
      }
      o += snprintf(last_tl + o, sizeof last_tl - o, "\n      per XCC stream end p50/max, end max:");
      for (int x = 0; x < 16; ++x) {
        if (xs[x].empty()) continue;
        std::sort(xs[x].begin(), xs[x].end()); std::sort(xe[x].begin(), xe[x].end());
        o += snprintf(last_tl + o, sizeof last_tl - o, " x%d %.1f/%.1f,%.1f", x, xs[x][xs[x].size() / 2], xs[x].back(),
                      xe[x].back());
      }
      {  // the slowest 5 % of the streams against the rest: their fragments per wave
        std::vector<std::pair<double, uint64_t>> dv;
        for (int w = 0; w < nw; ++w) {
          const uint64_t* e = q.data() + 8 * w;
          if (e[4] && e[0]) dv.push_back({(double)(e[0] - e[4]) / 100.0, e[3]});
        }
        std::sort(dv.begin(), dv.end());
        if (dv.size() >= 40) {
          const size_t n5 = dv.size() / 20;
          double fs = 0, fa = 0;
          for (size_t i = dv.size() - n5; i < dv.size(); ++i) fs += dv[i].second;
          for (auto& x : dv) fa += x.second;
          o += snprintf(last_tl + o, sizeof last_tl - o, "\n      fragments per wave: slowest 5 %% %.0f, all %.0f",
                        fs / n5, fa / dv.size());
        }
      }
      if (last >= 0) {
        const uint64_t* e = q.data() + 8 * last;
        double wsm = 0; uint64_t wit = 0;  // its workgroup's last stream end and items
        for (int v = 0; v < kCrcWaves; ++v) {
          const uint64_t* f = q.data() + 8 * ((last / kCrcWaves) * kCrcWaves + v);
          if (f[0]) wsm = std::max(wsm, (f[0] - t0) / 100.0);
          wit += f[2];
        }
        o += snprintf(last_tl + o, sizeof last_tl - o, "\n      last wave w%d (XCC %d, HW_ID %08lx): stream end %.1f, end "
                      "%.1f, items %lu; its workgroup: last stream end %.1f, items %lu", last, (int)((e[7] >> 32) & 15),
                      (unsigned long)(e[7] & 0xffffffffu), (e[0] - t0) / 100.0, (e[1] - t0) / 100.0,
                      (unsigned long)e[2], wsm, (unsigned long)wit);
      }
    }
    return f.empty() ? 0.0 : f[f.size() / 2];
  };
  int run_reps = reps;            // 0: run() launches once, untimed (seqk)
  uint64_t* seq_stamps = nullptr;  // seqk: this launch's stamp slice
  auto run = [&](auto kern, int grid, const EmitArgs& a0) {
    EmitArgs a = a0;
    if (kb_clock && !a.kb_stamps) a.kb_stamps = seq_stamps ? seq_stamps : clk_st;
    if (run_reps == 0) {
      kern<<<grid, kCrcThreads, 0, st>>>(d, n, 40, nblocks, s.fbase, s.fok, s.srec, s.frag_cap, ctx->tabs, a, 0u, 0ull, dres, s.misc, 0ull, nblocks, grid, s.wstart, s.xbal);
      return 0.0f;
    }
    const float ms = timeit([&] { kern<<<grid, kCrcThreads, 0, st>>>(d, n, 40, nblocks, s.fbase, s.fok, s.srec, s.frag_cap, ctx->tabs, a, 0u, 0ull, dres, s.misc, 0ull, nblocks, grid, s.wstart, s.xbal); },
                  reps, st);
    if (kb_clock && a.kb_stamps == clk_st) last_mhz = clock_of(clk_st, grid * kCrcWaves);
    return ms;
  };
  const int cus = ctx->num_cus;
  auto runv = [&](int v) -> float {
    switch (v) {
      case 8: return run(k_crc<8>, cus, ea);              // no emission
      case 64: return run(k_crc<64>, cus, ea);            // emission before the stream
      case 8388608: return run(k_crc<8388608>, cus, ea);  // every chunk on the fast chain
      case 8388616: return run(k_crc<8388616>, cus, ea);  // the same without emission
      case 32768: return run(k_crc<32768>, cus, ea);      // emission only (no CRC pass)
      case 4096: return run(k_crc<4096>, cus, ea);        // emission without row stores
      case 131072: return run(k_crc<131072>, cus, ea);    // emission without the RecordFromBytes parse
      case 163840: return run(k_crc<163840>, cus, ea);    // emission only, without the parse
      case 16384: return run(k_crc<16384>, cus, ea);      // each wave's range as 4 stream_verify calls
      case 16392: return run(k_crc<16392>, cus, ea);      // the same without emission
      case 36864: return run(k_crc<36864>, cus, ea);      // emission only, without row stores
      case 99: return run(k_crc<0>, cus, ea_off);
      case 98: { const float r = run(k_crc<0>, cus, ea_st); stamp_report(); return r; }
      default: return run(k_crc<0>, cus, ea);
    }
  };
  if (argc > 5 && std::string(argv[3]) == "seqk") {  // N back-to-back launches of one kernel, per-launch times
    // v: -1 plain HBM stream (k_stream), -2 the decode pipeline, otherwise the k_crc variant v (runv's list)
    const int nrep = atoi(argv[4]), v = atoi(argv[5]);
    uint32_t* dout;
    CK(hipMalloc(&dout, 4));
    std::vector<hipEvent_t> ev(2 * nrep);
    for (auto& e : ev) CK(hipEventCreate(&e));
    const uint64_t nb = (n - 40 + kBlock - 1) / kBlock;
    CK(hipStreamSynchronize(st));
    // KB_CLOCK (k_crc variants only): every launch writes per-wave stamps into its own slice; the in-kernel clock of a
    // launch is the median over waves of shader cycles / real time between k_crc's entry and the wave's end
    const bool clk = getenv("KB_CLOCK") != nullptr && v != -2;
    const size_t per = 8 * (size_t)cus * kCrcWaves;  // (>= the stream's 16 x cus workgroups)
    uint64_t* dst = nullptr;
    if (clk) CK(hipMalloc(&dst, per * 8 * (size_t)nrep));
    if (getenv("KB_IDLE_MS")) usleep(1000 * atoi(getenv("KB_IDLE_MS")));  // start from an idle chip
    timespec tm0, tb0;
    clock_gettime(CLOCK_MONOTONIC, &tm0);
    clock_gettime(CLOCK_BOOTTIME, &tb0);
    printf("mark seqk_start mono_ns %lld boot_ns %lld\n", tm0.tv_sec * 1000000000ll + tm0.tv_nsec,
           tb0.tv_sec * 1000000000ll + tb0.tv_nsec);
    for (int i = 0; i < nrep; ++i) {
      CK(hipEventRecord(ev[2 * i], st));
      if (v == -1 || (v == -3 && (i & 1))) {
        if (clk) k_stream_clk<<<cus * 16, 256, 0, st>>>((const uint4*)d, n / 16, dout, dst + per * i);
        else k_stream<<<cus * 16, 256, 0, st>>>((const uint4*)d, n / 16, dout);
      } else if (v == -2) {
        CK(launch_decode(d, p, t, dres, ctx->tabs, s, nb, 1, st, cus, nullptr));
      } else {
        run_reps = 0;
        seq_stamps = clk ? dst + per * i : nullptr;
        runv(v);
        run_reps = reps;
        seq_stamps = nullptr;
      }
      CK(hipEventRecord(ev[2 * i + 1], st));
    }
    CK(hipStreamSynchronize(st));
    if (clk) {
      std::vector<uint64_t> q(per * nrep);
      CK(hipMemcpy(q.data(), dst, q.size() * 8, hipMemcpyDeviceToHost));
      printf("seqk %d clock MHz:", v);
      for (int i = 0; i < nrep; ++i) {
        std::vector<double> f;
        for (int w = 0; w < cus * 16; ++w) {  // (k_crc: waves; the stream: workgroups)
          const uint64_t* e = q.data() + per * i + 8 * w;
          if (e[1] > e[4]) f.push_back((double)(e[6] - e[5]) / (double)(e[1] - e[4]) * 100.0);
        }
        std::sort(f.begin(), f.end());
        printf(" %.0f", f.empty() ? 0.0 : f[f.size() / 2]);
      }
      printf("\n");
    }
    printf("seqk %d us:", v);
    for (int i = 0; i < nrep; ++i) {
      float ms; CK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
      printf(" %.0f", ms * 1e3);
    }
    printf("\n");
    return 0;
  }
  if (argc > 3 && std::string(argv[3]) == "xbal") {  // pipelines with the per-XCD split on / off, interleaved
    const uint64_t nb = (n - 40 + kBlock - 1) / kBlock;
    std::vector<float> ton, toff;
    for (int r = 0; r < 7; ++r)
      for (int on = 0; on <= 1; ++on) {
        s.xbal_on = (uint32_t)on;
        const float ms = timeit([&] { CK(launch_decode(d, p, t, dres, ctx->tabs, s, nb, 1, st, cus, nullptr)); }, reps, st);
        (on ? ton : toff).push_back(ms);
      }
    std::sort(ton.begin(), ton.end()); std::sort(toff.begin(), toff.end());
    XBal xb;
    CK(hipMemcpy(&xb, s.xbal, sizeof xb, hipMemcpyDeviceToHost));
    printf("xbal pipeline on: min %.4f median %.4f max %.4f ms | off: min %.4f median %.4f max %.4f ms\n", ton[0], ton[3],
           ton[6], toff[0], toff[3], toff[6]);
    printf("xbal weights:");
    for (int y = 0; y < 8; ++y) printf(" %.3f", xb.w[y] / 65536.0);
    printf("\n");
    s.xbal_on = 1;
    return 0;
  }
  if (argc > 4 && std::string(argv[3]) == "seq") {  // N back-to-back pipelines (k_chase + k_crc), per-launch times
    const int nrep = atoi(argv[4]);
    const int gap_us = argc > 5 ? atoi(argv[5]) : 0;  // host sleep between launches (0: queued back to back)
    std::vector<hipEvent_t> ev(2 * nrep);
    for (auto& e : ev) CK(hipEventCreate(&e));
    const uint64_t nb = (n - 40 + kBlock - 1) / kBlock;
    for (int i = 0; i < nrep; ++i) {
      if (gap_us >= 0 || i == 0) CK(hipEventRecord(ev[2 * i], st));
      CK(launch_decode(d, p, t, dres, ctx->tabs, s, nb, 1, st, cus, nullptr));
      if (gap_us >= 0 || i == nrep - 1) CK(hipEventRecord(ev[2 * i + 1], st));
      if (gap_us > 0) { CK(hipStreamSynchronize(st)); usleep(gap_us); }
    }
    CK(hipStreamSynchronize(st));
    if (gap_us < 0) {
      float ms; CK(hipEventElapsedTime(&ms, ev[0], ev[2 * nrep - 1]));
      printf("seq pipeline (no events between): %.1f us per pipeline\n", ms * 1e3 / nrep);
      return 0;
    }
    printf("seq pipeline us:");
    for (int i = 0; i < nrep; ++i) {
      float ms; CK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
      printf(" %.0f", ms * 1e3);
    }
    printf("\n");
    return 0;
  }
  if (argc > 4 && std::string(argv[3]) == "cmp") {  // k_crc variants interleaved in one process (same buffers)
    const int nv = argc - 4;
    std::vector<std::vector<float>> ts(nv);
    std::vector<std::vector<double>> mc(nv), mh(nv);
    for (int r = 0; r < 7; ++r)
      for (int i = 0; i < nv; ++i) {
        const float ms = runv(atoi(argv[4 + i]));
        ts[i].push_back(ms);
        mh[i].push_back(last_mhz);
        mc[i].push_back(ms * last_mhz * 1e-3);  // Mcycles
      }
    for (int i = 0; i < nv; ++i) {
      std::sort(ts[i].begin(), ts[i].end());
      std::sort(mc[i].begin(), mc[i].end());
      std::sort(mh[i].begin(), mh[i].end());
      printf("k_crc<%s>: min %.4f  median %.4f  max %.4f ms", argv[4 + i], ts[i][0], ts[i][3], ts[i][6]);
      if (kb_clock) printf("  | clock median %.0f MHz, Mcycles min %.4f median %.4f", mh[i][3], mc[i][0], mc[i][3]);
      printf("\n");
      if (kb_clock) { last_tl[0] = 0; runv(atoi(argv[4 + i])); printf("    timeline: %s\n", last_tl); }
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
  }
  if (argc > 3) {  // counter-collection mode: only the product k_crc, a few launches
    const int k = atoi(argv[3]);
    const int v = argc > 4 ? atoi(argv[4]) : 0;  // ablation variant
    float tm = 0;
    for (int i = 0; i < k; ++i) {
      tm = runv(v);
    }
    CK(hipStreamSynchronize(st));
    printf("k_crc<%d> x%d done, %.4f ms\n", v, k, tm);
    return 0;
  }
  const float a0 = run(k_crc<0>, cus, ea), a1 = run(k_crc<8388616>, cus, ea), a8 = run(k_crc<8>, cus, ea),
              a9 = run(k_crc<32768>, cus, ea);
  printf("k_crc full      %.4f ms  %.1f GB/s\n", a0, n / (a0 * 1e-3) / 1e9);
  printf("k_crc fast chain only (no emission) %.4f  no emission %.4f  emission only %.4f ms\n", a1, a8, a9);
  const float as = timeit([&] {
    hipMemsetAsync(&s.misc[M_DONE_CRC], 0, 8, st);  // the last workgroup finalizes
    k_crc<0><<<cus, kCrcThreads, 0, st>>>(d, n, 40, nblocks, s.fbase, s.fok, s.srec, s.frag_cap, ctx->tabs, ea, 0u, 0ull, dres,
                                          s.misc, 0ull, nblocks, (uint32_t)cus, s.wstart, s.xbal);
  }, reps, st);
  printf("k_crc + finalize %.4f ms\n", as);
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
                                                              s.srec, s.frag_cap, s.lb, s.lbe, s.misc, s.epoch,
                                                              ctx->tabs.initc, s.chase_direct, 0ull, s.wstart,
                                                              (uint32_t)cus * kCrcWaves, s.xbal, s.xbal_on);
        ++s.epoch;
      }, reps, st);
    };
    printf("k_chase alone %.4f  no sum %.4f  no writes %.4f  chase only %.4f ms  hold 16: %.4f ms\n", crun(k_chase<0>),
           crun(k_chase<1>), crun(k_chase<2>), crun(k_chase<3>), crun(k_chase<256>));
    {
      uint32_t* pout;
      CK(hipMalloc(&pout, (nblocks + 64) * 4));
      const uint32_t pg = (uint32_t)((nblocks + 63) / 64);
      const float p0 = timeit([&] { k_chase_probe<0><<<pg, 64, 0, st>>>(d, n, 40, nblocks, pout); }, reps, st);
      const float p1 = timeit([&] { k_chase_probe<1><<<pg, 64, 0, st>>>(d, n, 40, nblocks, pout); }, reps, st);
      printf("chase probe: chase_block with a count-only visit %.4f ms, plain one-header chain %.4f ms\n", p0, p1);
    }
    {  // per-workgroup wall-clock stamps (entry, chase end, sum end, end) of one launch, relative to the first entry
      const uint64_t nwg = (nblocks + 63) / 64;
      uint64_t* stp;
      CK(hipMalloc(&stp, nwg * 32));
      for (int rep = 0; rep < 3; ++rep) {
        k_chase<32><<<(uint32_t)nwg, 64, 0, st>>>(d, n, 40, nblocks, s.fbase, s.rbase, s.bsum, s.frags, s.srec, s.frag_cap,
                                                  s.lb, stp, s.misc, s.epoch, ctx->tabs.initc, s.chase_direct, 0ull,
                                                  s.wstart, (uint32_t)cus * kCrcWaves, s.xbal, s.xbal_on);
        ++s.epoch;
        CK(hipStreamSynchronize(st));
      }
      std::vector<uint64_t> h4(nwg * 4);
      CK(hipMemcpy(h4.data(), stp, nwg * 32, hipMemcpyDeviceToHost));
      uint64_t t0 = ~0ull;
      for (uint64_t w = 0; w < nwg; ++w) t0 = std::min(t0, h4[4 * w]);
      std::vector<double> col[4];
      for (uint64_t w = 0; w < nwg; ++w)
        for (int k = 0; k < 4; ++k) col[k].push_back((h4[4 * w + k] - t0) / 100.0);
      const char* nm[4] = {"entry", "chase end", "sum end", "end"};
      for (int k = 0; k < 4; ++k) {
        std::vector<double> c = col[k];
        std::sort(c.begin(), c.end());
        printf("  k_chase stamps %-9s us: min %.2f p10 %.2f p50 %.2f p90 %.2f max %.2f\n", nm[k], c[0], c[c.size() / 10],
               c[c.size() / 2], c[c.size() * 9 / 10], c.back());
      }
      // entry by workgroup id (dispatch order), every 32nd
      printf("  k_chase entry by wg (every 32nd):");
      for (uint64_t w = 0; w < nwg; w += 32) printf(" %.2f", col[0][w]);
      printf("\n  k_chase chase end by wg (every 32nd):");
      for (uint64_t w = 0; w < nwg; w += 32) printf(" %.2f", col[1][w]);
      printf("\n");
      CK(hipFree(stp));
    }
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
