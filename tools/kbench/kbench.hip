// k_crc ablation harness (not product code): one TU with the codec sources, times the full decode
// pipeline and k_crc variants on a synthetic 1 GiB config-B segment.
#include "../../bitcaskdb_amd/csrc/bcw_api.cpp"
#include "../../bitcaskdb_amd/csrc/bcw_decode.hip"

#include <cstdio>
#include <cstdlib>

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
  CK(hipMalloc(&d, n));
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
  const uint64_t nblocks = (n - 40 + kBlock - 1) / kBlock;
  auto run = [&](auto kern, int grid) {
    return timeit([&] { kern<<<grid, kCrcThreads, 0, st>>>(d, n, 40, nblocks, s.fbase, s.frags, s.frag_cap, ctx->tabs, s.pre, s.wgagg, s.wgx, s.misc); },
                  reps, st);
  };
  const int cus = ctx->num_cus;
  {
    uint32_t* dout;
    CK(hipMalloc(&dout, 4));
    const float ms = timeit([&] { k_stream<<<cus * 16, 256, 0, st>>>((const uint4*)d, n / 16, dout); }, reps, st);
    printf("stream read     %.4f ms  %.1f GB/s\n", ms, n / (ms * 1e-3) / 1e9);
  }
  if (argc > 3) {  // counter-collection mode: only the product k_crc, a few launches
    const int k = atoi(argv[3]);
    for (int i = 0; i < k; ++i) run(k_crc<0>, cus);
    CK(hipStreamSynchronize(st));
    printf("k_crc x%d done\n", k);
    return 0;
  }
  float a0 = run(k_crc<0>, cus), a1 = run(k_crc<1>, cus), a2 = run(k_crc<2>, cus), a4 = run(k_crc<4>, cus),
        a3 = run(k_crc<3>, cus), a7 = run(k_crc<7>, cus), a8 = run(k_crc<8>, cus);
  printf("k_crc full      %.4f ms  %.1f GB/s\n", a0, n / (a0 * 1e-3) / 1e9);
  printf("k_crc no-chain  %.4f ms\n", a1);
  printf("k_crc no-loads  %.4f ms\n", a2);
  printf("k_crc no-comb   %.4f ms\n", a4);
  printf("k_crc loads+comb only (no chain, no loads) %.4f ms\n", a3);
  printf("k_crc skeleton (1|2|4) %.4f ms\n", a7);
  printf("k_crc no tail   %.4f ms\n", a8);
  const float as = timeit([&] {
    hipMemsetAsync(&s.misc[5], 0, 8, st);  // M_DONE_CRC: the last workgroup runs the aggregate scan
    k_crc<0><<<cus, kCrcThreads, 0, st>>>(d, n, 40, nblocks, s.fbase, s.frags, s.frag_cap, ctx->tabs, s.pre, s.wgagg,
                                          s.wgx, s.misc);
  }, reps, st);
  printf("k_crc + scan    %.4f ms\n", as);
  {
    uint64_t m[16];
    CK(hipMemcpy(m, s.misc, sizeof m, hipMemcpyDeviceToHost));
    int hz = 0;
    CK(hipDeviceGetAttribute(&hz, hipDeviceAttributeWallClockRate, 0));  // kHz
    printf("  stamps: first WG start -> scan start %.1f us, scan %.1f us (wall clock %d kHz)\n",
           (m[11] - m[10]) * 1e3 / hz, (m[12] - m[11]) * 1e3 / hz, hz);
  }
  // verify still OK after variants (re-run the real pipeline)
  CK(bcw_decode_segment_async(ctx, d, &p, &t, dres));
  CK(hipMemcpy(&res, dres, sizeof res, hipMemcpyDeviceToHost));
  printf("recheck: n_records=%lu err=%d bad=%d\n", res.n_records, res.err_class, res.first_bad_record);
  return 0;
}
