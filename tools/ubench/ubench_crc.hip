// Microbenchmark used to pick the CRC-32C strategy for the WAL decode kernel on gfx950.
// Not product code: it measures (a) streaming read bandwidth for several per-lane access
// shapes and (b) LDS-table CRC-32C throughput for slice-by-2 / slice-by-4 with 32-way
// replicated tables, one wavefront per 32 KiB WAL block (512 B contiguous per lane).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <cstring>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

static const size_t BYTES = 1ull << 30;

__global__ __launch_bounds__(256) void k_stream(const uint4* __restrict__ d, uint32_t* out, size_t n16) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
    uint4 v = d[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// each lane reads SEG contiguous bytes; a wave covers 64*SEG bytes
template <int SEG>
__global__ __launch_bounds__(256) void k_lane_contig(const uint4* __restrict__ d, uint32_t* out, size_t nbytes) {
  const int lane = threadIdx.x & 63;
  const size_t wave = (blockIdx.x * 256ull + threadIdx.x) >> 6;
  const size_t nwaves = (size_t)gridDim.x * 4;
  const size_t chunk = 64ull * SEG;
  uint32_t acc = 0;
  for (size_t c = wave; c * chunk < nbytes; c += nwaves) {
    const uint4* p = d + (c * chunk + (size_t)lane * SEG) / 16;
#pragma unroll
    for (int i = 0; i < SEG / 16; i += 8) {
      uint4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = p[i + j];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// slice-by-4 step over a 32-bit little-endian word with 32x replicated tables in LDS
__device__ __forceinline__ uint32_t s4(const uint32_t* t, uint32_t lo, uint32_t s, uint32_t w) {
  uint32_t x = s ^ w;
  uint32_t a = t[((3 * 256 + (x & 0xff)) << 5) + lo];
  uint32_t b = t[((2 * 256 + ((x >> 8) & 0xff)) << 5) + lo];
  uint32_t c = t[((1 * 256 + ((x >> 16) & 0xff)) << 5) + lo];
  uint32_t e = t[((0 * 256 + (x >> 24)) << 5) + lo];
  return a ^ b ^ c ^ e;
}
__device__ __forceinline__ uint32_t s2(const uint32_t* t, uint32_t lo, uint32_t s, uint32_t h) {
  uint32_t x = s ^ h;
  uint32_t a = t[((1 * 256 + (x & 0xff)) << 5) + lo];
  uint32_t b = t[((0 * 256 + ((x >> 8) & 0xff)) << 5) + lo];
  return (s >> 16) ^ a ^ b;
}

// SLICE = 2 or 4; ILP = independent chains per lane (lane segment split in ILP parts)
template <int SLICE, int ILP, int NT>
__global__ __launch_bounds__(NT) void k_crc(const uint4* __restrict__ d, uint32_t* __restrict__ out,
                                            const uint32_t* __restrict__ gt, size_t nblocks) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (int i = threadIdx.x; i < SLICE * 256 * 32; i += NT) lds[i] = gt[i >> 5];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t lo = lane & 31;
  const size_t wave = (blockIdx.x * (size_t)NT + threadIdx.x) >> 6;
  const size_t nwaves = (size_t)gridDim.x * (NT / 64);
  constexpr int PART = 32 / ILP;  // uint4 per chain
  for (size_t b = wave; b < nblocks; b += nwaves) {
    const uint4* p = d + b * 2048 + lane * 32;
    uint32_t s[ILP];
#pragma unroll
    for (int k = 0; k < ILP; ++k) s[k] = 0xffffffffu;
#pragma unroll 2
    for (int i = 0; i < PART; i += 4) {
      uint4 v[ILP][4];
#pragma unroll
      for (int k = 0; k < ILP; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[k][j] = p[k * PART + i + j];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
          for (int k = 0; k < ILP; ++k) {
            uint32_t w = q == 0 ? v[k][j].x : q == 1 ? v[k][j].y : q == 2 ? v[k][j].z : v[k][j].w;
            if (SLICE == 4) s[k] = s4(lds, lo, s[k], w);
            else { s[k] = s2(lds, lo, s[k], w & 0xffff); s[k] = s2(lds, lo, s[k], w >> 16); }
          }
        }
      }
    }
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < ILP; ++k) r ^= s[k];
    out[b * 64 + lane] = r;
  }
}

static void make_tables(std::vector<uint32_t>& t) {
  t.assign(4 * 256, 0);
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    t[b] = c;
  }
  for (int k = 1; k < 4; ++k)
    for (int b = 0; b < 256; ++b) t[k * 256 + b] = (t[(k - 1) * 256 + b] >> 8) ^ t[t[(k - 1) * 256 + b] & 0xff];
}

static uint32_t cpu_crc_seg(const uint8_t* p, size_t n, const std::vector<uint32_t>& t) {
  uint32_t s = 0xffffffffu;
  for (size_t i = 0; i < n; ++i) s = (s >> 8) ^ t[(s ^ p[i]) & 0xff];
  return s;
}

template <typename F>
static float timeit(F f, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  uint8_t* d; uint32_t *out, *gt, *crcout;
  CHECK(hipMalloc(&d, BYTES));
  CHECK(hipMalloc(&out, 1024));
  CHECK(hipMalloc(&gt, 4 * 256 * 4));
  size_t nblocks = BYTES / 32768;
  CHECK(hipMalloc(&crcout, nblocks * 64 * 4));
  std::vector<uint8_t> h(BYTES);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < BYTES; i += 8) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; std::memcpy(&h[i], &x, 8); }
  CHECK(hipMemcpy(d, h.data(), BYTES, hipMemcpyHostToDevice));
  std::vector<uint32_t> t; make_tables(t);
  CHECK(hipMemcpy(gt, t.data(), t.size() * 4, hipMemcpyHostToDevice));
  const int reps = 10;
  auto gbs = [](float ms) { return BYTES / (ms * 1e-3) / 1e9; };
  for (int grid : {1024, 2048, 4096}) {
    float ms = timeit([&] { k_stream<<<grid, 256>>>((const uint4*)d, out, BYTES / 16); }, reps);
    printf("stream grid=%d  %.3f ms  %.0f GB/s\n", grid, ms, gbs(ms));
  }
  for (int grid : {1024, 2048, 4096}) {
    float ms = timeit([&] { k_lane_contig<512><<<grid, 256>>>((const uint4*)d, out, BYTES); }, reps);
    printf("lane_contig512 grid=%d  %.3f ms  %.0f GB/s\n", grid, ms, gbs(ms));
    ms = timeit([&] { k_lane_contig<256><<<grid, 256>>>((const uint4*)d, out, BYTES); }, reps);
    printf("lane_contig256 grid=%d  %.3f ms  %.0f GB/s\n", grid, ms, gbs(ms));
    ms = timeit([&] { k_lane_contig<128><<<grid, 256>>>((const uint4*)d, out, BYTES); }, reps);
    printf("lane_contig128 grid=%d  %.3f ms  %.0f GB/s\n", grid, ms, gbs(ms));
  }
  std::vector<uint32_t> hc(nblocks * 64);
  auto check = [&](int ilp, const char* name) {
    CHECK(hipMemcpy(hc.data(), crcout, hc.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (size_t b = 0; b < nblocks && b < 64; ++b)
      for (int l = 0; l < 64; ++l) {
        uint32_t r = 0;
        for (int k = 0; k < ilp; ++k) r ^= cpu_crc_seg(&h[b * 32768 + l * 512 + k * 512 / ilp], 512 / ilp, t);
        if (r != hc[b * 64 + l]) ++bad;
      }
    printf("  %s check: %s\n", name, bad ? "MISMATCH" : "ok");
  };
  // LDS per WG = SLICE*32 KiB -> one WG per CU for s4; NT threads = NT/64 waves per CU
#define RUN(SL, IL, NT_, GRID, CHK) { float ms = timeit([&] { k_crc<SL, IL, NT_><<<GRID, NT_, SL * 32768>>>((const uint4*)d, crcout, gt, nblocks); }, reps); \
    printf("crc s%d ilp%d nt=%d grid=%d  %.3f ms  %.0f GB/s\n", SL, IL, NT_, GRID, ms, gbs(ms)); if (CHK) check(IL, "chk"); }
  RUN(4, 1, 256, 256, 1)
  RUN(4, 1, 512, 256, 1)
  RUN(4, 1, 1024, 256, 1)
  RUN(4, 2, 512, 256, 1)
  RUN(4, 2, 1024, 256, 1)
  RUN(4, 4, 1024, 256, 0)
  RUN(2, 1, 512, 512, 1)
  RUN(2, 1, 1024, 512, 1)
  RUN(2, 2, 1024, 512, 1)
  RUN(2, 4, 1024, 512, 0)
  RUN(4, 1, 1024, 512, 0)
  return 0;
}
