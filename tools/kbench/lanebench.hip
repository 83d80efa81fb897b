// Load-pattern probe for k_crc's window loads (not product code). A wave reads 8 KiB passes (64 windows of
// 128 B) of its own contiguous region with 8 x 16 B loads per lane, 12 waves per CU:
//   P0 lane-window: lane l reads window l (each instruction touches 64 lines)
//   P1 quads: lanes 4a..4a+3 read 64 contiguous bytes
//   P2 row-quads: lanes m, m+16, m+32, m+48 read 64 contiguous bytes
//   P3 P2 + the permlane16/32_swap transpose that leaves window l in lane l (the k_crc layout)
//   P4 1 KiB contiguous per instruction
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { auto e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d err %d\n", __FILE__, __LINE__, (int)e_); exit(1);} } while (0)

constexpr int kW = 12;

__device__ __forceinline__ uint32_t pat_off(int P, uint32_t lane, int g) {
  if (P == 0) return 128u * lane + 16u * g;
  if (P == 1) return 128u * ((lane >> 2) + 16u * (g >> 1)) + 16u * (4u * (g & 1) + (lane & 3u));
  if (P == 4) return 1024u * g + 16u * lane;
  return 128u * ((lane & 15u) + 16u * (g >> 1)) + 16u * (4u * (g & 1) + (lane >> 4));  // P2, P3
}

// P3: slot g = 2q + hf holds piece 4hf + h of window 16q + m (lane = 16h + m); afterwards slot 2q + hf holds
// piece 4hf + q of window lane
__device__ __forceinline__ void row_transpose(uint32_t (&w)[32]) {
#pragma unroll
  for (int hf = 0; hf < 2; ++hf)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {  // lane bit 4 <-> q bit 0
        uint32_t& x = w[4 * (2 * (2 * r) + hf) + d];
        uint32_t& y = w[4 * (2 * (2 * r + 1) + hf) + d];
        const auto s = __builtin_amdgcn_permlane16_swap(x, y, false, false);
        x = s[0]; y = s[1];
      }
#pragma unroll
      for (int b = 0; b < 2; ++b) {  // lane bit 5 <-> q bit 1
        uint32_t& x = w[4 * (2 * b + hf) + d];
        uint32_t& y = w[4 * (2 * (b + 2) + hf) + d];
        const auto s = __builtin_amdgcn_permlane32_swap(x, y, false, false);
        x = s[0]; y = s[1];
      }
    }
}

template <int P, int VALU = 0>
__global__ __launch_bounds__(64 * kW) void k_pat(const uint8_t* __restrict__ p, uint64_t n, uint32_t* out, int dump) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t gw = (uint64_t)blockIdx.x * kW + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * kW;
  const uint64_t per = (n / 8192) / nw;
  uint32_t acc = 0;
  for (uint64_t it = 0; it < per; ++it) {
    const uint8_t* b = p + (gw * per + it) * 8192;
    uint32_t w[32];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const uint4 v = *reinterpret_cast<const uint4*>(b + pat_off(P, lane, g));
      w[4 * g] = v.x; w[4 * g + 1] = v.y; w[4 * g + 2] = v.z; w[4 * g + 3] = v.w;
    }
    if (P == 3) row_transpose(w);
    if (dump && gw == 0 && it == 0) {  // natural window order: piece 4hf + q from slot 2q + hf
#pragma unroll
      for (int pc = 0; pc < 8; ++pc)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int slot = P == 3 ? 2 * (pc & 3) + (pc >> 2) : pc;
          out[1 + lane * 32 + 4 * pc + d] = w[4 * slot + d];
        }
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) acc = __builtin_amdgcn_alignbyte(acc, acc, 1) ^ w[k];
    // VALU: independent 4-chain busy work per pass (issue pressure beside the loads of the next pass)
    uint32_t c0 = acc, c1 = acc ^ 1u, c2 = acc ^ 2u, c3 = acc ^ 3u;
#pragma unroll
    for (int k = 0; k < VALU / 4; ++k) {
      c0 = __builtin_amdgcn_alignbyte(c0, c1, 1); c1 = __builtin_amdgcn_alignbyte(c1, c2, 2);
      c2 = __builtin_amdgcn_alignbyte(c2, c3, 3); c3 = __builtin_amdgcn_alignbyte(c3, c0, 1);
    }
    acc ^= c0 ^ c1 ^ c2 ^ c3;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <typename F>
static float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const uint64_t n = 1ull << 30;
  std::vector<uint8_t> h(n);
  for (uint64_t i = 0; i < n; ++i) h[i] = (uint8_t)(i * 2654435761ull >> 13);
  uint8_t* d; uint32_t* out;
  CK(hipMalloc(&d, n)); CK(hipMalloc(&out, (1 + 64 * 32) * 4));
  CK(hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice));
  int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  // P3 layout check: lane l holds window l of wave 0's first pass
  k_pat<3><<<cus, 64 * kW>>>(d, n, out, 1);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> o(1 + 64 * 32);
  CK(hipMemcpy(o.data(), out, o.size() * 4, hipMemcpyDeviceToHost));
  const uint64_t per = (n / 8192) / ((uint64_t)cus * kW);
  (void)per;
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int k = 0; k < 32; ++k) {
      uint32_t e; std::memcpy(&e, h.data() + 128 * l + 4 * k, 4);
      if (o[1 + l * 32 + k] != e) ++bad;
    }
  printf("P3 transpose check: %d mismatching words of 2048\n", bad);
  const int reps = 20;
  const char* nm[5] = {"P0 lane-window", "P1 quads", "P2 row-quads", "P3 row-quads+transpose", "P4 1KiB/instr"};
  float t[5];
  t[0] = timeit([&] { k_pat<0><<<cus, 64 * kW>>>(d, n, out, 0); }, reps);
  t[1] = timeit([&] { k_pat<1><<<cus, 64 * kW>>>(d, n, out, 0); }, reps);
  t[2] = timeit([&] { k_pat<2><<<cus, 64 * kW>>>(d, n, out, 0); }, reps);
  t[3] = timeit([&] { k_pat<3><<<cus, 64 * kW>>>(d, n, out, 0); }, reps);
  t[4] = timeit([&] { k_pat<4><<<cus, 64 * kW>>>(d, n, out, 0); }, reps);
  for (int i = 0; i < 5; ++i) printf("%-24s %.4f ms  %.0f GB/s\n", nm[i], t[i], n / (t[i] * 1e-3) / 1e9);
  // load pattern beside VALU work per pass (per wave; 12 waves per CU = 3 per SIMD)
  const float v0 = timeit([&] { k_pat<0, 0><<<cus, 64 * kW>>>(d, n, out, 0); }, reps);
  const float v2 = timeit([&] { k_pat<0, 200><<<cus, 64 * kW>>>(d, n, out, 0); }, reps);
  const float v4 = timeit([&] { k_pat<0, 400><<<cus, 64 * kW>>>(d, n, out, 0); }, reps);
  const float v8 = timeit([&] { k_pat<0, 800><<<cus, 64 * kW>>>(d, n, out, 0); }, reps);
  const float q4 = timeit([&] { k_pat<4, 400><<<cus, 64 * kW>>>(d, n, out, 0); }, reps);
  const float q8 = timeit([&] { k_pat<4, 800><<<cus, 64 * kW>>>(d, n, out, 0); }, reps);
  printf("P0 + VALU per pass: 0 %.4f  200 %.4f  400 %.4f  800 %.4f ms | P4 + 400 %.4f  800 %.4f ms\n", v0, v2, v4, v8,
         q4, q8);
  return 0;
}
