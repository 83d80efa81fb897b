// Copy-pattern probe for the encode writers (not product code): how fast can a wave move bytes between
// arbitrary source and destination alignments on MI355X? Reports GB/s of (read + write) bytes.
//   aligned      uint4 grid-stride copy
//   shift2       misaligned source: two aligned 16 B loads + funnel shift per unit
//   unaligned    misaligned source: one unaligned 16 B load per unit
//   rec*         4190 B records (per-record descriptors, one wave per record, misaligned both sides),
//                descriptor loaded at the record / prefetched one record ahead
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { auto e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d err %d\n", __FILE__, __LINE__, (int)e_); exit(1);} } while (0)

__device__ __forceinline__ uint4 shift16(uint4 v0, uint4 v1, uint32_t sh) {
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

template <int U, bool NT>
__device__ __forceinline__ void st16(uint4* d, uint4 v) {
  if (NT) {
    __builtin_nontemporal_store(v.x, reinterpret_cast<uint32_t*>(d));
    __builtin_nontemporal_store(v.y, reinterpret_cast<uint32_t*>(d) + 1);
    __builtin_nontemporal_store(v.z, reinterpret_cast<uint32_t*>(d) + 2);
    __builtin_nontemporal_store(v.w, reinterpret_cast<uint32_t*>(d) + 3);
  } else {
    *d = v;
  }
}

// MODE 0 aligned, 1 shift2 (src + off), 2 unaligned (src + off)
template <int MODE, int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint64_t nunits,
                                              uint32_t off) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i0 = blockIdx.x * 256ull + threadIdx.x; i0 < nunits; i0 += stride * U) {
    uint4 v[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const uint64_t i = i0 + stride * q;
      if (i < nunits) {
        if (MODE == 0) {
          v[q] = reinterpret_cast<const uint4*>(src)[i];
        } else if (MODE == 1) {
          const uint64_t sa = 16 * i + off;
          const uint4* w = reinterpret_cast<const uint4*>(src + (sa & ~15ull));
          v[q] = shift16(w[0], w[1], (uint32_t)(sa & 15u));
        } else {
          __builtin_memcpy(&v[q], src + 16 * i + off, 16);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const uint64_t i = i0 + stride * q;
      if (i < nunits) st16<U, NT>(reinterpret_cast<uint4*>(dst) + i, v[q]);
    }
  }
}

struct Rec {
  uint64_t s, d;
  uint32_t n, pad;
};

// one wave per record: MODE 1 shift2, 2 unaligned; PF: descriptor prefetched one record ahead
template <int MODE, bool PF, int U>
__global__ __launch_bounds__(256) void k_rec(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                             const Rec* __restrict__ recs, uint64_t nrec) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = (uint64_t)gridDim.x * 4, w0 = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  Rec nx{};
  if (PF && w0 < nrec) nx = recs[w0];
  for (uint64_t j = w0; j < nrec; j += nw) {
    Rec r;
    if (PF) {
      r = nx;
      if (j + nw < nrec) nx = recs[j + nw];
    } else {
      r = recs[j];
    }
    const uint64_t da = (uint64_t)(uintptr_t)(dst + r.d), de = da + r.n;
    const uint64_t u0 = da >> 4, nu = ((de - 1) >> 4) - u0 + 1;
    const uint64_t delta = (uint64_t)(uintptr_t)(src + r.s) - da;
    for (uint64_t k0 = 0; k0 < nu; k0 += 64 * U) {
      uint4 v[U];
      bool full[U];
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const uint64_t k = k0 + 64 * q + lane;
        const uint64_t ua = (u0 + k) << 4, sa = ua + delta;
        full[q] = k < nu && ua >= da && ua + 16 <= de;
        if (full[q]) {
          if (MODE == 1) {
            const uint4* w = reinterpret_cast<const uint4*>((uintptr_t)(sa & ~15ull));
            v[q] = shift16(w[0], w[1], (uint32_t)(sa & 15u));
          } else {
            __builtin_memcpy(&v[q], reinterpret_cast<const void*>((uintptr_t)sa), 16);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const uint64_t k = k0 + 64 * q + lane;
        const uint64_t ua = (u0 + k) << 4;
        if (full[q]) {
          *reinterpret_cast<uint4*>((uintptr_t)ua) = v[q];
        } else if (k < nu) {
          const uint64_t lo = ua > da ? ua : da, hi = ua + 16 < de ? ua + 16 : de;
          for (uint64_t b = lo; b < hi; ++b)
            *reinterpret_cast<uint8_t*>((uintptr_t)b) = *reinterpret_cast<const uint8_t*>((uintptr_t)(b + delta));
        }
      }
    }
  }
}

template <typename F>
static float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const uint64_t n = 4ull << 30;
  uint8_t *s, *d;
  CK(hipMalloc(&s, n + 4096));
  CK(hipMalloc(&d, n + 4096));
  CK(hipMemset(s, 1, n + 4096));
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
  const uint64_t nu = n / 16 - 1;
  const double gb = 2.0 * (double)nu * 16 / 1e9;
  auto rep = [&](const char* name, float ms) { printf("%-34s %8.3f ms  %7.1f GB/s\n", name, ms, gb / (ms / 1e3)); };
  const int R = 5;
  for (int g : {8, 16, 32}) {
    char nm[64];
    snprintf(nm, sizeof nm, "aligned U4 grid %dx", g);
    rep(nm, timeit([&] { k_copy<0, 4, false><<<cus * g, 256>>>(s, d, nu, 0); }, R));
  }
  rep("aligned U4 nt", timeit([&] { k_copy<0, 4, true><<<cus * 16, 256>>>(s, d, nu, 0); }, R));
  rep("aligned U8", timeit([&] { k_copy<0, 8, false><<<cus * 16, 256>>>(s, d, nu, 0); }, R));
  rep("shift2 U4", timeit([&] { k_copy<1, 4, false><<<cus * 16, 256>>>(s, d, nu, 5); }, R));
  rep("shift2 U4 nt", timeit([&] { k_copy<1, 4, true><<<cus * 16, 256>>>(s, d, nu, 5); }, R));
  rep("shift2 U8", timeit([&] { k_copy<1, 8, false><<<cus * 16, 256>>>(s, d, nu, 5); }, R));
  rep("unaligned U4", timeit([&] { k_copy<2, 4, false><<<cus * 16, 256>>>(s, d, nu, 5); }, R));
  rep("unaligned U4 off4", timeit([&] { k_copy<2, 4, false><<<cus * 16, 256>>>(s, d, nu, 4); }, R));
  rep("unaligned U8", timeit([&] { k_copy<2, 8, false><<<cus * 16, 256>>>(s, d, nu, 5); }, R));
  // records: 4190 B each, 7 B headers between them on the destination side
  const uint64_t nrec = n / 4200 - 2;
  Rec* h = (Rec*)malloc(nrec * sizeof(Rec));
  for (uint64_t i = 0; i < nrec; ++i) h[i] = Rec{i * 4197 + 3, i * 4197 + 7 + (i % 5), 4190, 0};
  Rec* dr;
  CK(hipMalloc(&dr, nrec * sizeof(Rec)));
  CK(hipMemcpy(dr, h, nrec * sizeof(Rec), hipMemcpyHostToDevice));
  const double gbr = 2.0 * (double)nrec * 4190 / 1e9;
  auto rep2 = [&](const char* name, float ms) { printf("%-34s %8.3f ms  %7.1f GB/s\n", name, ms, gbr / (ms / 1e3)); };
  for (int g : {4, 8, 16}) {
    char nm[64];
    snprintf(nm, sizeof nm, "rec shift2 pf U4 grid %dx", g);
    rep2(nm, timeit([&] { k_rec<1, true, 4><<<cus * g, 256>>>(s, d, dr, nrec); }, R));
  }
  rep2("rec shift2 nopf U4", timeit([&] { k_rec<1, false, 4><<<cus * 8, 256>>>(s, d, dr, nrec); }, R));
  rep2("rec unaligned pf U4", timeit([&] { k_rec<2, true, 4><<<cus * 8, 256>>>(s, d, dr, nrec); }, R));
  rep2("rec shift2 pf U2", timeit([&] { k_rec<1, true, 2><<<cus * 8, 256>>>(s, d, dr, nrec); }, R));
  return 0;
}
