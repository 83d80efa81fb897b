// bcw_read.hip -- batched point reads: Get / GetV2's record fetch (db_impl.go:567-631)
// = Wal.ReadRecord (wal.go:556-573: WalRecordSize, one read of the record's physical span) +
// WalParseRecord (wal.go:121-173: the fragment walk over that one buffer, optional CRC verify, size
// check) + RecordFromBytes (record.go:140-239), for many (offset, size) requests at once against a WAL
// image resident in HBM.
//
// One wave per request. The fragment headers of a record are walked in order (a record has
// ceil(size / 32761) + 1 of them at most); each fragment's data is copied to the request's payload slot
// by all lanes (16 B units aligned to the destination) and, with verifyChecksum, its CRC-32C is the
// XOR of the lanes' chunk CRCs shifted to the fragment end (shift operators A_{8*2^k}, nibble tables
// in LDS). The record header is then parsed by one lane straight from the segment, through the
// recorded fragment list.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "bcw_internal.h"
#include "bcw_parse.h"

namespace bcw {
namespace rd {

constexpr int kWaves = 4;
constexpr int kMaxF = 64;  // fragments recorded for the header parse (the header lies in the first ones)

__device__ __forceinline__ uint64_t wal_record_size(uint64_t offset, uint64_t size) {
  // WalRecordSize (wal.go:61-86), uint64 arithmetic
  uint64_t left = size, phy = 0;
  offset -= 40;
  while (left > 0) {
    uint64_t leftover = kBlock - (offset % kBlock);
    if (leftover < kHdr) {
      phy += leftover;
      offset += leftover;
      leftover = kBlock;
    }
    const uint64_t frag = left < leftover - kHdr ? left : leftover - kHdr;
    phy += kHdr + frag;
    offset += kHdr + frag;
    left -= frag;
  }
  return phy;
}

__device__ __forceinline__ uint32_t byte_at(const uint8_t* __restrict__ seg, uint64_t n, uint64_t a) {
  return a < n ? seg[a] : 0u;
}

// the payload's bytes through the fragment list recorded in LDS
struct FragReader {
  const uint8_t* seg;
  uint64_t seg_len;
  const uint64_t* fo;  // segment offset of each fragment's data
  const uint32_t* fl;  // its length
  uint32_t nf;
  __device__ __forceinline__ uint32_t operator()(uint64_t pos) const {
    for (uint32_t f = 0; f < nf; ++f) {
      if (pos < fl[f]) return byte_at(seg, seg_len, fo[f] + pos);
      pos -= fl[f];
    }
    return 0;
  }
};

__device__ __forceinline__ uint32_t apply_nib(const uint32_t* __restrict__ t, uint32_t x) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= t[i * 16 + ((x >> (4 * i)) & 15u)];
  return r;
}

struct ReadArgs {
  const uint8_t* seg;
  bcw_read_params p;
  uint64_t n;
  const uint64_t* off;
  const uint64_t* size;
  const uint64_t* pay_off;
  uint8_t* payload;
  uint8_t* rd_status;
  bcw_record_table tab;
  const uint32_t* pow2;   // [kPow2Ops][8][16] nibble images of A_{8 * 2^k}
  const uint32_t* initc;  // A_{8L}(0xFFFFFFFF)
};

__global__ __launch_bounds__(64 * kWaves) void k_read_records(ReadArgs A) {
  __shared__ uint32_t t0[256];
  __shared__ uint32_t sp2[kPow2Ops * 128];  // a fragment is < 2^16 bytes: shifts by up to 65535
  __shared__ uint64_t s_fo[kWaves][kMaxF];
  __shared__ uint32_t s_fl[kWaves][kMaxF];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  for (uint32_t i = tid; i < 256; i += 64 * kWaves) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    t0[i] = c;
  }
  for (uint32_t i = tid; i < kPow2Ops * 128; i += 64 * kWaves) sp2[i] = A.pow2[i];
  __syncthreads();
  const uint64_t r = (uint64_t)blockIdx.x * kWaves + wave;
  if (r >= A.n) return;
  const uint8_t* seg = A.seg;
  const uint64_t n = A.p.seg_len;
  const uint64_t off = A.off[r], size = A.size[r];
  uint8_t* out = A.payload + A.pay_off[r];
  uint32_t st = BCW_RD_OK;
  const uint64_t rs = wal_record_size(off, size);
  uint32_t nf = 0;
  if (off + rs > n || off + rs < off) {
    st = BCW_RD_BEYOND;  // "read beyond file size" (wal.go:562-564)
  } else {
    // WalParseRecord(size, 0, [][]byte{buffer}, verify) with buffer = the file's [off, off + rs)
    uint64_t bo = 0, got = 0;
    for (;;) {
      if (bo + kHdr > rs) { st = BCW_RD_PANIC; break; }  // header := blks[0][blkOff:blkOff+7] out of range
      const uint64_t ha = off + bo;
      const uint32_t crc = byte_at(seg, n, ha) | byte_at(seg, n, ha + 1) << 8 | byte_at(seg, n, ha + 2) << 16 |
                           byte_at(seg, n, ha + 3) << 24;
      const uint64_t len = byte_at(seg, n, ha + 4) | byte_at(seg, n, ha + 5) << 8;
      const uint32_t type = byte_at(seg, n, ha + 6);
      bo += kHdr;
      if (len > rs - bo) { st = BCW_RD_CORRUPTED; break; }  // ErrWalCorruptedData
      const uint64_t ds = off + bo;  // the fragment's data in the segment
      bo += len;
      if (nf < (uint32_t)kMaxF && lane == 0) { s_fo[wave][nf] = ds; s_fl[wave][nf] = (uint32_t)len; }
      ++nf;
      // copy what fits the payload slot (record = append(record, data...); a longer record is a size error)
      const uint64_t cl = got < size ? (len < size - got ? len : size - got) : 0;
      for (uint64_t b = (uint64_t)lane * 16; b < cl; b += 64 * 16) {
        uint8_t tmp[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) tmp[k] = (uint8_t)byte_at(seg, n, ds + b + k);
        const uint64_t m = cl - b < 16 ? cl - b : 16;
        for (uint64_t k = 0; k < m; ++k) out[got + b + k] = tmp[k];
      }
      if (A.p.verify) {
        // lane l: raw CRC-32C (init 0) of its chunk [l*c, min((l+1)*c, len)), shifted to the data end
        const uint64_t c = (len + 63) / 64;
        const uint64_t a0 = (uint64_t)lane * c, a1 = a0 + c < len ? a0 + c : len;
        uint32_t x = 0;
        for (uint64_t q = a0; q < a1; ++q) x = (x >> 8) ^ t0[(x ^ byte_at(seg, n, ds + q)) & 0xffu];
        if (a0 < a1) {
          uint64_t dsh = len - a1;  // zero bytes after the chunk
          for (int k = 0; dsh; ++k, dsh >>= 1)
            if (dsh & 1u) x = apply_nib(sp2 + k * 128, x);
        } else {
          x = 0;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) x ^= (uint32_t)__shfl_xor((int)x, d, 64);
        // the init contribution A_{8L}(~0): the table up to one block, beyond (crafted lengths) by shifts
        uint32_t ic = A.initc[len <= kBlock ? len : kBlock];
        for (uint64_t dsh = len > kBlock ? len - kBlock : 0, k = 0; dsh; ++k, dsh >>= 1)
          if (dsh & 1u) ic = apply_nib(sp2 + k * 128, ic);
        const uint32_t c32 = ~(x ^ ic);  // CRC-32C = ~crc_update(~0, data)
        const uint32_t masked = ((c32 >> 15) | (c32 << 17)) + 0xa282ead8u;  // ComputeCRC32 (utils.go:24-29)
        if (masked != crc) { st = BCW_RD_CRC; break; }
      }
      got += len;
      if (type == BCW_RECORD_FULL || type == BCW_RECORD_LAST) {
        if (got != size) st = BCW_RD_SIZE;  // ErrWalMismatchSize
        break;
      }
      if (type != BCW_RECORD_FIRST && type != BCW_RECORD_MIDDLE) { st = BCW_RD_TYPE; break; }
      if (rs - bo <= kHdr) { st = BCW_RD_INCOMPLETE; break; }  // leftover <= 7: the block loop ends
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane != 0) return;
  A.rd_status[r] = (uint8_t)st;
  if (!A.tab.status) return;
  bcw_decode_params dp{};
  dp.seg_len = n;
  dp.base_time = A.p.base_time;
  dp.ns_size = A.p.ns_size;
  dp.etag_size = A.p.etag_size;
  dp.mode = BCW_MODE_RECORD;
  uint8_t status = BCW_ST_OK, hdr = 0, flags = 0, etag_off = 0;
  uint64_t kl = 0, vl = 0, ml = 0, expire = 0, x0 = 0, x1 = 0;
  if (st == BCW_RD_OK) {
    FragReader fr{seg, n, s_fo[wave], s_fl[wave], nf < (uint32_t)kMaxF ? nf : (uint32_t)kMaxF};
    parse_record(dp, fr, size, status, hdr, flags, etag_off, kl, vl, ml, expire, x0, x1);
  }
  const bcw_record_table& t = A.tab;
  if (r >= t.capacity) return;
  t.foff[r] = off + kHdr;
  t.size[r] = size;
  t.expire[r] = expire;
  t.key_len[r] = (uint32_t)kl;
  t.val_len[r] = (uint32_t)vl;
  t.meta_len[r] = (uint32_t)ml;
  if (t.first_frag) t.first_frag[r] = 0;
  if (t.emit_frag) t.emit_frag[r] = nf ? nf - 1 : 0;
  t.hdr_size[r] = hdr;
  t.flags[r] = flags;
  t.etag_off[r] = etag_off;
  t.status[r] = status;
}

}  // namespace rd

hipError_t launch_read_records(const rd::ReadArgs& A, hipStream_t st) {
  if (A.n == 0) return hipSuccess;
  rd::k_read_records<<<(uint32_t)((A.n + rd::kWaves - 1) / rd::kWaves), 64 * rd::kWaves, 0, st>>>(A);
  return hipGetLastError();
}

}  // namespace bcw

using namespace bcw;

extern "C" {

int bcw_read_records_async(bcw_ctx* c, const uint8_t* d_seg, const bcw_read_params* p, uint64_t n,
                           const uint64_t* d_off, const uint64_t* d_size, const uint64_t* d_pay_off, uint8_t* d_payload,
                           uint8_t* d_rd_status, const bcw_record_table* d_table) {
  if (!c || !p || (n && (!d_seg || !d_off || !d_size || !d_pay_off || !d_payload || !d_rd_status))) return BCW_E_INVAL;
  if (d_table && d_table->status && (!d_table->foff || !d_table->size || !d_table->expire || !d_table->key_len ||
                                     !d_table->val_len || !d_table->meta_len || !d_table->hdr_size ||
                                     !d_table->flags || !d_table->etag_off))
    return BCW_E_INVAL;
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  rd::ReadArgs A{};
  A.seg = d_seg;
  A.p = *p;
  A.n = n;
  A.off = d_off;
  A.size = d_size;
  A.pay_off = d_pay_off;
  A.payload = d_payload;
  A.rd_status = d_rd_status;
  if (d_table) A.tab = *d_table;
  A.pow2 = c->tabs.pow2;
  A.initc = c->tabs.initc;
  return launch_read_records(A, c->cur) == hipSuccess ? BCW_OK : BCW_E_HIP;
}

int bcw_read_records(bcw_ctx* c, const uint8_t* h_seg, const bcw_read_params* p, uint64_t n, const uint64_t* h_off,
                     const uint64_t* h_size, uint8_t* h_payload, uint8_t* h_rd_status, const bcw_record_table* h_table) {
  if (!c || !p || (n && (!h_off || !h_size || !h_payload || !h_rd_status)) || (p->seg_len && !h_seg))
    return BCW_E_INVAL;
  if (n == 0) return BCW_OK;
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  std::vector<uint64_t> pay(n + 1, 0);
  for (uint64_t i = 0; i < n; ++i) pay[i + 1] = pay[i] + h_size[i];
  const uint64_t pb = (pay[n] + 15) & ~15ull, sb = (p->seg_len + 15) & ~15ull;
  const bool tab = h_table && h_table->status;
  const uint64_t tb = tab ? n * 64 : 0;
  void* mem = nullptr;
  if (hipMalloc(&mem, sb + pb + 8 * (3 * n + 1) + n + tb + 64) != hipSuccess) return BCW_E_NOMEM;
  uint8_t* m = (uint8_t*)mem;
  uint8_t* d_seg = m; m += sb;
  uint8_t* d_pay = m; m += pb;
  uint64_t* d_off = (uint64_t*)m; m += 8 * n;
  uint64_t* d_size = (uint64_t*)m; m += 8 * n;
  uint64_t* d_pay_off = (uint64_t*)m; m += 8 * (n + 1);
  bcw_record_table dt{};
  if (tab) {
    dt.capacity = n;
    dt.foff = (uint64_t*)m; m += 8 * n;
    dt.size = (uint64_t*)m; m += 8 * n;
    dt.expire = (uint64_t*)m; m += 8 * n;
    dt.key_len = (uint32_t*)m; m += 4 * n;
    dt.val_len = (uint32_t*)m; m += 4 * n;
    dt.meta_len = (uint32_t*)m; m += 4 * n;
    dt.first_frag = (uint32_t*)m; m += 4 * n;
    dt.emit_frag = (uint32_t*)m; m += 4 * n;
    dt.hdr_size = m; m += n;
    dt.flags = m; m += n;
    dt.etag_off = m; m += n;
    dt.status = m; m += n;
  }
  uint8_t* d_st = m;
  hipStream_t st = c->cur;
  bool ok = (p->seg_len == 0 || hipMemcpyAsync(d_seg, h_seg, p->seg_len, hipMemcpyHostToDevice, st) == hipSuccess) &&
            hipMemcpyAsync(d_off, h_off, 8 * n, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(d_size, h_size, 8 * n, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(d_pay_off, pay.data(), 8 * (n + 1), hipMemcpyHostToDevice, st) == hipSuccess;
  ok = ok && bcw_read_records_async(c, d_seg, p, n, d_off, d_size, d_pay_off, d_pay, d_st, tab ? &dt : nullptr) == BCW_OK;
  ok = ok && (pay[n] == 0 || hipMemcpyAsync(h_payload, d_pay, pay[n], hipMemcpyDeviceToHost, st) == hipSuccess) &&
       hipMemcpyAsync(h_rd_status, d_st, n, hipMemcpyDeviceToHost, st) == hipSuccess;
  if (ok && tab) {
    const uint64_t k = std::min(n, h_table->capacity);
    auto cp = [&](void* dst, const void* src, size_t esz) {
      return !dst || hipMemcpyAsync(dst, src, k * esz, hipMemcpyDeviceToHost, st) == hipSuccess;
    };
    ok = cp(h_table->foff, dt.foff, 8) && cp(h_table->size, dt.size, 8) && cp(h_table->expire, dt.expire, 8) &&
         cp(h_table->key_len, dt.key_len, 4) && cp(h_table->val_len, dt.val_len, 4) &&
         cp(h_table->meta_len, dt.meta_len, 4) && cp(h_table->first_frag, dt.first_frag, 4) &&
         cp(h_table->emit_frag, dt.emit_frag, 4) && cp(h_table->hdr_size, dt.hdr_size, 1) &&
         cp(h_table->flags, dt.flags, 1) && cp(h_table->etag_off, dt.etag_off, 1) && cp(h_table->status, dt.status, 1);
  }
  ok = ok && hipStreamSynchronize(st) == hipSuccess;
  (void)hipFree(mem);
  return ok ? BCW_OK : BCW_E_HIP;
}

}  // extern "C"
