// bcw_index.hip -- the bitcaskDB index (index.go) resident in HBM, for the two callers of the WAL
// codec that consult it: the compaction filter (doFilter, compaction.go:329-348) and
// the index rebuild from hint / data WALs (recoverFromWal db_impl.go:286-313, onePhase
// compaction.go:248-251; §8 f2).
//
// What is restated is the index's observable behaviour (index.go:81-165 over map.go's ShardMap): a map
// from MergedKey(ns, key) = ns || key (utils.go:133-139) to IndexValue{fid, valueOff, valueSize}, keyed by
// IndexOperator.Hash = murmur3 Sum64 (index.go:15-19, spaolacci/murmur3 v1.1.0); Put replaces, Delete
// removes, SoftDelete stores {0, 0, 0}, Get reports ErrKeyNotFound / ErrKeySoftDeleted (valueOff == 0).
// Bucket placement is unobservable; the reference's sampled approximate-LRU eviction (random slots,
// map.go:395-420) is not restated -- the device index holds every key (capacity grows instead).
//
// Layout (HBM): an open-addressing slot table (64 B slots, power-of-two capacity, linear probing from
// the hash) and a grow-only key arena of {hash, length, key bytes padded to 16} entries.
// A batch of operations (host-supplied, or every delivered row of a decoded record / hint table) runs
// as five stream-ordered launches, so every cross-workgroup hand-off is a kernel boundary:
//   k_ix_keys   one lane per op: murmur3 over the merged key's 16 B chunks (gathered from the WAL segment
//               when the ops come from a decoded table)
//   k_ix_claim  probe from the hash: find the slot holding the key (arena compare), or claim an empty
//               slot with a 64-bit CAS of a provisional reference to the op itself (ops of the batch
//               compare their keys straight from the source); an op that finds its key records the
//               value it replaces (WriteStat)
//   k_ix_seq    atomicMax of the op's sequence number into its slot: the last op of a key wins, as
//               in the reference's sequential loop
//   k_ix_commit the op that claimed a slot copies its key into the arena and makes the slot's reference
//               permanent: only keys new to the index take arena space (a rebuild over existing keys
//               takes none)
//   k_ix_write  the winning op writes the value / presence
// Lookups (Get, the compaction filter) are one launch: hash, probe, compare.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "bcw_internal.h"

namespace bcw {
namespace ix {

struct Slot {
  uint64_t kref;  // 0: empty; 1 + arena offset of the key entry; kProv | op: claimed by op of the running batch
  uint64_t seq;   // sequence number of the last op applied to this key
  uint64_t hash;  // murmur3 Sum64 of the merged key
  uint64_t fid, off, size;
  uint64_t live;  // 1: present (Put, SoftDelete); 0: absent (Delete)
  uint64_t pad;
};
static_assert(sizeof(Slot) == 64, "Slot layout");

constexpr uint64_t kProv = 1ull << 63;  // provisional slot reference (claim -> commit inside one batch)

// device counters (C_NEED: arena bytes the rows of a decoded table would take, k_ix_need)
// C_EVICTED / C_EVICTED_BYTES: keys evicted by the capacity bound (k_ix_evict) and the sum of their value sizes
enum { C_ARENA = 0, C_SLOTS = 1, C_LIVE = 2, C_OVERFLOW = 3, C_NIN = 4, C_DONE = 5, C_FAIL = 6, C_NEED = 7,
       C_EVICTED = 8, C_EVICTED_BYTES = 9, C_NUM = 10 };

// op sources
enum { SRC_FLAT = 0, SRC_RECORD = 1, SRC_HINT = 2 };

struct Src {
  int kind;
  // flat: merged keys concatenated, key i = keys[koff[i], koff[i+1])
  const uint8_t* keys;
  const uint64_t* koff;
  uint64_t keys_len;
  // decoded table: the segment, its fragment table and record table
  const uint8_t* seg;
  uint64_t seg_len;
  const Frag* frags;
  bcw_record_table t;
  uint32_t start_off, ns;
};

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}
// MurmurHash3_x64_128 (seed 0) fed 16-byte blocks; Sum64 = h1
struct Murmur {
  uint64_t h1 = 0, h2 = 0;
  __device__ __forceinline__ void block(uint64_t k1, uint64_t k2) {
    const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
  }
  // tail of t = n & 15 bytes, zero-padded into k1 (bytes 0-7) and k2 (bytes 8-15)
  __device__ __forceinline__ uint64_t finish(uint64_t k1, uint64_t k2, uint32_t t, uint64_t n) {
    const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
    if (t > 8) { k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2; }
    if (t > 0) { k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1; }
    h1 ^= n; h2 ^= n;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2;
    return h1;
  }
};

__device__ __forceinline__ uint4 shift16(uint4 v0, uint4 v1, uint32_t sh) {
  const bool s2 = (sh & 8u) != 0, s1 = (sh & 4u) != 0;
  const uint32_t b0 = s2 ? v0.z : v0.x, b1 = s2 ? v0.w : v0.y, b2 = s2 ? v1.x : v0.z, b3 = s2 ? v1.y : v0.w,
                 b4 = s2 ? v1.z : v1.x, b5 = s2 ? v1.w : v1.y;
  const uint32_t c0 = s1 ? b1 : b0, c1 = s1 ? b2 : b1, c2 = s1 ? b3 : b2, c3 = s1 ? b4 : b3, c4 = s1 ? b5 : b4;
  const uint32_t b = sh & 3u;
  return make_uint4(__builtin_amdgcn_alignbyte(c1, c0, b), __builtin_amdgcn_alignbyte(c2, c1, b),
                    __builtin_amdgcn_alignbyte(c3, c2, b), __builtin_amdgcn_alignbyte(c4, c3, b));
}
// 16 bytes of buf at signed offset a; bytes outside [0, n) read as 0
__device__ __forceinline__ uint4 load16u(const uint8_t* __restrict__ buf, uint64_t n, int64_t a) {
  if (a >= 0 && (uint64_t)(a & ~15ll) + 32 <= n) {
    const uint8_t* p = buf + (a & ~15ll);
    return shift16(*reinterpret_cast<const uint4*>(p), *reinterpret_cast<const uint4*>(p + 16), (uint32_t)(a & 15));
  }
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll 1
  for (int i = 0; i < 16; ++i) {
    const int64_t q = a + i;
    const uint32_t by = (q >= 0 && (uint64_t)q < n) ? buf[q] : 0u;
    w[i >> 2] |= by << (8 * (i & 3));
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}
// bytes [lo, hi) of a 16 B unit
__device__ __forceinline__ uint4 keep_bytes(uint4 v, int32_t lo, int32_t hi) {
  uint32_t m[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int32_t a = min(max(lo - 4 * k, 0), 4), b = min(max(hi - 4 * k, 0), 4);
    m[k] = (uint32_t)(((1ull << (8 * b)) - 1) & ~((1ull << (8 * a)) - 1));
  }
  return make_uint4(v.x & m[0], v.y & m[1], v.z & m[2], v.w & m[3]);
}
__device__ __forceinline__ uint4 or4(uint4 a, uint4 b) { return make_uint4(a.x | b.x, a.y | b.y, a.z | b.z, a.w | b.w); }

// One op's merged key: up to two byte ranges (ns, key) of a flat buffer or of a record payload.
struct Key {
  uint32_t la, lb;   // range lengths (merged key = A || B)
  int64_t a0, b0;    // start of A / B: flat -> buffer offset; payload -> file offset when contiguous
  bool ca, cb;       // the range is contiguous in the buffer (always, for flat keys)
  uint32_t pa, pb;   // payload offsets of A / B (slow path)
  uint32_t f0, f1;   // the payload's fragments
  bool ok;           // false: the row is not a delivered OK record (no key)
  __device__ __forceinline__ uint32_t len() const { return la + lb; }
};

// payload offset z of a record whose bytes are the data of fragments [f0, f1]
__device__ uint8_t payload_byte(const Src& s, uint32_t f0, uint32_t f1, uint64_t z) {
  uint32_t f = f0;
  for (;;) {
    const Frag F = s.frags[f];
    if (z < F.len || f >= f1) {
      const uint64_t a = (uint64_t)s.start_off + (uint64_t)F.blk * kBlock + F.start + z;
      return a < s.seg_len ? s.seg[a] : 0;
    }
    z -= F.len;
    ++f;
  }
}

__device__ __forceinline__ Key make_key(const Src& s, uint64_t i) {
  Key k{};
  k.ok = true;
  if (s.kind == SRC_FLAT) {
    const uint64_t a = s.koff[i], b = s.koff[i + 1];
    k.la = (uint32_t)(b - a);
    k.lb = 0;
    k.a0 = (int64_t)a;
    k.b0 = (int64_t)b;
    k.ca = k.cb = true;
    return k;
  }
  const bcw_record_table& t = s.t;
  k.f1 = t.emit_frag[i];
  k.f0 = t.first_frag[i];
  const Frag F0 = s.frags[k.f0];
  const Frag F1 = s.frags[k.f1];
  if (F1.type == BCW_RECORD_FULL) k.f0 = k.f1;  // a Full emission carries only its own data
  const Frag Fa = k.f0 == k.f1 ? F1 : F0;
  const uint64_t d0 = (uint64_t)s.start_off + (uint64_t)Fa.blk * kBlock + Fa.start;
  const uint32_t l0 = Fa.len;
  k.la = s.ns;
  k.pa = s.kind == SRC_RECORD ? 1u : 0u;  // RecordFromBytes: data[1:1+NsSize]; HintRecord: data[0:NsSize]
  k.lb = t.key_len[i];
  k.pb = t.hdr_size[i];                   // record: headerSize (key offset); hint: key offset mod 256
  if (s.kind == SRC_HINT && s.ns > 245u) {
    // the hint key offset NsSize + len(uvarint keyLen) (hint.go:62-66) no longer fits the table's u8 column:
    // count the varint's bytes in the payload (HintRecord.Decode accepted it, so it ends within 10 bytes)
    uint32_t u = 1;
    while (u < 10u && (payload_byte(s, k.f0, k.f1, (uint64_t)s.ns + u - 1) & 0x80u)) ++u;
    k.pb = s.ns + u;
  }
  k.ca = (uint64_t)k.pa + k.la <= l0;
  k.cb = (uint64_t)k.pb + k.lb <= l0;
  k.a0 = (int64_t)(d0 + k.pa);
  k.b0 = (int64_t)(d0 + k.pb);
  return k;
}

// chunk c (merged bytes [16c, 16c + 16), zero beyond the key) of op i's key
__device__ __forceinline__ uint4 key_chunk(const Src& s, const Key& k, uint32_t c) {
  const int32_t m0 = (int32_t)(16 * c);
  const int32_t L = (int32_t)k.len();
  uint4 v = make_uint4(0, 0, 0, 0);
  const uint8_t* buf = s.kind == SRC_FLAT ? s.keys : s.seg;
  const uint64_t n = s.kind == SRC_FLAT ? s.keys_len : s.seg_len;
  if (m0 < (int32_t)k.la) {  // part of A: merged [m0, min(la, m0 + 16))
    const int32_t hi = min((int32_t)k.la - m0, 16);
    if (k.ca) {
      v = keep_bytes(load16u(buf, n, k.a0 + m0), 0, hi);
    } else {
      uint32_t w[4] = {0, 0, 0, 0};
      for (int32_t b = 0; b < hi; ++b)
        w[b >> 2] |= (uint32_t)payload_byte(s, k.f0, k.f1, k.pa + (uint64_t)(m0 + b)) << (8 * (b & 3));
      v = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
  if (m0 + 16 > (int32_t)k.la && m0 < L) {  // part of B: merged [max(la, m0), min(L, m0 + 16))
    const int32_t lo = max((int32_t)k.la - m0, 0), hi = min(L - m0, 16);
    if (k.cb) {
      v = or4(v, keep_bytes(load16u(buf, n, k.b0 + (m0 - (int32_t)k.la)), lo, hi));
    } else {
      uint32_t w[4] = {0, 0, 0, 0};
      for (int32_t b = lo; b < hi; ++b)
        w[b >> 2] |= (uint32_t)payload_byte(s, k.f0, k.f1, k.pb + (uint64_t)(m0 + b - (int32_t)k.la)) << (8 * (b & 3));
      v = or4(v, make_uint4(w[0], w[1], w[2], w[3]));
    }
  }
  return v;
}

__device__ __forceinline__ uint64_t key_hash(const Src& s, const Key& k) {
  Murmur m;
  const uint32_t L = k.len(), nb = L / 16, t = L & 15u;
  for (uint32_t c = 0; c < nb; ++c) {
    const uint4 v = key_chunk(s, k, c);
    m.block((uint64_t)v.x | ((uint64_t)v.y << 32), (uint64_t)v.z | ((uint64_t)v.w << 32));
  }
  uint4 v = make_uint4(0, 0, 0, 0);
  if (t) v = key_chunk(s, k, nb);
  return m.finish((uint64_t)v.x | ((uint64_t)v.y << 32), (uint64_t)v.z | ((uint64_t)v.w << 32), t, L);
}

// rows of a decoded table that IterateRecord / IterateHint deliver to the callback: those before the
// first row RecordFromBytes / HintRecord.Decode rejects (record.go:246-263, hint.go:174-185)
__device__ __forceinline__ uint64_t delivered_rows(const bcw_decode_result* R) {
  const uint64_t nrec = R->n_records;
  return (R->first_bad_record >= 0 && (uint64_t)R->first_bad_record < nrec) ? (uint64_t)R->first_bad_record : nrec;
}

// the table source is usable: the context's latest decode (its fragment table), not truncated, and not a decode
// that gave up on an internal wait (BCW_ERR_INTERNAL: its rows, if any, are not to be applied)
__device__ __forceinline__ uint32_t table_fail(const bcw_decode_result* R, uint64_t gen, uint64_t rows) {
  return R->generation != gen ? BCW_ENC_ERR_STALE
         : (R->n_records > rows || R->err_class == BCW_ERR_INTERNAL) ? BCW_ENC_ERR_TABLE : 0u;
}

// wave-aggregated add of v to *ctr; returns this lane's exclusive offset
__device__ __forceinline__ uint64_t wave_alloc(uint64_t* ctr, uint64_t v) {
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t t = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += t;
  }
  const uint64_t tot = __shfl(incl, 63, 64);
  uint64_t base = 0;
  if (lane == 63 && tot) base = atomicAdd(reinterpret_cast<unsigned long long*>(ctr), (unsigned long long)tot);
  base = __shfl(base, 63, 64);
  return base + incl - v;
}

// ---- batch launch 1: key hashes ----------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ix_keys(Src s, uint64_t n, const bcw_decode_result* __restrict__ R,
                                                 uint64_t gen, uint64_t* __restrict__ cnt,
                                                 uint64_t* __restrict__ op_kref, uint64_t* __restrict__ op_hash) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  uint64_t nin = n;
  if (s.kind != SRC_FLAT) {
    const uint32_t fail = table_fail(R, gen, n);
    nin = fail ? 0 : delivered_rows(R);
    if (i == 0) { cnt[C_NIN] = nin; cnt[C_FAIL] = fail; }
  }
  if (i >= nin) return;
  const Key k = make_key(s, i);
  op_hash[i] = key_hash(s, k);
  op_kref[i] = kProv | i;  // the op's own provisional reference (its key is read from the source)
}

// the arena entry at offset a holds op k's key (length L)
__device__ __forceinline__ bool arena_matches(const Src& s, const Key& k, const uint8_t* __restrict__ arena,
                                              uint64_t a, uint32_t L) {
  const uint4* q = reinterpret_cast<const uint4*>(arena + a + 16);
  for (uint32_t c = 0; c < (L + 15) / 16; ++c) {
    const uint4 x = key_chunk(s, k, c), y = q[c];
    if (x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w) return false;
  }
  return true;
}
// ops k and kj of the batch have the same key (lengths equal)
__device__ __forceinline__ bool keys_match(const Src& s, const Key& k, const Key& kj, uint32_t L) {
  for (uint32_t c = 0; c < (L + 15) / 16; ++c) {
    const uint4 x = key_chunk(s, k, c), y = key_chunk(s, kj, c);
    if (x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w) return false;
  }
  return true;
}

// ---- batch launch 2: find or claim each op's slot --------------------------------------------------
// old_*: per op, the value the slot held before the batch when the key existed (WriteStat of the key's first
// op in the batch; the host composes the later ones, bcw_index_apply_stat)
__global__ __launch_bounds__(256) void k_ix_claim(Src s, uint64_t n, const uint64_t* __restrict__ cnt_in,
                                                  Slot* __restrict__ slots, uint64_t mask,
                                                  const uint8_t* __restrict__ arena, uint64_t* __restrict__ cnt,
                                                  const uint64_t* __restrict__ op_kref,
                                                  const uint64_t* __restrict__ op_hash, uint64_t* __restrict__ op_slot,
                                                  uint8_t* __restrict__ old_found, uint64_t* __restrict__ old_fid,
                                                  uint64_t* __restrict__ old_size) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t nin = s.kind == SRC_FLAT ? n : cnt_in[C_NIN];
  bool claimed = false;
  if (i < nin) {
    uint64_t slot = ~0ull;
    uint8_t found = 0;
    uint64_t ofid = 0, osize = 0;
    if (op_kref[i]) {
      const uint64_t h = op_hash[i];
      const Key k = make_key(s, i);
      const uint32_t L = k.len();
      uint64_t j = h & mask;
      for (uint64_t probe = 0; probe <= mask; ++probe, j = (j + 1) & mask) {
        uint64_t c = __hip_atomic_load(&slots[j].kref, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (c == 0) {
          c = atomicCAS(reinterpret_cast<unsigned long long*>(&slots[j].kref), 0ull, (unsigned long long)(kProv | i));
          if (c == 0) { slot = j; claimed = true; break; }
        }
        if (c & kProv) {  // claimed by another op of this batch: compare with its key at the source
          const uint64_t o = c & ~kProv;
          if (op_hash[o] != h) continue;
          const Key ko = make_key(s, o);
          if (ko.len() == L && keys_match(s, k, ko, L)) { slot = j; break; }
        } else {
          const uint4 hd = *reinterpret_cast<const uint4*>(arena + (c - 1));
          if (((uint64_t)hd.x | ((uint64_t)hd.y << 32)) == h && hd.z == L && arena_matches(s, k, arena, c - 1, L)) {
            slot = j;
            const Slot S = slots[j];  // values are only written by k_ix_write, after this launch
            if (S.live) { found = 1; ofid = S.fid; osize = S.size; }
            break;
          }
        }
      }
      if (slot == ~0ull) atomicOr(reinterpret_cast<unsigned long long*>(&cnt[C_OVERFLOW]), 2ull);
    }
    op_slot[i] = slot;
    if (old_found) { old_found[i] = found; old_fid[i] = ofid; old_size[i] = osize; }
  }
  (void)wave_alloc(&cnt[C_SLOTS], claimed ? 1ull : 0ull);
}

// ---- batch launch 3: the last op of each key wins ----------------------------------------------------
__global__ __launch_bounds__(256) void k_ix_seq(uint64_t n, const uint64_t* __restrict__ cnt_in, int flat,
                                                Slot* __restrict__ slots, const uint64_t* __restrict__ op_slot,
                                                uint64_t seq_base) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t nin = flat ? n : cnt_in[C_NIN];
  if (i >= nin) return;
  const uint64_t s = op_slot[i];
  if (s == ~0ull) return;
  atomicMax(reinterpret_cast<unsigned long long*>(&slots[s].seq), (unsigned long long)(seq_base + i));
}

// ---- batch launch 4: the claiming op copies its key into the arena ------------------------------------
__global__ __launch_bounds__(256) void k_ix_commit(Src s, uint64_t n, uint64_t* __restrict__ cnt,
                                                   Slot* __restrict__ slots, uint8_t* __restrict__ arena,
                                                   uint64_t arena_cap, const uint64_t* __restrict__ op_hash,
                                                   const uint64_t* __restrict__ op_slot) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t nin = s.kind == SRC_FLAT ? n : cnt[C_NIN];
  bool own = false;
  uint64_t sl = ~0ull;
  Key k{};
  if (i < nin) {
    sl = op_slot[i];
    own = sl != ~0ull && slots[sl].kref == (kProv | i);
    if (own) k = make_key(s, i);
  }
  const uint64_t esz = own ? 16ull + (((uint64_t)k.len() + 15) & ~15ull) : 0;
  const uint64_t a = wave_alloc(&cnt[C_ARENA], esz);
  if (!own) return;
  if (a + esz > arena_cap) {  // the host sizes the arena before the launch; never expected
    atomicOr(reinterpret_cast<unsigned long long*>(&cnt[C_OVERFLOW]), 1ull);
    slots[sl].kref = 0;
    return;
  }
  uint8_t* e = arena + a;
  const uint32_t L = k.len();
  for (uint32_t c = 0; c < (L + 15) / 16; ++c) *reinterpret_cast<uint4*>(e + 16 + 16 * c) = key_chunk(s, k, c);
  const uint64_t h = op_hash[i];
  *reinterpret_cast<uint4*>(e) = make_uint4((uint32_t)h, (uint32_t)(h >> 32), L, 0u);
  slots[sl].hash = h;
  slots[sl].kref = a + 1;
}

// arena bytes the delivered rows of a decoded table would take if every key were new (the exact bound the
// host reads when its cheap bound does not fit the arena)
__global__ __launch_bounds__(256) void k_ix_need(Src s, uint64_t rows, const bcw_decode_result* __restrict__ R,
                                                 uint64_t gen, uint64_t* __restrict__ cnt) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t nin = table_fail(R, gen, rows) ? 0 : delivered_rows(R);
  uint64_t b = 0;
  if (i < nin) b = 16ull + (((uint64_t)s.ns + s.t.key_len[i] + 15) & ~15ull);
  (void)wave_alloc(&cnt[C_NEED], b);
}

// ---- batch launch 5: values ---------------------------------------------------------------------------
struct OpVals {
  // flat ops (host arrays copied to the device): op code and value per op
  const uint8_t* op;
  const uint64_t* fid;
  const uint64_t* off;
  const uint64_t* size;
  // table ops: value columns (PUT of every delivered row)
  uint64_t file_fid;
  int use_rec_fid;
};

__global__ __launch_bounds__(256) void k_ix_write(Src s, uint64_t n, uint64_t* __restrict__ cnt, OpVals v,
                                                  Slot* __restrict__ slots, const uint64_t* __restrict__ op_slot,
                                                  uint64_t seq_base) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  const bool flat = s.kind == SRC_FLAT;
  const uint64_t nin = flat ? n : cnt[C_NIN];
  int64_t dlive = 0;
  uint64_t done = 0;
  if (i < nin) {
    const uint64_t sl = op_slot[i];
    if (sl != ~0ull &&
        __hip_atomic_load(&slots[sl].seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == seq_base + i) {
      Slot& S = slots[sl];
      uint32_t op = BCW_IDX_PUT;
      uint64_t fid = 0, off = 0, size = 0;
      if (flat) {
        op = v.op[i];
        fid = v.fid[i];
        off = v.off[i];
        size = v.size[i];
      } else if (s.kind == SRC_RECORD) {
        fid = v.file_fid;                       // db_impl.go:307-313: Put(ns, key, wal.Fid(), foff - 7, size)
        off = s.t.foff[i] - kHdr;
        size = s.t.size[i];
      } else {
        fid = v.use_rec_fid ? s.t.expire[i] : v.file_fid;  // compaction.go:250 (record.fid) / db_impl.go:297 (fid)
        off = s.t.aux0[i];
        size = s.t.aux1[i];
      }
      const uint64_t was = S.live;
      if (op == BCW_IDX_DELETE) {
        S.live = 0;
      } else {
        if (op == BCW_IDX_SOFT_DELETE) fid = off = size = 0;  // IndexValue{valueOff: 0} (index.go:128-130)
        S.fid = fid;
        S.off = off;
        S.size = size;
        S.live = 1;
      }
      dlive = (int64_t)S.live - (int64_t)was;
    }
    done = 1;
  }
  (void)wave_alloc(&cnt[C_LIVE], (uint64_t)dlive);
  (void)wave_alloc(&cnt[C_DONE], done);
}

// ---- lookups -----------------------------------------------------------------------------------------
// the slot holding op i's key, or ~0
__device__ __forceinline__ uint64_t find_slot(const Src& s, const Key& k, uint64_t h, const Slot* __restrict__ slots,
                                              uint64_t mask, const uint8_t* __restrict__ arena) {
  const uint32_t L = k.len();
  uint64_t j = h & mask;
  for (uint64_t probe = 0; probe <= mask; ++probe, j = (j + 1) & mask) {
    const uint64_t kr = slots[j].kref;
    if (kr == 0) return ~0ull;
    if (slots[j].hash != h) continue;
    const uint4 hd = *reinterpret_cast<const uint4*>(arena + (kr - 1));
    if (hd.z != L) continue;
    const uint4* q = reinterpret_cast<const uint4*>(arena + (kr - 1) + 16);
    bool eq = true;
    for (uint32_t c = 0; c < (L + 15) / 16 && eq; ++c) {
      const uint4 x = key_chunk(s, k, c), y = q[c];
      eq = x.x == y.x && x.y == y.y && x.z == y.z && x.w == y.w;
    }
    if (eq) return j;
  }
  return ~0ull;
}

// Index.Get (index.go:81-98) of flat keys
__global__ __launch_bounds__(256) void k_ix_get(Src s, uint64_t n, const Slot* __restrict__ slots, uint64_t mask,
                                                const uint8_t* __restrict__ arena, uint64_t* __restrict__ fid,
                                                uint64_t* __restrict__ off, uint64_t* __restrict__ size,
                                                uint8_t* __restrict__ status) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n) return;
  const Key k = make_key(s, i);
  const uint64_t h = key_hash(s, k);
  const uint64_t j = find_slot(s, k, h, slots, mask, arena);
  uint8_t st = BCW_IDX_NOT_FOUND;
  uint64_t f = 0, o = 0, z = 0;
  if (j != ~0ull && slots[j].live) {
    f = slots[j].fid;
    o = slots[j].off;
    z = slots[j].size;
    st = o == 0 ? BCW_IDX_SOFT_DELETED : BCW_IDX_FOUND;
  }
  fid[i] = f;
  off[i] = o;
  size[i] = z;
  status[i] = st;
}

// compactOneWal's doFilter (compaction.go:329-348, without the user CompactionFilter) of every delivered
// row of a decoded data WAL: keep = Get succeeds (not deleted / soft-deleted) and still points at
// (src fid, foff - 7) (compaction.go:302); rows the iteration does not deliver get 0
__global__ __launch_bounds__(256) void k_ix_filter(Src s, uint64_t rows, const bcw_decode_result* __restrict__ R,
                                                   uint64_t gen, const Slot* __restrict__ slots, uint64_t mask,
                                                   const uint8_t* __restrict__ arena, uint64_t src_fid,
                                                   uint8_t* __restrict__ keep, uint64_t* __restrict__ cnt) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  const uint32_t fail = table_fail(R, gen, rows);
  const uint64_t nin = fail ? 0 : delivered_rows(R);
  if (i == 0) { cnt[C_NIN] = nin; cnt[C_FAIL] = fail; }
  uint8_t kp = 0;
  if (i < nin) {
    const Key k = make_key(s, i);
    const uint64_t h = key_hash(s, k);
    const uint64_t j = find_slot(s, k, h, slots, mask, arena);
    if (j != ~0ull && slots[j].live && slots[j].off != 0)
      kp = (slots[j].fid == src_fid && slots[j].off == s.t.foff[i] - kHdr) ? 1 : 0;
  }
  if (i < rows) keep[i] = kp;
  (void)wave_alloc(&cnt[C_DONE], kp ? 1ull : 0ull);
}

__global__ void k_ix_result(const uint64_t* __restrict__ cnt, bcw_index_result* __restrict__ r) {
  bcw_index_result o{};
  o.n_in = cnt[C_NIN];
  o.n_done = cnt[C_DONE];
  o.err_class = (int32_t)cnt[C_FAIL];
  if (!o.err_class && cnt[C_OVERFLOW]) o.err_class = BCW_IDX_ERR_FULL;
  *r = o;
}

// ---- growth: re-insert every claimed slot into a larger table ---------------------------------------
__global__ __launch_bounds__(256) void k_ix_rehash(const Slot* __restrict__ old, uint64_t old_cap,
                                                   Slot* __restrict__ nw, uint64_t mask) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= old_cap) return;
  const Slot S = old[i];
  if (S.kref == 0) return;
  uint64_t j = S.hash & mask;
  for (uint64_t probe = 0; probe <= mask; ++probe, j = (j + 1) & mask) {
    if (atomicCAS(reinterpret_cast<unsigned long long*>(&nw[j].kref), 0ull, (unsigned long long)S.kref) == 0) {
      nw[j].seq = S.seq;
      nw[j].hash = S.hash;
      nw[j].fid = S.fid;
      nw[j].off = S.off;
      nw[j].size = S.size;
      nw[j].live = S.live;
      return;
    }
  }
}

// ---- export of the live entries (the Go shim loads them into its ShardMap after a GPU rebuild) --------
// fids (sorted, nf > 0): only entries whose value fid is one of them (the slice of the index that points into
// a set of WAL files: the compaction fan-out's filter snapshot)
__device__ __forceinline__ bool fid_in(const uint64_t* __restrict__ fids, uint32_t nf, uint64_t f) {
  if (nf == 0) return true;
  uint32_t lo = 0, hi = nf;
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    if (fids[m] < f) lo = m + 1; else hi = m;
  }
  return lo < nf && fids[lo] == f;
}

__global__ __launch_bounds__(256) void k_ix_count(const Slot* __restrict__ slots, uint64_t cap,
                                                  const uint8_t* __restrict__ arena, const uint64_t* __restrict__ fids,
                                                  uint32_t nf, uint64_t* __restrict__ blk_n,
                                                  uint64_t* __restrict__ blk_b) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  uint64_t c = 0, b = 0;
  if (i < cap && slots[i].kref && slots[i].live && fid_in(fids, nf, slots[i].fid)) {
    c = 1;
    b = *reinterpret_cast<const uint32_t*>(arena + (slots[i].kref - 1) + 8);
  }
  for (int d = 32; d >= 1; d >>= 1) {
    c += __shfl_xor(c, d, 64);
    b += __shfl_xor(b, d, 64);
  }
  __shared__ uint64_t sc[4], sb[4];
  if ((threadIdx.x & 63) == 0) { sc[threadIdx.x >> 6] = c; sb[threadIdx.x >> 6] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    blk_n[blockIdx.x] = sc[0] + sc[1] + sc[2] + sc[3];
    blk_b[blockIdx.x] = sb[0] + sb[1] + sb[2] + sb[3];
  }
}

__global__ __launch_bounds__(256) void k_ix_export(const Slot* __restrict__ slots, uint64_t cap,
                                                   const uint8_t* __restrict__ arena, const uint64_t* __restrict__ fids,
                                                   uint32_t nf, const uint64_t* __restrict__ blk_n,
                                                   const uint64_t* __restrict__ blk_b, uint8_t* __restrict__ keys,
                                                   uint64_t* __restrict__ koff, uint64_t* __restrict__ fid,
                                                   uint64_t* __restrict__ off, uint64_t* __restrict__ size) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  uint64_t c = 0, b = 0;
  Slot S{};
  if (i < cap) S = slots[i];
  const bool act = i < cap && S.kref && S.live && fid_in(fids, nf, S.fid);
  if (act) {
    c = 1;
    b = *reinterpret_cast<const uint32_t*>(arena + (S.kref - 1) + 8);
  }
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint64_t ic = c, ib = b;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t tc = __shfl_up(ic, d, 64), tb = __shfl_up(ib, d, 64);
    if (lane >= (uint32_t)d) { ic += tc; ib += tb; }
  }
  __shared__ uint64_t wc[4], wb[4];
  if (lane == 63) { wc[wave] = ic; wb[wave] = ib; }
  __syncthreads();
  uint64_t pc = blk_n[blockIdx.x], pb = blk_b[blockIdx.x];
  for (uint32_t w = 0; w < wave; ++w) { pc += wc[w]; pb += wb[w]; }
  pc += ic - c;
  pb += ib - b;
  if (!act) return;
  koff[pc] = pb;
  koff[pc + 1] = pb + b;  // the next entry writes the same value (or this is the last entry)
  fid[pc] = S.fid;
  off[pc] = S.off;
  size[pc] = S.size;
  const uint8_t* src = arena + (S.kref - 1) + 16;
  for (uint64_t q = 0; q < b; ++q) keys[pb + q] = src[q];
}

// ---- the capacity bound (bcw_index_set_limit): map.go's ShardMap keeps 16 shards (hash % 16) of Limited / 16 keys
// each and, when an insert would exceed a shard's limit, evicts the entry of minimum expire among sampled ones
// (SimpleMap.Set map.go:185-187, evict map.go:395-420, evictMinExpireEntry map.go:319). The device restates the
// bound with a deterministic policy: an entry's expire is the sequence number of the last op that set it (the
// index's logical clock in place of genExpire's wall seconds), and at the end of every batch each shard holding more
// than its limit evicts its entries of smallest sequence number (exact LRU order, every entry sampled) until it holds
// its limit. One workgroup per shard: count its live keys, radix-select (11-bit digits over npass passes) the
// (n - limit)-th smallest sequence number T (sequence numbers are unique), then evict every entry with seq <= T (live
// = 0, as Delete: the slot stays claimed). The evicted keys and their value sizes are counted (C_EVICTED*), the
// WriteStat of an eviction (index.go:144-165 reports the evicted value from Set's eviction path).
__global__ __launch_bounds__(1024) void k_ix_evict(Slot* __restrict__ slots, uint64_t cap, uint64_t lim,
                                                   uint64_t* __restrict__ cnt, uint32_t npass) {
  __shared__ uint32_t hist[2048];
  __shared__ unsigned long long s_acc[3];
  __shared__ uint64_t s_sel[2];  // prefix so far, rank left
  const uint32_t shard = blockIdx.x, tid = threadIdx.x;
  if (tid < 3) s_acc[tid] = 0;
  __syncthreads();
  uint64_t n = 0;
  for (uint64_t i = tid; i < cap; i += blockDim.x) n += (slots[i].live != 0 && (slots[i].hash & 15u) == shard) ? 1 : 0;
  atomicAdd(&s_acc[0], (unsigned long long)n);
  __syncthreads();
  const uint64_t total = s_acc[0];
  if (total <= lim) return;
  if (tid == 0) { s_sel[0] = 0; s_sel[1] = total - lim; }
  for (int p = (int)npass - 1; p >= 0; --p) {
    const uint32_t sh = 11u * (uint32_t)p;
    const uint64_t hi = (uint32_t)p + 1u >= npass ? 0ull : ~((1ull << (sh + 11u)) - 1ull);  // digits already chosen
    for (uint32_t b = tid; b < 2048u; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    const uint64_t pre = s_sel[0];
    for (uint64_t i = tid; i < cap; i += blockDim.x) {
      const Slot& q = slots[i];
      if (q.live != 0 && (q.hash & 15u) == shard && (q.seq & hi) == (pre & hi))
        atomicAdd(&hist[(q.seq >> sh) & 2047u], 1u);
    }
    __syncthreads();
    if (tid == 0) {  // the digit holding the rank-th smallest (a serial scan: evictions are rare)
      uint64_t rank = s_sel[1], c = 0;
      uint32_t b = 0;
      for (; b < 2047u && c + hist[b] < rank; ++b) c += hist[b];
      s_sel[0] = pre | ((uint64_t)b << sh);
      s_sel[1] = rank - c;
    }
    __syncthreads();
  }
  const uint64_t T = s_sel[0];
  uint64_t ev = 0, evb = 0;
  for (uint64_t i = tid; i < cap; i += blockDim.x) {
    Slot& q = slots[i];
    if (q.live != 0 && (q.hash & 15u) == shard && q.seq <= T) {
      q.live = 0;
      ++ev;
      evb += q.size;
    }
  }
  atomicAdd(&s_acc[1], (unsigned long long)ev);
  atomicAdd(&s_acc[2], (unsigned long long)evb);
  __syncthreads();
  if (tid == 0 && s_acc[1]) {
    atomicAdd(reinterpret_cast<unsigned long long*>(&cnt[C_EVICTED]), s_acc[1]);
    atomicAdd(reinterpret_cast<unsigned long long*>(&cnt[C_EVICTED_BYTES]), s_acc[2]);
    atomicAdd(reinterpret_cast<unsigned long long*>(&cnt[C_LIVE]), (unsigned long long)(0ull - s_acc[1]));
  }
}

}  // namespace ix
}  // namespace bcw

using namespace bcw;
using namespace bcw::ix;

struct bcw_index {
  bcw_ctx* ctx = nullptr;
  Slot* slots = nullptr;
  uint64_t cap = 0;  // slots (power of two)
  uint8_t* arena = nullptr;
  uint64_t arena_cap = 0;
  uint64_t* cnt = nullptr;  // device counters
  uint64_t slots_ub = 0, arena_ub = 0;  // host upper bounds of the device counters
  uint64_t seq_base = 1;                // sequence number of the next op
  uint64_t limited = 0;                 // the capacity bound (bcw_index_set_limit; 0: none)
  // per-op scratch
  uint64_t* op_kref = nullptr;
  uint64_t* op_hash = nullptr;
  uint64_t* op_slot = nullptr;
  uint64_t op_cap = 0;
  // host-batch staging (device copies)
  void* stage = nullptr;
  uint64_t stage_cap = 0;
  bcw_index_result* d_res = nullptr;
};

namespace bcw {
bcw_ctx* index_ctx(const bcw_index* ix) { return ix ? ix->ctx : nullptr; }
}  // namespace bcw

namespace {

constexpr double kMaxLoad = 0.7;

uint64_t pow2_at_least(uint64_t v) {
  uint64_t p = 1024;
  while (p < v) p <<= 1;
  return p;
}

int ix_sync_counters(bcw_index* x, uint64_t* out) {
  if (hipMemcpyAsync(out, x->cnt, C_NUM * sizeof(uint64_t), hipMemcpyDeviceToHost, x->ctx->cur) != hipSuccess ||
      hipStreamSynchronize(x->ctx->cur) != hipSuccess)
    return BCW_E_HIP;
  return BCW_OK;
}

// grow the slot table to hold `slots` claimed slots at kMaxLoad and the arena to `arena` bytes
int ix_grow(bcw_index* x, uint64_t slots, uint64_t arena) {
  hipStream_t st = x->ctx->cur;
  if (arena > x->arena_cap) {
    const uint64_t na = std::max(arena, x->arena_cap * 2);
    uint8_t* a = nullptr;
    if (hipMalloc(&a, na) != hipSuccess) return BCW_E_NOMEM;
    if (x->arena && hipMemcpyAsync(a, x->arena, x->arena_ub < x->arena_cap ? x->arena_ub : x->arena_cap,
                                   hipMemcpyDeviceToDevice, st) != hipSuccess) {
      (void)hipFree(a);
      return BCW_E_HIP;
    }
    (void)hipStreamSynchronize(st);
    (void)hipFree(x->arena);
    x->arena = a;
    x->arena_cap = na;
  }
  const uint64_t want = pow2_at_least((uint64_t)((double)slots / kMaxLoad) + 1);
  if (want > x->cap) {
    Slot* ns = nullptr;
    if (hipMalloc(&ns, want * sizeof(Slot)) != hipSuccess) return BCW_E_NOMEM;
    if (hipMemsetAsync(ns, 0, want * sizeof(Slot), st) != hipSuccess) { (void)hipFree(ns); return BCW_E_HIP; }
    if (x->slots && x->cap)
      k_ix_rehash<<<(uint32_t)((x->cap + 255) / 256), 256, 0, st>>>(x->slots, x->cap, ns, want - 1);
    if (hipStreamSynchronize(st) != hipSuccess) { (void)hipFree(ns); return BCW_E_HIP; }
    (void)hipFree(x->slots);
    x->slots = ns;
    x->cap = want;
  }
  return BCW_OK;
}

// make room for a batch of n ops whose arena entries total at most `arena_bytes`
int ix_room(bcw_index* x, uint64_t n, uint64_t arena_bytes) {
  const bool fits = (double)(x->slots_ub + n) <= kMaxLoad * (double)x->cap && x->arena_ub + arena_bytes <= x->arena_cap;
  if (!fits) {
    uint64_t c[C_NUM];
    int rc = ix_sync_counters(x, c);
    if (rc != BCW_OK) return rc;
    if (c[C_OVERFLOW]) return BCW_E_CAPACITY;  // a previous batch overflowed: the index is inconsistent
    x->slots_ub = c[C_SLOTS];
    x->arena_ub = c[C_ARENA];
    rc = ix_grow(x, x->slots_ub + n, x->arena_ub + arena_bytes);
    if (rc != BCW_OK) return rc;
  }
  if (n > x->op_cap) {
    (void)hipStreamSynchronize(x->ctx->cur);
    (void)hipFree(x->op_kref);
    (void)hipFree(x->op_hash);
    (void)hipFree(x->op_slot);
    x->op_kref = x->op_hash = x->op_slot = nullptr;
    x->op_cap = 0;
    const uint64_t c = std::max<uint64_t>(n, 1024);
    if (hipMalloc(&x->op_kref, c * 8) != hipSuccess || hipMalloc(&x->op_hash, c * 8) != hipSuccess ||
        hipMalloc(&x->op_slot, c * 8) != hipSuccess)
      return BCW_E_NOMEM;
    x->op_cap = c;
  }
  x->slots_ub += n;
  x->arena_ub += arena_bytes;
  return BCW_OK;
}

int ix_stage(bcw_index* x, uint64_t bytes) {
  if (bytes <= x->stage_cap) return BCW_OK;
  (void)hipStreamSynchronize(x->ctx->cur);
  (void)hipFree(x->stage);
  x->stage = nullptr;
  x->stage_cap = 0;
  if (hipMalloc(&x->stage, bytes) != hipSuccess) return BCW_E_NOMEM;
  x->stage_cap = bytes;
  return BCW_OK;
}

// the capacity bound after a batch (k_ix_evict), when one is set
void ix_bound(bcw_index* x) {
  if (!x->limited) return;
  uint32_t npass = 1;
  while (npass < 6 && (x->seq_base >> (11u * npass)) != 0) ++npass;  // digits of the largest sequence number
  k_ix_evict<<<16, 1024, 0, x->ctx->cur>>>(x->slots, x->cap, x->limited / 16, x->cnt, npass);
}

// the five launches of a batch (ops [0, n) of src); old_*: optional WriteStat outputs of k_ix_claim
void ix_batch(bcw_index* x, const Src& s, uint64_t n, const bcw_decode_result* R, uint64_t gen, const OpVals& v,
              uint8_t* old_found = nullptr, uint64_t* old_fid = nullptr, uint64_t* old_size = nullptr) {
  hipStream_t st = x->ctx->cur;
  const uint32_t grid = (uint32_t)((n + 255) / 256);
  (void)hipMemsetAsync(x->cnt + C_NIN, 0, 3 * sizeof(uint64_t), st);  // C_NIN, C_DONE, C_FAIL
  if (!grid) return;
  k_ix_keys<<<grid, 256, 0, st>>>(s, n, R, gen, x->cnt, x->op_kref, x->op_hash);
  k_ix_claim<<<grid, 256, 0, st>>>(s, n, x->cnt, x->slots, x->cap - 1, x->arena, x->cnt, x->op_kref, x->op_hash,
                                   x->op_slot, old_found, old_fid, old_size);
  k_ix_seq<<<grid, 256, 0, st>>>(n, x->cnt, s.kind == SRC_FLAT, x->slots, x->op_slot, x->seq_base);
  k_ix_commit<<<grid, 256, 0, st>>>(s, n, x->cnt, x->slots, x->arena, x->arena_cap, x->op_hash, x->op_slot);
  k_ix_write<<<grid, 256, 0, st>>>(s, n, x->cnt, v, x->slots, x->op_slot, x->seq_base);
  x->seq_base += n;
  ix_bound(x);
}

Src table_src(bcw_ctx* c, const uint8_t* d_seg, const bcw_decode_params* p, const bcw_record_table* t, int kind) {
  Src s{};
  s.kind = kind;
  s.seg = d_seg;
  s.seg_len = p->seg_len;
  s.frags = c->s.frags;
  s.t = *t;
  s.start_off = p->start_off;
  s.ns = p->ns_size;
  return s;
}

}  // namespace

namespace bcw {
int ix_export(bcw_index* x, const uint64_t* h_fids, uint64_t n_fids, IxSink& sink, uint64_t* n_out,
              uint64_t* key_bytes) {
  DeviceGuard dg(x->ctx->device);
  if (!dg.ok) return BCW_E_HIP;
  hipStream_t st = x->ctx->cur;
  std::vector<uint64_t> fids(h_fids, h_fids + n_fids);
  std::sort(fids.begin(), fids.end());
  fids.erase(std::unique(fids.begin(), fids.end()), fids.end());
  if (fids.size() > 0xffffffffull) return BCW_E_INVAL;
  const uint32_t nf = (uint32_t)fids.size();
  const uint64_t fb = (8 * (uint64_t)nf + 15) & ~15ull, nblk = (x->cap + 255) / 256;
  // staging: fids | per-block entry counts | per-block key bytes (then their exclusive prefixes) | outputs
  int rc = ix_stage(x, fb + nblk * 16 + 64);
  if (rc != BCW_OK) return rc;
  uint64_t* d_fids = (uint64_t*)x->stage;
  uint64_t* blk_n = (uint64_t*)((uint8_t*)x->stage + fb);
  uint64_t* blk_b = blk_n + nblk;
  if (nf && hipMemcpyAsync(d_fids, fids.data(), 8 * (uint64_t)nf, hipMemcpyHostToDevice, st) != hipSuccess)
    return BCW_E_HIP;
  k_ix_count<<<(uint32_t)nblk, 256, 0, st>>>(x->slots, x->cap, x->arena, d_fids, nf, blk_n, blk_b);
  std::vector<uint64_t> hn(nblk), hb(nblk);
  if (hipGetLastError() != hipSuccess ||
      hipMemcpyAsync(hn.data(), blk_n, nblk * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(hb.data(), blk_b, nblk * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return BCW_E_HIP;
  uint64_t tn = 0, tb = 0;
  for (uint64_t b = 0; b < nblk; ++b) {
    const uint64_t a = hn[b], k = hb[b];
    hn[b] = tn;
    hb[b] = tb;
    tn += a;
    tb += k;
  }
  *n_out = tn;
  *key_bytes = tb;
  rc = sink.room(tn, tb);
  if (rc != BCW_OK || tn == 0) return rc;
  const uint64_t tbp = (tb + 15) & ~15ull;
  rc = ix_stage(x, fb + nblk * 16 + tbp + 8 * (tn + 1) + 24 * tn + 64);  // a regrow drops the contents
  if (rc != BCW_OK) return rc;
  d_fids = (uint64_t*)x->stage;
  uint64_t* pn = (uint64_t*)((uint8_t*)x->stage + fb);
  uint64_t* pb = pn + nblk;
  uint8_t* keys = (uint8_t*)(pb + nblk);
  uint64_t* koff = (uint64_t*)(keys + tbp);
  uint64_t* fid = koff + tn + 1;
  uint64_t* off = fid + tn;
  uint64_t* size = off + tn;
  bool ok = (!nf || hipMemcpyAsync(d_fids, fids.data(), 8 * (uint64_t)nf, hipMemcpyHostToDevice, st) == hipSuccess) &&
            hipMemcpyAsync(pn, hn.data(), nblk * 8, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(pb, hb.data(), nblk * 8, hipMemcpyHostToDevice, st) == hipSuccess;
  if (ok)
    k_ix_export<<<(uint32_t)nblk, 256, 0, st>>>(x->slots, x->cap, x->arena, d_fids, nf, pn, pb, keys, koff, fid, off,
                                                  size);
  ok = ok && hipGetLastError() == hipSuccess &&
       hipMemcpyAsync(sink.keys, keys, tb, hipMemcpyDeviceToHost, st) == hipSuccess &&
       hipMemcpyAsync(sink.koff, koff, 8 * (tn + 1), hipMemcpyDeviceToHost, st) == hipSuccess &&
       hipMemcpyAsync(sink.fid, fid, 8 * tn, hipMemcpyDeviceToHost, st) == hipSuccess &&
       hipMemcpyAsync(sink.off, off, 8 * tn, hipMemcpyDeviceToHost, st) == hipSuccess &&
       hipMemcpyAsync(sink.size, size, 8 * tn, hipMemcpyDeviceToHost, st) == hipSuccess &&
       hipStreamSynchronize(st) == hipSuccess;
  return ok ? BCW_OK : BCW_E_HIP;
}
}  // namespace bcw

namespace bcw {
int ix_filter_on(bcw_index* x, bcw_ctx* c, const uint8_t* d_seg, const bcw_decode_params* p,
                 const bcw_record_table* d_table, const bcw_decode_result* d_result, uint64_t src_fid, uint8_t* d_keep,
                 uint64_t* d_cnt, bcw_index_result* d_out) {
  static_assert(C_NUM <= kIxCounters, "the per-call counters hold every index counter");
  if (!x || !c || !p || !d_table || !d_result || !d_keep || !d_cnt || p->mode != BCW_MODE_RECORD ||
      c->device != x->ctx->device)
    return BCW_E_INVAL;
  if (!c->s.frags || !d_table->foff || !d_table->key_len || !d_table->first_frag || !d_table->emit_frag ||
      !d_table->hdr_size)
    return BCW_E_INVAL;
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  const uint64_t rows = d_table->capacity;
  hipStream_t st = c->cur;
  // the index's counters (its overflow flag included), then this call's own zeroed
  (void)hipMemcpyAsync(d_cnt, x->cnt, C_NUM * sizeof(uint64_t), hipMemcpyDeviceToDevice, st);
  (void)hipMemsetAsync(d_cnt + C_NIN, 0, 3 * sizeof(uint64_t), st);
  const Src s = table_src(c, d_seg, p, d_table, SRC_RECORD);
  if (rows)
    k_ix_filter<<<(uint32_t)((rows + 255) / 256), 256, 0, st>>>(s, rows, d_result, c->frag_gen, x->slots, x->cap - 1,
                                                                 x->arena, src_fid, d_keep, d_cnt);
  if (d_out) k_ix_result<<<1, 1, 0, st>>>(d_cnt, d_out);
  return hipGetLastError() == hipSuccess ? BCW_OK : BCW_E_HIP;
}
}  // namespace bcw

extern "C" {

int bcw_index_create(bcw_ctx* c, uint64_t keys, uint64_t arena_bytes, bcw_index** out) {
  if (!c || !out) return BCW_E_INVAL;
  *out = nullptr;
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  bcw_index* x = new (std::nothrow) bcw_index();
  if (!x) return BCW_E_NOMEM;
  x->ctx = c;
  if (hipMalloc(&x->cnt, C_NUM * sizeof(uint64_t)) != hipSuccess ||
      hipMalloc(&x->d_res, sizeof(bcw_index_result)) != hipSuccess ||
      hipMemsetAsync(x->cnt, 0, C_NUM * sizeof(uint64_t), c->cur) != hipSuccess) {
    bcw_index_destroy(x);
    return BCW_E_NOMEM;
  }
  const int rc = ix_grow(x, std::max<uint64_t>(keys, 1024), std::max<uint64_t>(arena_bytes, 1 << 20));
  if (rc != BCW_OK) { bcw_index_destroy(x); return rc; }
  *out = x;
  return BCW_OK;
}

int bcw_index_destroy(bcw_index* x) {
  if (!x) return BCW_E_INVAL;
  DeviceGuard dg(x->ctx->device);
  (void)hipStreamSynchronize(x->ctx->cur);
  void* ptrs[] = {x->slots, x->arena, x->cnt, x->op_kref, x->op_hash, x->op_slot, x->stage, x->d_res};
  for (void* q : ptrs) (void)hipFree(q);
  delete x;
  return BCW_OK;
}

int bcw_index_reserve(bcw_index* x, uint64_t keys, uint64_t arena_bytes) {
  if (!x) return BCW_E_INVAL;
  DeviceGuard dg(x->ctx->device);
  if (!dg.ok) return BCW_E_HIP;
  uint64_t c[C_NUM];
  int rc = ix_sync_counters(x, c);
  if (rc != BCW_OK) return rc;
  x->slots_ub = c[C_SLOTS];
  x->arena_ub = c[C_ARENA];
  return ix_grow(x, std::max(keys, x->slots_ub), std::max(arena_bytes, x->arena_ub));
}

int bcw_index_stats(bcw_index* x, bcw_index_info* out) {
  if (!x || !out) return BCW_E_INVAL;
  DeviceGuard dg(x->ctx->device);
  if (!dg.ok) return BCW_E_HIP;
  uint64_t c[C_NUM];
  const int rc = ix_sync_counters(x, c);
  if (rc != BCW_OK) return rc;
  out->live = c[C_LIVE];
  out->slots_used = c[C_SLOTS];
  out->slot_capacity = x->cap;
  out->arena_used = c[C_ARENA];
  out->arena_capacity = x->arena_cap;
  out->overflow = c[C_OVERFLOW];
  out->limited = x->limited;
  out->evicted = c[C_EVICTED];
  out->evicted_bytes = c[C_EVICTED_BYTES];
  return BCW_OK;
}

int bcw_index_set_limit(bcw_index* x, uint64_t limited) {
  if (!x || (limited != 0 && limited < 16)) return BCW_E_INVAL;
  DeviceGuard dg(x->ctx->device);
  if (!dg.ok) return BCW_E_HIP;
  x->limited = limited;
  ix_bound(x);  // an index already past the new bound is brought within it at once
  return hipGetLastError() == hipSuccess && hipStreamSynchronize(x->ctx->cur) == hipSuccess ? BCW_OK : BCW_E_HIP;
}

int bcw_index_apply_stat(bcw_index* x, uint64_t n, const uint8_t* h_keys, const uint64_t* h_key_off,
                         const uint8_t* h_ops, const uint64_t* h_fid, const uint64_t* h_off, const uint64_t* h_size,
                         uint8_t* h_found, uint64_t* h_free_fid, uint64_t* h_free_bytes) {
  if (!x || (n && (!h_key_off || !h_ops || !h_fid || !h_off || !h_size))) return BCW_E_INVAL;
  const bool stat = h_found || h_free_fid || h_free_bytes;
  if (stat && !(h_found && h_free_fid && h_free_bytes)) return BCW_E_INVAL;
  if (n == 0) return BCW_OK;
  const uint64_t kb = h_key_off[n] - h_key_off[0];
  if (kb && !h_keys) return BCW_E_INVAL;
  for (uint64_t i = 0; i < n; ++i)
    if (h_key_off[i + 1] < h_key_off[i] || h_ops[i] > BCW_IDX_SOFT_DELETE) return BCW_E_INVAL;
  DeviceGuard dg(x->ctx->device);
  if (!dg.ok) return BCW_E_HIP;
  const uint64_t arena_b = 16 * n + kb + 15 * n;
  int rc = ix_room(x, n, arena_b);
  if (rc != BCW_OK) return rc;
  // staging: keys | key offsets (rebased) | fid | off | size | WriteStat (fid, size) | ops | found
  const uint64_t kbp = (kb + 15) & ~15ull;
  rc = ix_stage(x, kbp + 8 * (n + 1) + 40 * n + 2 * n + 64);
  if (rc != BCW_OK) return rc;
  uint8_t* m = (uint8_t*)x->stage;
  uint8_t* d_keys = m;
  uint64_t* d_koff = (uint64_t*)(m + kbp);
  uint64_t* d_fid = d_koff + (n + 1);
  uint64_t* d_off = d_fid + n;
  uint64_t* d_size = d_off + n;
  uint64_t* d_ofid = d_size + n;
  uint64_t* d_osize = d_ofid + n;
  uint8_t* d_ops = (uint8_t*)(d_osize + n);
  uint8_t* d_found = d_ops + n;
  hipStream_t st = x->ctx->cur;
  std::vector<uint64_t> koff(n + 1);
  for (uint64_t i = 0; i <= n; ++i) koff[i] = h_key_off[i] - h_key_off[0];
  bool ok = (kb == 0 || hipMemcpyAsync(d_keys, h_keys + h_key_off[0], kb, hipMemcpyHostToDevice, st) == hipSuccess) &&
            hipMemcpyAsync(d_koff, koff.data(), 8 * (n + 1), hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(d_fid, h_fid, 8 * n, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(d_off, h_off, 8 * n, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(d_size, h_size, 8 * n, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(d_ops, h_ops, n, hipMemcpyHostToDevice, st) == hipSuccess;
  if (!ok) return BCW_E_HIP;
  Src s{};
  s.kind = SRC_FLAT;
  s.keys = d_keys;
  s.koff = d_koff;
  s.keys_len = kb;
  OpVals v{d_ops, d_fid, d_off, d_size, 0, 0};
  ix_batch(x, s, n, nullptr, 0, v, stat ? d_found : nullptr, d_ofid, d_osize);
  if (stat)
    ok = hipMemcpyAsync(h_found, d_found, n, hipMemcpyDeviceToHost, st) == hipSuccess &&
         hipMemcpyAsync(h_free_fid, d_ofid, 8 * n, hipMemcpyDeviceToHost, st) == hipSuccess &&
         hipMemcpyAsync(h_free_bytes, d_osize, 8 * n, hipMemcpyDeviceToHost, st) == hipSuccess;
  if (!ok || hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) return BCW_E_HIP;
  if (stat) {
    // the device reported, per op, the value the key held before the batch; an op preceded by another op on the
    // same key in this batch replaces that op's value instead (Put: its fid / size, SoftDelete: IndexValue{} with
    // fid 0 / size 0, Delete: nothing -- index.go:108-165)
    std::unordered_map<std::string_view, uint64_t> last;
    last.reserve(n * 2);
    const char* kbase = reinterpret_cast<const char*>(h_keys);
    for (uint64_t i = 0; i < n; ++i) {
      const std::string_view key(kbase ? kbase + h_key_off[i] : "", h_key_off[i + 1] - h_key_off[i]);
      auto it = last.find(key);
      if (it != last.end()) {
        const uint64_t p = it->second;
        h_found[i] = h_ops[p] != BCW_IDX_DELETE;
        h_free_fid[i] = h_ops[p] == BCW_IDX_PUT ? h_fid[p] : 0;
        h_free_bytes[i] = h_ops[p] == BCW_IDX_PUT ? h_size[p] : 0;
        it->second = i;
      } else {
        last.emplace(key, i);
      }
      if (!h_found[i]) h_free_fid[i] = h_free_bytes[i] = 0;
    }
  }
  uint64_t c[C_NUM];
  rc = ix_sync_counters(x, c);
  if (rc != BCW_OK) return rc;
  return c[C_OVERFLOW] ? BCW_E_CAPACITY : BCW_OK;
}

int bcw_index_apply(bcw_index* x, uint64_t n, const uint8_t* h_keys, const uint64_t* h_key_off, const uint8_t* h_ops,
                    const uint64_t* h_fid, const uint64_t* h_off, const uint64_t* h_size) {
  return bcw_index_apply_stat(x, n, h_keys, h_key_off, h_ops, h_fid, h_off, h_size, nullptr, nullptr, nullptr);
}

int bcw_index_clear(bcw_index* x) {
  if (!x) return BCW_E_INVAL;
  DeviceGuard dg(x->ctx->device);
  if (!dg.ok) return BCW_E_HIP;
  hipStream_t st = x->ctx->cur;
  if (hipMemsetAsync(x->slots, 0, x->cap * sizeof(Slot), st) != hipSuccess ||
      hipMemsetAsync(x->cnt, 0, C_NUM * sizeof(uint64_t), st) != hipSuccess)
    return BCW_E_HIP;
  x->slots_ub = 0;
  x->arena_ub = 0;
  return BCW_OK;
}

int bcw_index_get(bcw_index* x, uint64_t n, const uint8_t* h_keys, const uint64_t* h_key_off, uint64_t* h_fid,
                  uint64_t* h_off, uint64_t* h_size, uint8_t* h_status) {
  if (!x || (n && (!h_key_off || !h_fid || !h_off || !h_size || !h_status))) return BCW_E_INVAL;
  if (n == 0) return BCW_OK;
  const uint64_t kb = h_key_off[n] - h_key_off[0];
  if (kb && !h_keys) return BCW_E_INVAL;
  for (uint64_t i = 0; i < n; ++i)
    if (h_key_off[i + 1] < h_key_off[i]) return BCW_E_INVAL;
  DeviceGuard dg(x->ctx->device);
  if (!dg.ok) return BCW_E_HIP;
  const uint64_t kbp = (kb + 15) & ~15ull;
  int rc = ix_stage(x, kbp + 8 * (n + 1) + 24 * n + n + 64);
  if (rc != BCW_OK) return rc;
  uint8_t* m = (uint8_t*)x->stage;
  uint8_t* d_keys = m;
  uint64_t* d_koff = (uint64_t*)(m + kbp);
  uint64_t* d_fid = d_koff + (n + 1);
  uint64_t* d_off = d_fid + n;
  uint64_t* d_size = d_off + n;
  uint8_t* d_st = (uint8_t*)(d_size + n);
  hipStream_t st = x->ctx->cur;
  std::vector<uint64_t> koff(n + 1);
  for (uint64_t i = 0; i <= n; ++i) koff[i] = h_key_off[i] - h_key_off[0];
  bool ok = (kb == 0 || hipMemcpyAsync(d_keys, h_keys + h_key_off[0], kb, hipMemcpyHostToDevice, st) == hipSuccess) &&
            hipMemcpyAsync(d_koff, koff.data(), 8 * (n + 1), hipMemcpyHostToDevice, st) == hipSuccess;
  if (!ok) return BCW_E_HIP;
  Src s{};
  s.kind = SRC_FLAT;
  s.keys = d_keys;
  s.koff = d_koff;
  s.keys_len = kb;
  k_ix_get<<<(uint32_t)((n + 255) / 256), 256, 0, st>>>(s, n, x->slots, x->cap - 1, x->arena, d_fid, d_off, d_size,
                                                         d_st);
  ok = hipGetLastError() == hipSuccess &&
       hipMemcpyAsync(h_fid, d_fid, 8 * n, hipMemcpyDeviceToHost, st) == hipSuccess &&
       hipMemcpyAsync(h_off, d_off, 8 * n, hipMemcpyDeviceToHost, st) == hipSuccess &&
       hipMemcpyAsync(h_size, d_size, 8 * n, hipMemcpyDeviceToHost, st) == hipSuccess &&
       hipMemcpyAsync(h_status, d_st, n, hipMemcpyDeviceToHost, st) == hipSuccess &&
       hipStreamSynchronize(st) == hipSuccess;
  return ok ? BCW_OK : BCW_E_HIP;
}

int bcw_index_put_decoded_async(bcw_index* x, const uint8_t* d_seg, const bcw_decode_params* p,
                                const bcw_record_table* d_table, const bcw_decode_result* d_result, uint64_t fid,
                                int use_record_fid, bcw_index_result* d_out) {
  if (!x || !p || !d_table || !d_result) return BCW_E_INVAL;
  if (p->mode != BCW_MODE_RECORD && p->mode != BCW_MODE_HINT) return BCW_E_INVAL;
  bcw_ctx* c = x->ctx;
  if (!c->s.frags || !d_table->foff || !d_table->size || !d_table->key_len || !d_table->first_frag ||
      !d_table->emit_frag || !d_table->hdr_size)
    return BCW_E_INVAL;
  if (p->mode == BCW_MODE_HINT && (!d_table->aux0 || !d_table->aux1 || !d_table->expire)) return BCW_E_INVAL;
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  const uint64_t rows = d_table->capacity;
  const Src s = table_src(c, d_seg, p, d_table, p->mode == BCW_MODE_RECORD ? SRC_RECORD : SRC_HINT);
  // arena bound: a merged key is at most its record's payload (ns + key <= size), all payloads fit the segment.
  // When that cheap bound does not fit the arena (a large segment), the exact need of the delivered rows is
  // read back instead (one small launch and a sync): only keys new to the index take arena space, so an
  // index rebuilt over keys it already holds does not grow.
  uint64_t arena_b = p->seg_len + 32 * rows;
  if (x->arena_ub + arena_b > x->arena_cap && rows) {
    if (hipMemsetAsync(x->cnt + C_NEED, 0, sizeof(uint64_t), c->cur) != hipSuccess) return BCW_E_HIP;
    k_ix_need<<<(uint32_t)((rows + 255) / 256), 256, 0, c->cur>>>(s, rows, d_result, c->frag_gen, x->cnt);
    uint64_t cc[C_NUM];
    int rc0 = ix_sync_counters(x, cc);
    if (rc0 != BCW_OK) return rc0;
    if (cc[C_OVERFLOW]) return BCW_E_CAPACITY;
    x->arena_ub = cc[C_ARENA];
    x->slots_ub = cc[C_SLOTS];
    arena_b = cc[C_NEED];
  }
  int rc = ix_room(x, rows, arena_b);
  if (rc != BCW_OK) return rc;
  OpVals v{nullptr, nullptr, nullptr, nullptr, fid, use_record_fid};
  ix_batch(x, s, rows, d_result, c->frag_gen, v);
  if (d_out) k_ix_result<<<1, 1, 0, c->cur>>>(x->cnt, d_out);
  return hipGetLastError() == hipSuccess ? BCW_OK : BCW_E_HIP;
}

int bcw_compact_filter_async(bcw_index* x, const uint8_t* d_seg, const bcw_decode_params* p,
                             const bcw_record_table* d_table, const bcw_decode_result* d_result, uint64_t src_fid,
                             uint8_t* d_keep, bcw_index_result* d_out) {
  if (!x || !p || !d_table || !d_result || !d_keep || p->mode != BCW_MODE_RECORD) return BCW_E_INVAL;
  bcw_ctx* c = x->ctx;
  if (!c->s.frags || !d_table->foff || !d_table->key_len || !d_table->first_frag || !d_table->emit_frag ||
      !d_table->hdr_size)
    return BCW_E_INVAL;
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  const uint64_t rows = d_table->capacity;
  hipStream_t st = c->cur;
  (void)hipMemsetAsync(x->cnt + C_NIN, 0, 3 * sizeof(uint64_t), st);
  const Src s = table_src(c, d_seg, p, d_table, SRC_RECORD);
  if (rows)
    k_ix_filter<<<(uint32_t)((rows + 255) / 256), 256, 0, st>>>(s, rows, d_result, c->frag_gen, x->slots, x->cap - 1,
                                                                 x->arena, src_fid, d_keep, x->cnt);
  if (d_out) k_ix_result<<<1, 1, 0, st>>>(x->cnt, d_out);
  return hipGetLastError() == hipSuccess ? BCW_OK : BCW_E_HIP;
}

int bcw_index_export(bcw_index* x, uint8_t* h_keys, uint64_t keys_cap, uint64_t* h_key_off, uint64_t* h_fid,
                     uint64_t* h_off, uint64_t* h_size, uint64_t entries_cap, uint64_t* n_out, uint64_t* key_bytes) {
  return bcw_index_export_fids(x, nullptr, 0, h_keys, keys_cap, h_key_off, h_fid, h_off, h_size, entries_cap, n_out,
                               key_bytes);
}

int bcw_index_export_fids(bcw_index* x, const uint64_t* h_fids, uint64_t n_fids, uint8_t* h_keys, uint64_t keys_cap,
                          uint64_t* h_key_off, uint64_t* h_fid, uint64_t* h_off, uint64_t* h_size,
                          uint64_t entries_cap, uint64_t* n_out, uint64_t* key_bytes) {
  if (!x || !n_out || !key_bytes || (n_fids && !h_fids)) return BCW_E_INVAL;
  struct Fixed : IxSink {
    uint64_t ecap, kcap;
    int room(uint64_t n, uint64_t kb) override {
      if (n > ecap || kb > kcap) return BCW_E_CAPACITY;
      return n == 0 || (keys && koff && fid && off && size) ? BCW_OK : BCW_E_INVAL;
    }
  } sink;
  sink.ecap = entries_cap;
  sink.kcap = keys_cap;
  sink.keys = h_keys;
  sink.koff = h_key_off;
  sink.fid = h_fid;
  sink.off = h_off;
  sink.size = h_size;
  const int rc = ix_export(x, h_fids, n_fids, sink, n_out, key_bytes);
  if (rc == BCW_OK && *n_out == 0 && h_key_off) h_key_off[0] = 0;
  return rc;
}

uint64_t bcw_murmur3_sum64(const uint8_t* p, uint64_t n) {
  // host restatement of the device hash (spaolacci/murmur3 New64().Sum64(), index.go:15-19)
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  auto rl = [](uint64_t v, int r) { return (v << r) | (v >> (64 - r)); };
  auto fm = [](uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33;
    return k;
  };
  uint64_t h1 = 0, h2 = 0;
  const uint64_t nb = n / 16;
  for (uint64_t i = 0; i < nb; ++i) {
    uint64_t k1, k2;
    memcpy(&k1, p + 16 * i, 8);
    memcpy(&k2, p + 16 * i + 8, 8);
    k1 *= c1; k1 = rl(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rl(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= c2; k2 = rl(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rl(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
  }
  uint64_t k1 = 0, k2 = 0;
  const uint64_t t = n & 15;
  for (uint64_t i = 0; i < t; ++i) {
    const uint64_t b = p[16 * nb + i];
    if (i < 8) k1 |= b << (8 * i); else k2 |= b << (8 * (i - 8));
  }
  if (t > 8) { k2 *= c2; k2 = rl(k2, 33); k2 *= c1; h2 ^= k2; }
  if (t > 0) { k1 *= c1; k1 = rl(k1, 31); k1 *= c2; h1 ^= k1; }
  h1 ^= n; h2 ^= n;
  h1 += h2; h2 += h1;
  h1 = fm(h1); h2 = fm(h2);
  h1 += h2;
  return h1;
}

}  // extern "C"
