// Internal definitions shared by the host API (bcw_api.cpp) and the device kernels (bcw_decode.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <vector>

#include "bcw.h"

namespace bcw {

constexpr uint32_t kBlock = BCW_BLOCK_SIZE;  // wal.go:46
constexpr uint32_t kHdr = BCW_HEADER_SIZE;   // wal.go:53
constexpr uint32_t kWin = 128;               // CRC window per lane (bytes)
constexpr int kWaveLanes = 64;

// One parsed fragment header (wal_iterator.go:62-77), 16 bytes.
struct Frag {
  uint32_t blk;    // block index within the segment
  uint16_t start;  // block-relative offset of the data (header + 7)
  uint16_t len;    // data length after the clamp of wal_iterator.go:75
  uint32_t crc;    // stored masked CRC (header bytes [0,4))
  uint8_t type;    // header byte 6
  uint8_t ok;      // CRC verified
  uint16_t pad;
};
static_assert(sizeof(Frag) == 16, "Frag layout");

// Per-block record-state transform (the composition of the iterator's per-fragment state
// machine over one block, wal_iterator.go:69-96). See DESIGN.md "record assembly".
struct BlockSum {
  uint64_t pre_len;   // sum of lengths of fragments before the first emission (or all, if none)
  uint64_t pre_off;   // data offset of the first non-empty fragment among them
  uint64_t out_acc;   // state after the last emission: accumulated length
  uint64_t out_off;   // ... its iterator offset
  uint32_t pre_first; // global fragment index of that first non-empty fragment
  uint32_t out_first; // ... first fragment of the pending record
  uint32_t n_emit;    // emissions in the block before the error (if any)
  uint32_t err_frag;  // global index of the first failing fragment in the block, or ~0u
  uint8_t has_emit;
  uint8_t pre_nz;
  uint8_t err_class;
  uint8_t pad[5];
};
static_assert(sizeof(BlockSum) == 56, "BlockSum layout");

// Incoming state of a block after the scan.
struct BlockIn {
  uint64_t acc;
  uint64_t off;
  uint64_t rec_base;  // global record index of the block's first emission
  uint32_t first;
  uint32_t live;      // 0 if an earlier block already failed
};
static_assert(sizeof(BlockIn) == 32, "BlockIn layout");

// Device-side constant tables, built on the host once per context.
struct Tables {
  uint32_t* slice;   // [2][256] slice-by-2 CRC-32C tables (T0 = byte table, T1)
  uint32_t* fwd;     // [64][8][16] lane shift operators F_l = A_{8*128*(63-l)} (nibble images)
  uint32_t* carry;   // [8][16] A_{8*8192} (nibble images)
  uint32_t* initc;   // [kBlock+1] A_{8L}(0xFFFFFFFF)
};

struct Scratch {
  uint64_t nblocks_cap = 0;
  uint64_t frag_cap = 0;
  uint32_t* nfrag = nullptr;   // [nblocks]
  uint32_t* fbase = nullptr;   // [nblocks+1]
  Frag* frags = nullptr;       // [frag_cap]
  BlockSum* sums = nullptr;    // [nblocks]
  BlockIn* ins = nullptr;      // [nblocks]
  uint64_t* misc = nullptr;    // [16] device counters (see bcw_decode.hip)
};

// Optional per-kernel HIP-event timing (bcw_ctx_set_profiling): events recorded on the launch
// stream around every kernel of the pipeline.
enum KernelId { K_CHASE_COUNT = 0, K_SCAN, K_CHASE_WRITE, K_CRC, K_BLOCKSUM, K_BLOCKSCAN, K_RECORDS, K_FINALIZE,
                K_NUM };
struct Prof {
  bool on = false;
  struct Mark { int kid; hipEvent_t a, b; };
  std::vector<Mark> marks;
  std::vector<hipEvent_t> pool;
  hipEvent_t get() {
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  void begin(int kid, hipStream_t s, hipEvent_t& a) { if (on) { a = get(); (void)hipEventRecord(a, s); } (void)kid; }
  void end(int kid, hipStream_t s, hipEvent_t a) {
    if (!on) return;
    hipEvent_t b = get();
    (void)hipEventRecord(b, s);
    marks.push_back({kid, a, b});
  }
};

// Launch the full decode pipeline on `stream`. Defined in bcw_decode.hip.
hipError_t launch_decode(const uint8_t* d_seg, const bcw_decode_params& p, const bcw_record_table& t,
                         bcw_decode_result* d_result, const Tables& tabs, Scratch& s, uint64_t nblocks,
                         hipStream_t stream, int num_cus, Prof* prof);
hipError_t launch_export_frags(const Scratch& s, const bcw_frag_table& out, uint32_t start_off, hipStream_t stream,
                               uint64_t n);

// Host-side table builders (bcw_api.cpp).
void build_slice_tables(uint32_t* t2x256);
void build_lane_tables(uint32_t* fwd64x8x16, uint32_t* carry8x16);
void build_initc(uint32_t* initc);

}  // namespace bcw
