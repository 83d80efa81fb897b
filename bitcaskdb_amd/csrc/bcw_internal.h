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

// k_crc's stream balanced per XCD (bcw_decode.hip): workgroup r streams range r of the segment, and the dispatcher
// places workgroup r on XCD (r + s) % 8 with the same s every decode (both kernels' grids are multiples of 8), so each
// class r % 8 is one XCD. The ranges of class y are sized in proportion to its weight, the rate measured by the
// previous decode on the context (the XCDs of an MI355X stream up to ~6 % apart, kbench per-XCD timelines). Only the
// work split depends on it, never a result.
struct XBal {
  uint32_t w[8];    // byte weight of a range of class y (65536: equal)
  uint32_t pad0[8];
  uint64_t t[8];    // k_crc: summed stream times (wall_clock64 ticks) of class y's waves (the finalize resets them)
  uint64_t n[8];    // their count
  uint32_t on;      // k_chase used the weights (BCW_OPT_XCD_BALANCE): the finalize updates them only then
  uint32_t pad[7];
};
// One parsed fragment header (wal_iterator.go:62-77), 16 bytes.
struct Frag {
  uint32_t blk;    // block index within the segment
  uint16_t start;  // block-relative offset of the data (header + 7)
  uint16_t len;    // data length after the clamp of wal_iterator.go:75
  uint32_t chk;    // check word J = ~unmask(stored CRC) ^ A_{8 len}(0xFFFFFFFF) (bcw_decode.hip, k_crc): the
                   // fragment's data passes ComputeCRC32 iff its raw CRC-32C equals this (stored CRC recoverable)
  uint8_t type;    // header byte 6
  uint8_t ok;      // CRC verified
  uint16_t pad;
};
static_assert(sizeof(Frag) == 16, "Frag layout");

// shift operators A_{8 * 2^k} for k < kPow2Ops: any shift below 2^16 bytes (a fragment's u16 length)
constexpr int kPow2Ops = 16;

// Device-side constant tables, built on the host once per context.
struct Tables {
  uint32_t* initc;   // [kBlock+1] A_{8L}(0xFFFFFFFF)
  uint32_t* lds_image2; // the stream verify's LDS image (kS2Image)
  uint32_t* enc_ops;    // [kEncOpsWords] encode shift operators (nibble images, see build_enc_ops)
  uint32_t* pow2;       // [kPow2Ops][8][16] A_{8 * 2^k} (nibble images), k < 16: shifts by any distance < 64 KiB
};
// enc_ops layout (operators of 128 words): [n] A_{8*16*n}, [16 + n] A_{8*256*n} (n < 16), [32 + n]
// A_{8*4096*n} (n < 8), [40 + t] A_{8t}^-1 (t < 16), [56 + k] A_{8*2^k} (k < 32), [88 + k] A_{8*2^k}^-1 (k < 15)
constexpr int kOpInv = 40, kOpPow2 = 56, kOpPow2Inv = 88;
constexpr int kEncOpsWords = 103 * 128;

// k_crc stream verify (bcw_decode.hip, stream_verify): absolute 1 KiB chunks, 16 B per lane (one fully contiguous
// load per chunk). LDS image (dwords): the lane operators G_l = A_{8*16*(63-l)} transposed to [8][16][64 lanes]
// (first: byte offsets i * 4096 + v * 256 + 4 l, each table base a ds_read immediate); slice-by-4 rows of 256 B
// {T3, T2, T1, T0} x 8 copies then the shifted tables T'_k (a byte followed by k + 1008 zero bytes) x 8 copies; the
// split operators A_{8*(4*(4-k) + 1008)} (k = 0..3) as byte tables [k][byte t][256]; and the per-lane byte-select
// tables of the fragment-end masks (16 B entries, one per lane offset): GE (bytes >= n), JSEL (the check word's bytes
// at piece offset m - 3), GAP (check word at piece offset g - 6, then 3 zero bytes).
constexpr int kSPiece = 16;
constexpr int kSChunk = 64 * kSPiece;
constexpr int kSPW = kSPiece / 4;  // words per lane
constexpr int kS2Slice = 256 * 64, kS2Lop = 8 * 16 * 64, kS2Kop = kSPW * 4 * 256;
constexpr int kS2LopOff = 0, kS2SliceOff = kS2Lop, kS2KopOff = kS2Lop + kS2Slice;
constexpr int kS2GeN = 17, kS2JselN = 20, kS2GapN = 23;  // entries (4 dwords each)
constexpr int kS2Ge = kS2Slice + kS2Lop + kS2Kop, kS2Jsel = kS2Ge + 4 * kS2GeN, kS2Gap = kS2Jsel + 4 * kS2JselN;
constexpr int kS2Image = kS2Gap + 4 * kS2GapN + 4;  // (+ pad to 16 B)
#ifndef BCW_CRC_WAVES
#define BCW_CRC_WAVES 16
#endif
constexpr int kCrcWaves = BCW_CRC_WAVES;  // waves per k_crc workgroup (one workgroup per CU)
constexpr int kCrcThreads = kCrcWaves * 64;

struct Scratch {
  uint64_t nblocks_cap = 0;
  uint64_t frag_cap = 0;
  uint32_t* fbase = nullptr;   // [nblocks+1] global index of each block's first fragment
  uint32_t* rbase = nullptr;   // [nblocks+1] Full/Last fragments before each block (its first record row)
  uint2* bsum = nullptr;       // [nblocks] record-state summary of each block (bcw_decode.hip, kSumHasE)
  uint64_t* lb = nullptr;      // [nblocks/64+2] k_chase look-back words (zeroed at allocation)
  uint64_t* lbe = nullptr;     // [nblocks/64+2] k_chase look-back words of the Full/Last counts (> kDirect groups)
  uint64_t nlb = 0;
  uint64_t epoch = 1;          // look-back epoch of the next launch
  Frag* frags = nullptr;       // [frag_cap]
  uint4* srec = nullptr;       // [frag_cap + 4] stream record per fragment (k_chase -> k_crc, bcw_decode.hip kRecUsual)
  uint8_t* fok = nullptr;      // [frag_cap] CRC verdict per fragment (k_crc; dense: 64 verdicts are one 64 B store)
  uint32_t* wstart = nullptr;  // [CUs x kCrcWaves + 1] each k_crc wave's first fragment (byte-balanced, k_chase)
  XBal* xbal = nullptr;        // the per-XCD split of k_crc's stream (persists across decodes)
  uint32_t xbal_on = 1;        // BCW_OPT_XCD_BALANCE
  uint64_t* misc = nullptr;    // [16] device counters (see bcw_decode.hip)
  uint32_t chase_direct = BCW_CHASE_DIRECT_MAX;  // k_chase: direct predecessor sum up to this many workgroups
  uint64_t test_abort_wg = 0;  // BCW_OPT_TEST_ABORT_WAIT for the next launch only (k_chase workgroup + 1; 0: none)
};

// Optional per-kernel HIP-event timing (bcw_ctx_set_profiling): events recorded on the launch
// stream around every kernel of the pipeline.
enum KernelId { K_CHASE = 0, K_CRC, K_RETIRED, K_ENC_PREP, K_ENC_SCAN, K_ENC_EVENTS, K_ENC_WRITE, K_ENC_HINT_LAYOUT,
                K_ENC_EVENTS_HINT, K_NUM };
struct Prof {
  uint32_t mask = 0;   // bit k: time kernel id k
  uint32_t every = 1;  // time every `every`-th launch of a selected kernel
  uint32_t seq[K_NUM] = {};
  bool open[K_NUM] = {};
  struct Mark { int kid; hipEvent_t a, b; };
  std::vector<Mark> marks;
  std::vector<hipEvent_t> pool;
  hipEvent_t get() {
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  bool on(int kid) const { return (mask >> kid) & 1u; }
  void begin(int kid, hipStream_t s, hipEvent_t& a) {
    open[kid] = on(kid) && (seq[kid]++ % every) == 0;
    if (open[kid]) { a = get(); (void)hipEventRecord(a, s); }
  }
  void end(int kid, hipStream_t s, hipEvent_t a) {
    if (!open[kid]) return;
    open[kid] = false;
    hipEvent_t b = get();
    (void)hipEventRecord(b, s);
    marks.push_back({kid, a, b});
  }
};

// Launch the full decode pipeline on `stream`. Defined in bcw_decode.hip.
hipError_t launch_decode(const uint8_t* d_seg, const bcw_decode_params& p, const bcw_record_table& t,
                         bcw_decode_result* d_result, const Tables& tabs, Scratch& s, uint64_t nblocks,
                         uint64_t gen, hipStream_t stream, int num_cus, Prof* prof);
hipError_t launch_export_frags(const Scratch& s, const bcw_frag_table& out, uint32_t start_off, hipStream_t stream,
                               uint64_t n, const uint32_t* initc);

// Encode scratch (grow-only, per context). rows: source table rows.
struct EncScratch {
  uint64_t rows_cap = 0;
  uint32_t* sz = nullptr;     // [rows] payload size per source row (0: not written)
  uint8_t* mflag = nullptr;   // [rows] meta dropped by Record.Encode
  uint32_t* dsrc = nullptr;   // [rows] dense record -> source row
  uint64_t* da = nullptr;     // [rows+1] dst WAL y-coordinates
  uint64_t* hda = nullptr;    // [rows+1] hint WAL y-coordinates
  uint32_t* hsz = nullptr;    // [rows] hint payload sizes (compaction)
  uint64_t* dpos = nullptr;   // [rows] dst record offsets
  uint64_t* hpos = nullptr;   // [rows] hint record offsets (compaction)
  void* tiles = nullptr;      // scan tile sums
  void* ev = nullptr;         // [rows+2] layout events
  uint32_t* evb = nullptr;    // [rows/win+2] governing event per event-scan window
  uint64_t* evt = nullptr;    // [rows/win+2][32768] per-window entry tables (k_ev_win)
  uint16_t* hnl = nullptr;    // [rows] next event inside the window (k_ev_win)
  uint32_t* evw = nullptr;    // [rows/win+2][3] window entries (k_ev_walk)
  void* recdesc = nullptr;    // [rows] 128 B payload descriptors (k_recdesc_w -> k_write), dst WAL
  uint32_t* wl = nullptr;     // [rows] dst records k_wcopy leaves to k_write<16> / k_write_general
  uint64_t* emisc = nullptr;  // [64] counters
  int wcopy_resident = 0;     // k_wcopy workgroups resident per CU (occupancy query on the context's device, once)
  // the payload descriptors are built on an auxiliary stream while the serial layout scans run
  hipStream_t aux = nullptr;
  hipEvent_t ev_scan = nullptr, ev_hscan = nullptr, ev_desc = nullptr;
};

struct EncLaunch {
  const uint8_t* d_src;
  bcw_encode_params p;
  bcw_record_table table;
  uint64_t rows;
  const bcw_decode_result* d_src_result;
  const uint8_t* d_keep;
  bcw_encode_out out;
  bcw_encode_result* d_result;
  const Frag* frags;
  const uint32_t* crc_ops;
  const uint32_t* initc;
  int num_cus;
  uint64_t gen;  // generation of the context's latest decode (the owner of `frags`)
};

hipError_t launch_encode(const EncLaunch& L, EncScratch& s, hipStream_t stream, Prof* prof);
size_t enc_sizeof_ev();
size_t enc_sizeof_recdesc();
size_t enc_sizeof_tile();
int enc_tile_items();
int enc_ev_win();

// Every C-ABI entry point that touches the device selects the context's device on the calling thread
// and restores the caller's current device when it returns.
struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

// The context an index was created on (bcw_index.hip): the sync entry points refuse an index of another context.
bcw_ctx* index_ctx(const bcw_index* ix);
// doFilter (bcw_compact_filter_async) of context c's latest decode against index x, on c's stream, with the call's
// counters in d_cnt (kIxCounters words of c's device): another context on the index's device filters against the
// index itself, read-only, while no call modifies it (bcw_compact_wals).
constexpr int kIxCounters = 16;
int ix_filter_on(bcw_index* x, bcw_ctx* c, const uint8_t* d_seg, const bcw_decode_params* p,
                 const bcw_record_table* d_table, const bcw_decode_result* d_result, uint64_t src_fid, uint8_t* d_keep,
                 uint64_t* d_cnt, bcw_index_result* d_out);

// Host-side table builders (bcw_api.cpp).
void build_initc(uint32_t* initc);

// The sync API's steps (bcw_api.cpp), shared with the multi-context fan-out (bcw_fanout.cpp): upload + decode into
// the context's device table; the keep mask's scratch; the decode parameters of a source WAL file; the encode of
// the context's decoded source with its keep mask, outputs copied to the host.
int sync_decode(bcw_ctx* c, const uint8_t* h_src, const bcw_decode_params& dp, bcw_decode_result& dres);
int ensure_keep(bcw_ctx* c, uint64_t rows);
bcw_decode_params src_params(const uint8_t* h_src, const bcw_encode_params* p);
int encode_to_host(bcw_ctx* c, const bcw_encode_params* p, const bcw_encode_out* h, bcw_encode_result* h_result,
                   const bcw_decode_result& dres);
// encode_to_host in two steps (bcw_compact_wals): the encode and its result (the dst / hint ends the next source
// starts from), then the copies of the outputs to the host. *d_out: the device-side outputs between the two.
int encode_run(bcw_ctx* c, const bcw_encode_params* p, const bcw_encode_out* h, bcw_encode_result* h_result,
               bcw_encode_out* d_out);
int encode_copy_out(bcw_ctx* c, const bcw_encode_params* p, const bcw_encode_out* h, const bcw_encode_result& r,
                    const bcw_encode_out& d, const bcw_decode_result& dres);

// Export of an index's live entries (bcw_index.hip) into host arrays the sink provides once the sizes are known:
// room(n, key_bytes) fills the five pointers (koff has n + 1 entries) or refuses (BCW_E_CAPACITY). h_fids / n_fids
// (n_fids > 0): only entries whose value fid is one of them.
struct IxSink {
  virtual ~IxSink() = default;
  virtual int room(uint64_t n, uint64_t key_bytes) = 0;
  uint8_t* keys = nullptr;
  uint64_t* koff = nullptr;
  uint64_t* fid = nullptr;
  uint64_t* off = nullptr;
  uint64_t* size = nullptr;
};
int ix_export(bcw_index* x, const uint64_t* h_fids, uint64_t n_fids, IxSink& sink, uint64_t* n_out,
              uint64_t* key_bytes);

}  // namespace bcw

// The context behind the C-ABI handle (bcw.h): one device, one launch stream, constant tables and
// grow-only scratch. Defined here so every translation unit of libbcw.so can reach its stream,
// device and the fragment table of its latest decode.
struct bcw_ctx {
  int device = 0;
  uint64_t id = 0;         // unique per context (high half of every decode generation)
  uint64_t gen_seq = 0;    // decodes issued on this context
  uint64_t frag_gen = 0;   // generation of the decode whose fragment table the scratch holds
  int num_cus = 256;
  hipStream_t own = nullptr;
  hipStream_t cur = nullptr;
  bcw::Tables tabs{};
  bcw::Scratch s{};
  bcw::EncScratch es{};
  // sync encode staging
  uint8_t* d_keep = nullptr;
  uint64_t d_keep_cap = 0;
  void* d_eout = nullptr;
  uint64_t d_eout_cap = 0;
  bcw_encode_result* d_eres = nullptr;
  uint64_t frag_hint = 0;  // capacity requested by a retry
  // sync-API staging
  uint8_t* d_seg = nullptr;
  uint64_t d_seg_cap = 0;
  void* d_tab_mem = nullptr;
  uint64_t d_tab_cap = 0;
  bcw_record_table d_tab{};
  bcw_decode_result* d_result = nullptr;
  bcw_index_result* d_ires = nullptr;  // sync index calls
  uint32_t last_start_off = 0;
  uint32_t chase_direct = BCW_CHASE_DIRECT_MAX;  // BCW_OPT_CHASE_DIRECT
  uint64_t test_abort_wg = 0;                    // BCW_OPT_TEST_ABORT_WAIT (one-shot)
  bool filter_snapshot = false;                  // BCW_OPT_FILTER_SNAPSHOT (bcw_compact_wals)
  uint64_t last_nfrag_cap = 0;
  bcw::Prof prof;
};
