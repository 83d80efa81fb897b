// bcw_io.cpp -- host I/O staging between WAL files and HBM: the reference reads a
// segment with PreadFull per 32 KiB block (utils.go:32-48, wal_iterator.go:55) and writes the rewritten
// WAL through a buffer flushed every >= 1 MiB (WalRewriter, wal_rewriter.go:37-49 -> Wal.Flush
// wal.go:451-465). Here a whole segment moves between a file descriptor and device memory through
// pinned staging slices: reader threads pread slices into pinned buffers while earlier slices are
// already crossing PCIe (hipMemcpyAsync on the caller's stream), and device output comes back in
// slices whose pwrite overlaps the next slice's copy.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <new>
#include <thread>
#include <vector>

#include "bcw.h"
#include "bcw_internal.h"

namespace {

struct Slot {
  uint8_t* host = nullptr;  // pinned
  hipEvent_t done = nullptr;
  bool busy = false;
};

}  // namespace

struct bcw_stage {
  bcw_ctx* ctx = nullptr;
  uint64_t slice = 0;
  std::vector<Slot> slots;
};

using namespace bcw;

extern "C" {

int bcw_stage_create(bcw_ctx* c, uint64_t slice_bytes, uint32_t nslices, bcw_stage** out) {
  if (!c || !out || slice_bytes < 4096 || nslices < 2 || nslices > 64) return BCW_E_INVAL;
  *out = nullptr;
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  bcw_stage* s = new (std::nothrow) bcw_stage();
  if (!s) return BCW_E_NOMEM;
  s->ctx = c;
  s->slice = slice_bytes;
  s->slots.resize(nslices);
  for (Slot& q : s->slots) {
    if (hipHostMalloc(reinterpret_cast<void**>(&q.host), slice_bytes, hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&q.done, hipEventDisableTiming) != hipSuccess) {
      bcw_stage_destroy(s);
      return BCW_E_NOMEM;
    }
  }
  *out = s;
  return BCW_OK;
}

int bcw_stage_destroy(bcw_stage* s) {
  if (!s) return BCW_E_INVAL;
  DeviceGuard dg(s->ctx->device);
  for (Slot& q : s->slots) {
    if (q.done) { (void)hipEventSynchronize(q.done); (void)hipEventDestroy(q.done); }
    if (q.host) (void)hipHostFree(q.host);
  }
  delete s;
  return BCW_OK;
}

int bcw_stage_read(bcw_stage* s, int fd, uint64_t file_off, uint64_t len, uint8_t* d_dst, void* hip_stream,
                   uint32_t threads) {
  if (!s || fd < 0 || (len && !d_dst)) return BCW_E_INVAL;
  if (len == 0) return BCW_OK;
  DeviceGuard dg(s->ctx->device);
  if (!dg.ok) return BCW_E_HIP;
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : s->ctx->cur;
  // a descriptor opened with O_DIRECT (reads from the device, past the page cache, like the reference's io_uring
  // block reader on an O_DIRECT file, block_reader/iouring.go): offsets 4 KiB-aligned, every request a whole
  // number of 4 KiB units (the pinned slices are page-aligned; a short read at end of file is the tail)
  const int fl = fcntl(fd, F_GETFL);
  const bool direct = fl >= 0 && (fl & O_DIRECT) != 0;
  constexpr uint64_t kDio = 4096;
  if (direct && (file_off % kDio != 0 || s->slice % kDio != 0)) return BCW_E_INVAL;
  const uint64_t nsl = (len + s->slice - 1) / s->slice;
  const uint32_t ns = (uint32_t)s->slots.size();
  const uint32_t nt = std::max<uint32_t>(1, std::min<uint32_t>({threads ? threads : 4, ns, (uint32_t)nsl}));
  std::atomic<int> err{BCW_OK};
  // thread t owns slots t, t + nt, ... and slices t, t + nt, ... (slice k uses slot k % (ns / nt * nt))
  const uint32_t per = ns / nt;
  auto worker = [&](uint32_t t) {
    uint32_t use = 0;
    for (uint64_t k = t; k < nsl && err.load() == BCW_OK; k += nt, ++use) {
      Slot& q = s->slots[t + nt * (use % per)];
      if (q.busy && hipEventSynchronize(q.done) != hipSuccess) { err = BCW_E_HIP; return; }
      const uint64_t off = k * s->slice, n = std::min(s->slice, len - off);
      uint64_t got = 0;
      while (got < n) {  // PreadFull (utils.go:32-48)
        const uint64_t want = direct ? (n - got + kDio - 1) / kDio * kDio : n - got;  // <= slice - got
        const ssize_t r = pread(fd, q.host + got, want, (off_t)(file_off + off + got));
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) { err = BCW_E_IO; return; }
        got += (uint64_t)r;
        if (direct && got < n && (got % kDio) != 0) { err = BCW_E_IO; return; }  // a short read before the end
      }
      if (hipMemcpyAsync(d_dst + off, q.host, n, hipMemcpyHostToDevice, st) != hipSuccess ||
          hipEventRecord(q.done, st) != hipSuccess) {
        err = BCW_E_HIP;
        return;
      }
      q.busy = true;
    }
  };
  std::vector<std::thread> th;
  for (uint32_t t = 1; t < nt; ++t) th.emplace_back(worker, t);
  worker(0);
  for (auto& x : th) x.join();
  return err.load();
}

int bcw_stage_write(bcw_stage* s, int fd, uint64_t file_off, const uint8_t* d_src, uint64_t len, void* hip_stream,
                    uint32_t threads) {
  if (!s || fd < 0 || (len && !d_src)) return BCW_E_INVAL;
  if (len == 0) return BCW_OK;
  DeviceGuard dg(s->ctx->device);
  if (!dg.ok) return BCW_E_HIP;
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : s->ctx->cur;
  const uint64_t nsl = (len + s->slice - 1) / s->slice;
  const uint32_t ns = (uint32_t)s->slots.size();
  const uint32_t nt = std::max<uint32_t>(1, std::min<uint32_t>({threads ? threads : 4, ns, (uint32_t)nsl}));
  const uint32_t per = ns / nt;
  std::atomic<int> err{BCW_OK};
  // thread t: slices t, t + nt, ...: the slice's copy is queued on the stream (after the work that
  // produced the data), then pwritten once it has landed while the other threads' copies proceed
  auto worker = [&](uint32_t t) {
    uint32_t use = 0;
    for (uint64_t k = t; k < nsl && err.load() == BCW_OK; k += nt, ++use) {
      Slot& q = s->slots[t + nt * (use % per)];
      if (q.busy && hipEventSynchronize(q.done) != hipSuccess) { err = BCW_E_HIP; return; }  // an earlier read
      const uint64_t off = k * s->slice, n = std::min(s->slice, len - off);
      if (hipMemcpyAsync(q.host, d_src + off, n, hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipEventRecord(q.done, st) != hipSuccess || hipEventSynchronize(q.done) != hipSuccess) {
        err = BCW_E_HIP;
        return;
      }
      q.busy = false;
      uint64_t put = 0;
      while (put < n) {
        const ssize_t r = pwrite(fd, q.host + put, n - put, (off_t)(file_off + off + put));
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) { err = BCW_E_IO; return; }
        put += (uint64_t)r;
      }
    }
  };
  std::vector<std::thread> th;
  for (uint32_t t = 1; t < nt; ++t) th.emplace_back(worker, t);
  worker(0);
  for (auto& x : th) x.join();
  return err.load();
}

int bcw_peer_enable(int a, int b) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || a < 0 || b < 0 || a >= n || b >= n) return BCW_E_INVAL;
  if (a == b) return BCW_OK;
  for (int k = 0; k < 2; ++k) {
    const int from = k ? b : a, to = k ? a : b;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, from, to) != hipSuccess || !can) return BCW_E_HIP;
    DeviceGuard dg(from);
    if (!dg.ok) return BCW_E_HIP;
    const hipError_t e = hipDeviceEnablePeerAccess(to, 0);
    if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();  // (clears the sticky status)
    else if (e != hipSuccess) return BCW_E_HIP;
  }
  return BCW_OK;
}

int bcw_stage_peer(bcw_ctx* c, uint8_t* d_dst, const uint8_t* d_src, int src_device, uint64_t len, void* hip_stream) {
  if (!c || (len && (!d_dst || !d_src)) || src_device < 0) return BCW_E_INVAL;
  if (!len) return BCW_OK;
  DeviceGuard dg(c->device);
  if (!dg.ok) return BCW_E_HIP;
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->cur;
  const hipError_t e = src_device == c->device
                           ? hipMemcpyAsync(d_dst, d_src, len, hipMemcpyDeviceToDevice, st)
                           : hipMemcpyPeerAsync(d_dst, c->device, d_src, src_device, len, st);
  return e == hipSuccess ? BCW_OK : BCW_E_HIP;
}

}  // extern "C"
