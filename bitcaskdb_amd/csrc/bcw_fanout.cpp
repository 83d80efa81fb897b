// bcw_fanout.cpp -- one process, several contexts (devices): the index rebuild and the compaction of many WAL files
// with the decodes spread over the contexts, one host thread each, while the puts into the index and the appends to
// the dst files keep the reference's order.
//   recoverFromWals   db_impl.go:268-314   bcw_recover_wals
//   doCompactionWork  compaction.go:201-211 (compactOneWal + doFilter, compaction.go:294-348)   bcw_compact_wals
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <numeric>
#include <thread>
#include <vector>

#include "bcw.h"
#include "bcw_internal.h"

using namespace bcw;

namespace {

// an index export held on the host
struct Entries : IxSink {
  std::vector<uint8_t> k;
  std::vector<uint64_t> ko, f, o, z;
  uint64_t n = 0;
  int room(uint64_t n_, uint64_t kb) override {
    n = n_;
    k.resize(std::max<uint64_t>(kb, 1));
    ko.resize(n_ + 1);
    f.resize(std::max<uint64_t>(n_, 1));
    o.resize(f.size());
    z.resize(f.size());
    keys = k.data();
    koff = ko.data();
    fid = f.data();
    off = o.data();
    size = z.data();
    return BCW_OK;
  }
  void release() {
    std::vector<uint8_t>().swap(k);
    std::vector<uint64_t>().swap(ko);
    std::vector<uint64_t>().swap(f);
    std::vector<uint64_t>().swap(o);
    std::vector<uint64_t>().swap(z);
    n = 0;
  }
};

// Index.Put of every exported entry, in one batch (the keys of one export are distinct)
int put_entries(bcw_index* ix, const Entries& e, uint64_t lo = 0, uint64_t hi = ~0ull) {
  hi = std::min(hi, e.n);
  if (lo >= hi) return BCW_OK;
  const std::vector<uint8_t> ops(hi - lo, BCW_IDX_PUT);
  return bcw_index_apply(ix, hi - lo, e.k.data(), e.ko.data() + lo, ops.data(), e.f.data() + lo, e.o.data() + lo,
                         e.z.data() + lo);
}

// the fragment errors IterateRecord / IterateHint return (record.go:246-263); BCW_ERR_INTERNAL: the decode gave up
bool frag_error(int32_t e) {
  return e == BCW_ERR_CRC || e == BCW_ERR_TYPE || e == BCW_ERR_PANIC || e == BCW_ERR_INTERNAL;
}

// a staging index on a worker's context, created with the first file's sizes, capped (it grows on demand)
struct Staging {
  bcw_index* ix = nullptr;
  ~Staging() {
    if (ix) (void)bcw_index_destroy(ix);
  }
  int ready(bcw_ctx* c, uint64_t keys, uint64_t arena) {
    if (ix) return bcw_index_clear(ix);
    return bcw_index_create(c, std::min<uint64_t>(std::max<uint64_t>(keys, 1024), 1ull << 20),
                            std::min<uint64_t>(std::max<uint64_t>(arena, 1 << 16), 64ull << 20), &ix);
  }
};

struct RecoverSlot {
  bool ready = false;
  bool stop = false;
  Entries e;
};

// one file of recoverFromWal (db_impl.go:286-313) into the staging index: its status and whether recovery stops
bool recover_one(bcw_ctx* c, bcw_index* stg, const bcw_recover_file& F, bcw_recover_status& S) {
  if (F.hint) {
    S.used = BCW_RECOVER_HINT;
    S.rc = bcw_index_recover_segment(c, stg, F.hint, &F.hint_p, F.fid, 0, &S.hint_dres, &S.hint_ires);
    if (S.rc != BCW_OK || S.hint_ires.err_class) return true;
    const bool rejected = S.hint_ires.n_in < S.hint_dres.n_records;  // a corrupted hint record
    if (!rejected && S.hint_dres.err_class == BCW_ERR_INTERNAL) return true;
    if (!rejected && !frag_error(S.hint_dres.err_class)) return false;
    S.used = BCW_RECOVER_HINT_WAL;  // IterateHint failed: the data WAL, keeping the hint's puts
  } else {
    S.used = BCW_RECOVER_WAL;
  }
  S.rc = bcw_index_recover_segment(c, stg, F.wal, &F.wal_p, F.fid, 0, &S.wal_dres, &S.wal_ires);
  return S.rc != BCW_OK || S.wal_ires.err_class || S.wal_ires.n_in < S.wal_dres.n_records ||
         frag_error(S.wal_dres.err_class);
}

// every context non-null and named once: each worker thread owns its context's scratch (decode tables, keep mask,
// staging), so one context listed twice would have two threads decoding into the same buffers (bcw.h: a context
// belongs to one caller thread at a time)
bool distinct_contexts(bcw_ctx* const* ctxs, uint32_t n) {
  for (uint32_t w = 0; w < n; ++w) {
    if (!ctxs[w]) return false;
    for (uint32_t v = 0; v < w; ++v)
      if (ctxs[v] == ctxs[w]) return false;
  }
  return true;
}

}  // namespace

extern "C" {

int bcw_recover_wals(bcw_index* ix, bcw_ctx* const* ctxs, uint32_t n_ctx, const bcw_recover_file* files,
                     uint64_t n_files, bcw_recover_status* st, int64_t* stop_file) {
  if (!ix || !ctxs || !n_ctx || (n_files && (!files || !st)) || !stop_file) return BCW_E_INVAL;
  if (!distinct_contexts(ctxs, n_ctx)) return BCW_E_INVAL;
  for (uint64_t i = 0; i < n_files; ++i) {
    const bcw_recover_file& F = files[i];
    if ((F.wal_p.seg_len && !F.wal) || F.wal_p.mode != BCW_MODE_RECORD) return BCW_E_INVAL;
    if (F.hint && F.hint_p.mode != BCW_MODE_HINT) return BCW_E_INVAL;
    st[i] = bcw_recover_status{};
  }
  *stop_file = -1;
  std::vector<uint64_t> order(n_files);  // db_impl.go:269-274: ascending fid
  std::iota(order.begin(), order.end(), 0ull);
  std::stable_sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return files[a].fid < files[b].fid; });

  std::vector<RecoverSlot> slot(n_files);
  std::mutex mu;
  std::condition_variable cv;
  uint64_t applied = 0;  // files whose puts the index has received
  bool quit = false;
  const uint64_t ahead = 2ull * n_ctx;  // exports held on the host at most (per context: the one applied next + 1)

  auto worker = [&](uint32_t w) {
    Staging stg;
    for (uint64_t j = w; j < n_files; j += n_ctx) {
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return quit || j < applied + ahead; });
        if (quit) return;
      }
      const bcw_recover_file& F = files[order[j]];
      bcw_recover_status& S = st[order[j]];
      bool stop = true;
      const uint64_t seg = std::max(F.wal_p.seg_len, F.hint ? F.hint_p.seg_len : 0);
      S.rc = stg.ready(ctxs[w], seg / 64 + 16, seg / 4 + 4096);
      if (S.rc == BCW_OK) stop = recover_one(ctxs[w], stg.ix, F, S);
      uint64_t n = 0, kb = 0;
      RecoverSlot& R = slot[j];
      if (S.rc == BCW_OK && (S.rc = ix_export(stg.ix, nullptr, 0, R.e, &n, &kb)) != BCW_OK) stop = true;
      {
        std::lock_guard<std::mutex> lk(mu);
        R.stop = stop;
        R.ready = true;
      }
      cv.notify_all();
      if (stop) return;  // the files after this one are not applied
    }
  };
  std::vector<std::thread> pool;
  pool.reserve(n_ctx);
  for (uint32_t w = 0; w < n_ctx && w < n_files; ++w) pool.emplace_back(worker, w);

  int rc = BCW_OK;
  for (uint64_t j = 0; j < n_files; ++j) {
    RecoverSlot& R = slot[j];
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return R.ready; });
    }
    const uint64_t i = order[j];
    if (st[i].rc == BCW_OK) rc = put_entries(ix, R.e);
    R.e.release();
    {
      std::lock_guard<std::mutex> lk(mu);
      applied = j + 1;
      if (rc != BCW_OK || R.stop) quit = true;
    }
    cv.notify_all();
    if (R.stop) *stop_file = (int64_t)i;
    if (rc != BCW_OK || R.stop) break;
  }
  for (auto& t : pool) t.join();
  return rc;
}

int bcw_compact_wals(bcw_index* ix, bcw_ctx* const* ctxs, uint32_t n_ctx, const bcw_compact_src* srcs,
                     uint64_t n_src, const bcw_encode_params* dst, bcw_encode_result* res, bcw_index_result* filt,
                     uint64_t* n_done) {
  if (!ix || !ctxs || !n_ctx || !dst || !n_done || (n_src && (!srcs || !res || !filt))) return BCW_E_INVAL;
  if (!distinct_contexts(ctxs, n_ctx)) return BCW_E_INVAL;
  for (uint64_t k = 0; k < n_src; ++k) {
    if (srcs[k].len && !srcs[k].data) return BCW_E_INVAL;
    res[k] = bcw_encode_result{};
    filt[k] = bcw_index_result{};
  }
  *n_done = 0;
  if (!n_src) return BCW_OK;

  // A context on the index's device filters against the index itself (read-only: nothing modifies it during the
  // call; its own stream's work is drained first). The others filter against a snapshot: the index's entries that
  // point into the sources, split by fid, each source's slice loaded into a staging index on that context.
  bcw_ctx* const ixc = index_ctx(ix);
  if (!ixc) return BCW_E_INVAL;
  bool any_remote = false;
  for (uint32_t w = 0; w < n_ctx; ++w) any_remote |= ctxs[w]->device != ixc->device || ctxs[w]->filter_snapshot;
  {
    DeviceGuard dg(ixc->device);
    if (!dg.ok || hipStreamSynchronize(ixc->cur) != hipSuccess) return BCW_E_HIP;
  }
  std::vector<uint64_t> fids(n_src);
  for (uint64_t k = 0; k < n_src; ++k) fids[k] = srcs[k].fid;
  Entries snap;
  uint64_t sn = 0, skb = 0;
  if (any_remote) {
    const int rc = ix_export(ix, fids.data(), n_src, snap, &sn, &skb);
    if (rc != BCW_OK) return rc;
  }
  std::vector<uint64_t> by(sn);  // entry indices grouped by fid
  std::iota(by.begin(), by.end(), 0ull);
  std::stable_sort(by.begin(), by.end(), [&](uint64_t a, uint64_t b) { return snap.f[a] < snap.f[b]; });

  std::mutex mu;
  std::condition_variable cv;
  uint64_t turn = 0;  // the source whose encode runs next
  std::vector<uint8_t> copied(n_src, 0);  // sources whose outputs reached the host
  uint64_t wal_pos = dst->wal_pos, hint_pos = dst->hint_pos;
  bool quit = false;
  int err = BCW_OK;

  auto worker = [&](uint32_t w) {
    bcw_ctx* c = ctxs[w];
    const bool direct = c->device == ixc->device && !c->filter_snapshot;
    Staging stg;
    Entries mine;
    uint64_t* d_cnt = nullptr;  // (direct) the filter's counters
    struct FreeCnt {
      bcw_ctx* c;
      uint64_t*& p;
      ~FreeCnt() {
        if (p) {
          DeviceGuard dg(c->device);
          (void)hipFree(p);
        }
      }
    } free_cnt{c, d_cnt};
    for (uint64_t k = w; k < n_src; k += n_ctx) {
      const bcw_compact_src& S = srcs[k];
      bcw_encode_params p = *dst;
      p.src_len = S.len;
      p.src_start_off = S.start_off;
      p.mode = BCW_ENC_COMPACT;
      // this source's slice of the snapshot, loaded into the staging index
      auto lo = std::lower_bound(by.begin(), by.end(), S.fid, [&](uint64_t e, uint64_t f) { return snap.f[e] < f; });
      auto hi = std::upper_bound(lo, by.end(), S.fid, [&](uint64_t f, uint64_t e) { return f < snap.f[e]; });
      const uint64_t m = direct ? 0 : (uint64_t)(hi - lo);
      int r = BCW_OK;
      if (direct && !d_cnt) {
        DeviceGuard dg(c->device);
        r = dg.ok && hipMalloc(&d_cnt, kIxCounters * sizeof(uint64_t)) == hipSuccess ? BCW_OK : BCW_E_HIP;
      }
      if (!direct) r = stg.ready(c, m + 16, 64 * m + 4096);
      if (r == BCW_OK && m) {
        mine.room(m, 0);
        mine.k.clear();
        for (uint64_t q = 0; q < m; ++q) {
          const uint64_t e = lo[q];
          mine.ko[q] = mine.k.size();
          mine.k.insert(mine.k.end(), snap.k.begin() + snap.ko[e], snap.k.begin() + snap.ko[e + 1]);
          mine.f[q] = snap.f[e];
          mine.o[q] = snap.o[e];
          mine.z[q] = snap.z[e];
        }
        mine.ko[m] = mine.k.size();
        if (mine.k.empty()) mine.k.push_back(0);
        r = put_entries(stg.ix, mine);
      }
      // upload + decode + doFilter against the slice (the same keep mask as against the whole index: a row is
      // kept when Get(key) points at (src fid, foff - 7), and every entry that can do so is in the slice)
      bcw_decode_result dres{};
      const bcw_decode_params dp = src_params(S.data, &p);
      if (r == BCW_OK) {
        DeviceGuard dg(c->device);
        r = dg.ok ? sync_decode(c, S.data, dp, dres) : BCW_E_HIP;
        if (r == BCW_OK) r = ensure_keep(c, c->d_tab.capacity);
        if (r == BCW_OK)
          r = direct ? ix_filter_on(ix, c, c->d_seg, &dp, &c->d_tab, c->d_result, S.fid, c->d_keep, d_cnt, c->d_ires)
                     : bcw_compact_filter_async(stg.ix, c->d_seg, &dp, &c->d_tab, c->d_result, S.fid, c->d_keep,
                                                c->d_ires);
        if (r == BCW_OK && (hipMemcpyAsync(&filt[k], c->d_ires, sizeof filt[k], hipMemcpyDeviceToHost, c->cur) !=
                                hipSuccess ||
                            hipStreamSynchronize(c->cur) != hipSuccess))
          r = BCW_E_HIP;
      }
      // the encode, in source order: the turn is held until its result (the dst / hint ends) is in; the copies of
      // its outputs to the host then run beside the next source's encode (only the ends chain the sources,
      // compaction.go:294-327 appends each source where the previous one ended)
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return quit || turn == k; });
        if (quit) return;
        p.wal_pos = wal_pos;
        p.hint_pos = hint_pos;
      }
      bcw_encode_out dout{};
      if (r == BCW_OK) {
        DeviceGuard dg(c->device);
        r = dg.ok ? encode_run(c, &p, &S.out, &res[k], &dout) : BCW_E_HIP;
      }
      {
        std::lock_guard<std::mutex> lk(mu);
        if (r != BCW_OK) {
          err = r;
          quit = true;
        } else {
          wal_pos = res[k].wal_end;
          hint_pos = res[k].hint_end;
          if (res[k].err_class != BCW_ENC_ERR_NONE) quit = true;  // doCompactionWork returns the error
          turn = k + 1;
        }
      }
      cv.notify_all();
      if (r != BCW_OK) return;
      {
        DeviceGuard dg(c->device);
        r = dg.ok ? encode_copy_out(c, &p, &S.out, res[k], dout, dres) : BCW_E_HIP;
      }
      {
        std::lock_guard<std::mutex> lk(mu);
        if (r != BCW_OK) {
          if (err == BCW_OK) err = r;
          quit = true;
        } else {
          copied[k] = 1;
          while (*n_done < n_src && copied[*n_done]) ++*n_done;  // the leading sources whose output is final
        }
      }
      cv.notify_all();
      if (r != BCW_OK) return;
    }
  };
  std::vector<std::thread> pool;
  pool.reserve(n_ctx);
  for (uint32_t w = 0; w < n_ctx && w < n_src; ++w) pool.emplace_back(worker, w);
  for (auto& t : pool) t.join();
  return err;
}

}  // extern "C"
