#!/usr/bin/env python3
"""Config E measurement: compaction re-encode (compactOneWal: Record.Encode + WriteRecord + hint) of
N records (default 10 M, NsSize 20, 100 B keys, 4 KiB values, every record kept, dst baseTime = src
baseTime) on one MI355X, device-resident, through the C-ABI (bcw_decode_segment_async then
bcw_encode_segment_async on the same context).

Full-size parity: with everything kept and equal baseTimes the re-encoded records equal the source
records and a fresh dst WAL repeats the source layout, so the appended dst bytes must equal the source
file from byte 40 (checked with torch.equal on the device); the hint WAL is decoded back on the device
and its (off, size) fields must equal the returned offsets / source sizes. Prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BASE_TIME = 1_700_000_000
HBM_PEAK_GBS = 8000.0


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds: float) -> dict:
    """the oracle's restated compactOneWal (oc_compact_append: iterate, Record.Encode, WriteRecord,
    HintRecord.Encode; 1 thread) over a bounded sample of the same record shape, in GB/s of the same
    algorithmic bytes (source read + WAL + hint written) and records/s"""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O  # noqa: E402  (cpu_baseline leg only)
    src = np.frombuffer(O.synth(256 << 20, 0, 42, 20, 100, 4096, 0, BASE_TIME), dtype=np.uint8)
    dec = O.decode(src, 40, BASE_TIME, 20, 20, want_bytes=False)
    keep = np.ones(len(dec.recs), np.uint8)
    passes, alg, t = 0, 0, time.perf_counter()
    while True:
        dst, hint = O.Writer(BASE_TIME, BASE_TIME), O.Writer(BASE_TIME, BASE_TIME)
        ec, _, nin, _ = O.compact_append(dst, hint, 1, src, 40, BASE_TIME, BASE_TIME, 20, 20, keep)
        assert ec == 0 and nin == len(keep)
        alg += src.size + (dst.size() - 40) + (hint.size() - 40)
        passes += 1
        if time.perf_counter() - t >= seconds:
            break
    dt = time.perf_counter() - t
    return {"value": round(alg / dt / 1e9, 3), "unit": "GB/s (src read + WAL + hint written)", "cores": 1,
            "kind": "port", "records_per_s": round(passes * len(keep) / dt),
            "sample": f"{passes} compactions of a {src.size} B segment ({len(keep)} records of the config-E shape) "
                      f"with the restated compactOneWal (oc_compact_append, SSE4.2 CRC), 1 thread, {dt:.1f} s, "
                      f"{cpu_model()}"}


def index_leg(L, ctx, stream, d_src, dparams, table, d_res, n_rec, steps, decode_checked, encode, keep):
    """SURVEY.md §8 f2 / f1 on the same 10 M records: the index rebuild (recoverFromWal's Put of every
    delivered row, bcw_index_put_decoded_async) into an empty device index, then the compaction filter
    (doFilter against that index, bcw_compact_filter_async) producing the keep mask the encode consumes.
    Every row must be kept (the index points at exactly these records)."""
    import torch
    from bitcaskdb_amd.index import Index
    ix = Index(ctx, keys=n_rec + (n_rec >> 2), arena_bytes=n_rec * 160 + (1 << 20))
    d_ir = torch.zeros(C.sizeof(L.IndexResult), dtype=torch.uint8, device=d_src.device)
    decode_checked(d_src.data_ptr(), dparams)

    def put():
        assert L.lib.bcw_index_put_decoded_async(ix.handle, C.c_void_p(d_src.data_ptr()), C.byref(dparams),
                                                 C.byref(table), C.c_void_p(d_res.data_ptr()), 7, 0,
                                                 C.c_void_p(d_ir.data_ptr())) == 0

    def filt():
        assert L.lib.bcw_compact_filter_async(ix.handle, C.c_void_p(d_src.data_ptr()), C.byref(dparams),
                                              C.byref(table), C.c_void_p(d_res.data_ptr()), 7,
                                              C.c_void_p(keep.data_ptr()), C.c_void_p(d_ir.data_ptr())) == 0

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    put()  # first insert of every key into the empty index (slot claims)
    e1.record(stream)
    torch.cuda.synchronize()
    first_ms = e0.elapsed_time(e1)
    r = L.IndexResult.from_buffer_copy(bytes(d_ir.cpu().numpy()))
    assert r.err_class == 0 and r.n_done == n_rec, (r.err_class, r.n_done)
    e0.record(stream)
    for _ in range(steps):
        put()  # rebuild over an index already holding the keys (replace in place)
    e1.record(stream)
    torch.cuda.synchronize()
    put_ms = e0.elapsed_time(e1) / steps
    keep.zero_()
    e0.record(stream)
    for _ in range(steps):
        filt()
    e1.record(stream)
    torch.cuda.synchronize()
    filt_ms = e0.elapsed_time(e1) / steps
    r = L.IndexResult.from_buffer_copy(bytes(d_ir.cpu().numpy()))
    kept = int(keep[:n_rec].sum().item())
    assert r.err_class == 0 and kept == n_rec, (r.err_class, kept)
    # decode -> filter -> encode without leaving HBM (the whole device compactOneWal with doFilter)
    e0.record(stream)
    for _ in range(steps):
        decode_checked_async = L.lib.bcw_decode_segment_async(ctx.handle, C.c_void_p(d_src.data_ptr()),
                                                              C.byref(dparams), C.byref(table),
                                                              C.c_void_p(d_res.data_ptr()))
        assert decode_checked_async == 0
        filt()
        encode()
    e1.record(stream)
    torch.cuda.synchronize()
    full_ms = e0.elapsed_time(e1) / steps
    st = ix.stats()
    ix.close()
    return {"rebuild_first_insert_ms": round(first_ms, 3), "rebuild_put_ms": round(put_ms, 3), "rebuild_keys_per_s": round(n_rec / (put_ms * 1e-3)),
            "filter_ms": round(filt_ms, 3), "filter_rows_per_s": round(n_rec / (filt_ms * 1e-3)),
            "decode_filter_encode_ms": round(full_ms, 3), "kept": kept, "index_live": int(st.live),
            "note": "rebuild = recoverFromWal Put of every delivered row (murmur3 over ns||key, probe, last op "
                    "wins) into a device index already holding the keys; filter = doFilter Get + (fid, off) "
                    "compare per row; decode_filter_encode = decode + filter + re-encode + hint, all in HBM"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--out", default=None)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-index", action="store_true", help="skip the index rebuild / compaction filter leg")
    args = ap.parse_args()
    line = measure(args.records, args.steps, args.warmup, with_index=not args.no_index, realistic=True)
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    s = json.dumps(line)
    print(s, flush=True)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(s + "\n")
    if not (line["parity"]["wal_equals_source"] and line["parity"]["hint_decodes_to_offsets"]
            and all(line["realistic"]["parity"].values())):
        raise SystemExit("config E parity check failed")


def measure(records: int, steps: int, warmup: int, with_index: bool = False, realistic: bool = False) -> dict:
    """the config-E encode of `records` records (synthesised on the host, uploaded once): warmup untimed encodes,
    then `steps` timed ones (HIP events on the codec's stream); also used by bench.py's encode_e key"""
    import torch
    from bitcaskdb_amd import _lib as L
    from bitcaskdb_amd import Context

    dev = torch.device("cuda", torch.cuda.current_device())
    t0 = time.time()
    n, r = C.c_uint64(), C.c_uint64()
    assert L.lib.bcw_synth_segment(1 << 62, records, 42, 20, 100, 4096, 0, BASE_TIME, None, 0, C.byref(n),
                                   C.byref(r)) == 0
    host = np.empty(n.value, dtype=np.uint8)  # (pageable: pinning 42 GB costs more than the copy it saves)
    assert L.lib.bcw_synth_segment(1 << 62, records, 42, 20, 100, 4096, 0, BASE_TIME,
                                   C.c_void_p(host.ctypes.data), n.value, C.byref(n), C.byref(r)) == 0
    seg_len, n_rec = int(n.value), int(r.value)
    print(f"synth {seg_len} B, {n_rec} records in {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    d_src = torch.from_numpy(host).to(dev)
    torch.cuda.synchronize()
    del host

    cap = n_rec + 64
    cols = {}
    for name, dt in L.TABLE_COLUMNS:
        tdt = {"u8": torch.int64, "u4": torch.int32, "u1": torch.uint8}[dt]
        cols[name] = torch.empty(cap, dtype=tdt, device=dev)
    ptr_t = {"u8": L.u64p, "u4": L.u32p, "u1": L.u8p}
    table = L.RecordTable(cap, *[C.cast(C.c_void_p(cols[nm].data_ptr()), ptr_t[dt]) for nm, dt in L.TABLE_COLUMNS])
    d_res = torch.zeros(C.sizeof(L.DecodeResult), dtype=torch.uint8, device=dev)
    d_eres = torch.zeros(C.sizeof(L.EncodeResult), dtype=torch.uint8, device=dev)
    keep = torch.ones(cap, dtype=torch.uint8, device=dev)
    wal_cap = seg_len + (seg_len >> 6)
    hint_cap = n_rec * 160 + (1 << 20)
    d_wal = torch.empty(wal_cap, dtype=torch.uint8, device=dev)
    d_hint = torch.empty(hint_cap, dtype=torch.uint8, device=dev)
    d_off = torch.empty(cap, dtype=torch.int64, device=dev)
    dparams = L.DecodeParams(seg_len, BASE_TIME, 40, 20, 20, L.MODE_RECORD)
    eparams = L.EncodeParams(seg_len, BASE_TIME, 1, 40, 40, 40, L.ENC_COMPACT, 20, 20)
    out = L.EncodeOut(C.cast(C.c_void_p(d_wal.data_ptr()), L.u8p), wal_cap,
                      C.cast(C.c_void_p(d_hint.data_ptr()), L.u8p), hint_cap,
                      C.cast(C.c_void_p(d_off.data_ptr()), L.u64p))
    ctx = Context(0)
    stream = torch.cuda.Stream()
    ctx.set_stream(stream.cuda_stream)

    def decode():
        assert L.lib.bcw_decode_segment_async(ctx.handle, C.c_void_p(d_src.data_ptr()), C.byref(dparams),
                                              C.byref(table), C.c_void_p(d_res.data_ptr())) == 0

    def decode_checked(seg_ptr, prm):
        # async API contract: a result with retry_frag_capacity != 0 is invalid; reserve that many fragments
        # on the context (bcw_ctx_reserve_fragments) and decode again
        for _ in range(2):
            assert L.lib.bcw_decode_segment_async(ctx.handle, C.c_void_p(seg_ptr), C.byref(prm), C.byref(table),
                                                  C.c_void_p(d_res.data_ptr())) == 0
            torch.cuda.synchronize()
            rr = L.DecodeResult.from_buffer_copy(bytes(d_res.cpu().numpy()))
            if not rr.retry_frag_capacity:
                return rr
            assert L.lib.bcw_ctx_reserve_fragments(ctx.handle, rr.retry_frag_capacity + 64) == 0
        raise SystemExit("decode retry failed")

    def encode():
        assert L.lib.bcw_encode_segment_async(ctx.handle, C.c_void_p(d_src.data_ptr()), C.byref(eparams),
                                              C.byref(table), C.c_void_p(d_res.data_ptr()),
                                              C.c_void_p(keep.data_ptr()), C.byref(out),
                                              C.c_void_p(d_eres.data_ptr())) == 0

    decode_checked(d_src.data_ptr(), dparams)
    for _ in range(warmup):
        encode()
    torch.cuda.synchronize()
    res = L.EncodeResult.from_buffer_copy(bytes(d_eres.cpu().numpy()))
    assert res.fits and res.err_class == 0 and res.n_written == n_rec, (res.fits, res.err_class, res.n_written)
    wal_bytes, hint_bytes = int(res.wal_need), int(res.hint_need)
    # full-size parity: dst WAL == source WAL from byte 40
    same = wal_bytes == seg_len - 40 and bool(torch.equal(d_wal[:wal_bytes], d_src[40:]))
    # the hint WAL decodes to (off, size) = (returned offsets, source sizes)
    sb = (C.c_uint8 * 40)()
    L.lib.bcw_write_super_block(sb, BASE_TIME, BASE_TIME)
    himg = torch.empty(40 + hint_bytes, dtype=torch.uint8, device=dev)
    himg[:40] = torch.frombuffer(bytearray(bytes(sb)), dtype=torch.uint8).to(dev)
    himg[40:] = d_hint[:hint_bytes]
    hp = L.DecodeParams(40 + hint_bytes, BASE_TIME, 40, 20, 0, L.MODE_HINT)
    torch.cuda.synchronize()  # the image was assembled on torch's stream, the codec runs on its own
    hres = decode_checked(himg.data_ptr(), hp)
    hint_ok = (hres.err_class == 0 and hres.n_records == n_rec and int(hres.first_bad_record) == -1
               and bool(torch.equal(cols["aux0"][:n_rec], d_off[:n_rec])))
    if not hint_ok:
        a, b = cols["aux0"][:n_rec], d_off[:n_rec]
        bad = torch.nonzero(a != b)
        print("hint check:", hres.err_class, hres.n_records, n_rec, hres.first_bad_record, hres.err_frag,
              "mismatches", bad.numel(), bad[:5].flatten().tolist(),
              [(int(a[i]), int(b[i])) for i in bad[:5].flatten().tolist()], file=sys.stderr)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import _oracle as O  # noqa: E402  (diagnostics only)
        hcpu = himg.cpu().numpy()
        od = O.decode(hcpu, 40, BASE_TIME, 20, 0, 1, want_bytes=False)
        print("oracle hint decode:", od.err_class, len(od.recs), od.err_frag, file=sys.stderr)
        if od.err_class:
            f = od.frags[od.err_frag]
            print("bad frag", f, "block", (int(f["data_off"]) - 40) // 32768, file=sys.stderr)
    del himg
    # the timed loop re-decodes the source first (the encode reads the context's fragment table)
    decode_checked(d_src.data_ptr(), dparams)
    torch.cuda.synchronize()
    nk = int(L.lib.bcw_ctx_kernel_times(ctx.handle, None, None, 0))
    names = [L.lib.bcw_kernel_name(k).decode() for k in range(nk)]
    L.lib.bcw_ctx_set_profiling(ctx.handle, -1)
    L.lib.bcw_ctx_kernel_times(ctx.handle, None, None, nk)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        encode()
    e1.record(stream)
    torch.cuda.synchronize()
    enc_ms = e0.elapsed_time(e1) / steps
    tot = (C.c_double * nk)()
    cnt = (C.c_uint64 * nk)()
    L.lib.bcw_ctx_kernel_times(ctx.handle, tot, cnt, nk)
    kern = {names[k]: round(tot[k] / cnt[k], 4) for k in range(nk) if cnt[k]}
    # decode + encode (a whole compactOneWal of the segment)
    L.lib.bcw_ctx_set_profiling(ctx.handle, 0)
    e0.record(stream)
    for _ in range(steps):
        decode()
        encode()
    e1.record(stream)
    torch.cuda.synchronize()
    both_ms = e0.elapsed_time(e1) / steps
    alg = seg_len + wal_bytes + hint_bytes  # source read once + both outputs written
    pack_ms = kern.get("k_write", 0)
    line = {
        "metric": "compaction re-encode GB/s (device-resident, config E)", "value": round(alg / (enc_ms * 1e-3) / 1e9, 1),
        "unit": "GB/s (src read + WAL + hint written)", "records": n_rec, "src_bytes": seg_len, "wal_bytes": wal_bytes,
        "hint_bytes": hint_bytes, "encode_ms": round(enc_ms, 3), "decode_plus_encode_ms": round(both_ms, 3),
        "records_per_s": round(n_rec / (enc_ms * 1e-3)), "kernel_ms": kern,
        "roofline": {"bound": "hbm", "kernel": "k_write",
                     "achieved": round(alg / (pack_ms * 1e-3) / 1e9, 1) if pack_ms else None, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(alg / (pack_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if pack_ms else None},
        "layout_events": {"wal": int(res.wal_events), "hint": int(res.hint_events)},
        "parity": {"wal_equals_source": same, "hint_decodes_to_offsets": hint_ok},
    }
    if with_index:
        line["index"] = index_leg(L, ctx, stream, d_src, dparams, table, d_res, n_rec, steps, decode_checked,
                                  encode, keep)
    if realistic:
        line["realistic"] = realistic_leg(L, ctx, stream, d_src, seg_len, n_rec, dparams, table, cols, d_res, d_eres,
                                          keep, d_wal, d_hint, d_off, wal_cap, hint_cap, steps, warmup, decode_checked)
    ctx.close()
    return line


def realistic_leg(L, ctx, stream, d_src, seg_len, n_rec, dparams, table, cols, d_res, d_eres, keep, d_wal, d_hint,
                  d_off, wal_cap, hint_cap, steps, warmup, decode_checked):
    """the realistic compaction of the same source: a seeded 70 % keep mask (the index's doFilter
    verdicts, compaction.go:303) and a dst baseTime 500,000 s below the source's (compaction.go:25-29), so the dst
    layout is shifted against the source's and the records split across dst blocks are others than the source's
    (their piece CRCs hashed, bcw_encode.hip k_wcopy). Timed like the identity encode. Parity here is
    self-consistency (the full-size oracle comparison of exactly this shape is tests/test_gpu_fullsize.py
    test_config_e_full_size_realistic_chunks): the dst WAL decodes on the device to the kept rows with no error, its
    record sizes equal the kept source rows', and the hint WAL decodes to the returned offsets of the kept rows.
    split_records: dst records written in two or more fragments."""
    import torch
    dev = d_src.device
    dst_base = BASE_TIME - 500_000
    rng = np.random.default_rng(7)
    km = rng.random(n_rec) < 0.7
    keep.zero_()
    keep[:n_rec] = torch.from_numpy(km.astype(np.uint8)).to(dev)
    kept = int(km.sum())
    eparams = L.EncodeParams(seg_len, dst_base, 1, 40, 40, 40, L.ENC_COMPACT, 20, 20)
    out = L.EncodeOut(C.cast(C.c_void_p(d_wal.data_ptr()), L.u8p), wal_cap,
                      C.cast(C.c_void_p(d_hint.data_ptr()), L.u8p), hint_cap,
                      C.cast(C.c_void_p(d_off.data_ptr()), L.u64p))

    def encode():
        assert L.lib.bcw_encode_segment_async(ctx.handle, C.c_void_p(d_src.data_ptr()), C.byref(eparams),
                                              C.byref(table), C.c_void_p(d_res.data_ptr()),
                                              C.c_void_p(keep.data_ptr()), C.byref(out),
                                              C.c_void_p(d_eres.data_ptr())) == 0

    decode_checked(d_src.data_ptr(), dparams)
    src_size = cols["size"][:n_rec].clone()
    for _ in range(max(warmup, 1)):
        encode()
    torch.cuda.synchronize()
    res = L.EncodeResult.from_buffer_copy(bytes(d_eres.cpu().numpy()))
    assert res.fits and res.err_class == 0 and res.n_written == kept, (res.fits, res.err_class, res.n_written, kept)
    wal_bytes, hint_bytes = int(res.wal_need), int(res.hint_need)
    L.lib.bcw_ctx_set_profiling(ctx.handle, -1)
    nk = int(L.lib.bcw_ctx_kernel_times(ctx.handle, None, None, 0))
    names = [L.lib.bcw_kernel_name(k).decode() for k in range(nk)]
    L.lib.bcw_ctx_kernel_times(ctx.handle, None, None, nk)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        encode()
    e1.record(stream)
    torch.cuda.synchronize()
    enc_ms = e0.elapsed_time(e1) / steps
    tot = (C.c_double * nk)()
    cnt = (C.c_uint64 * nk)()
    L.lib.bcw_ctx_kernel_times(ctx.handle, tot, cnt, nk)
    L.lib.bcw_ctx_set_profiling(ctx.handle, 0)
    kern = {names[k]: round(tot[k] / cnt[k], 4) for k in range(nk) if cnt[k]}
    kept_rows = torch.from_numpy(np.nonzero(km)[0]).to(dev)
    offs_kept = d_off[kept_rows].clone()
    size_kept = src_size[kept_rows]
    # the dst WAL decodes to the kept rows: their count, no error, the kept sources' sizes; split records counted
    sb = (C.c_uint8 * 40)()
    L.lib.bcw_write_super_block(sb, dst_base, dst_base)
    img = torch.empty(40 + wal_bytes, dtype=torch.uint8, device=dev)
    img[:40] = torch.frombuffer(bytearray(bytes(sb)), dtype=torch.uint8).to(dev)
    img[40:] = d_wal[:wal_bytes]
    torch.cuda.synchronize()
    dres = decode_checked(img.data_ptr(), L.DecodeParams(40 + wal_bytes, dst_base, 40, 20, 20, L.MODE_RECORD))
    wal_ok = (dres.err_class == 0 and dres.n_records == kept and int(dres.first_bad_record) == -1
              and bool(torch.equal(cols["size"][:kept], size_kept)))
    split = int((cols["first_frag"][:kept] != cols["emit_frag"][:kept]).sum().item())
    del img
    himg = torch.empty(40 + hint_bytes, dtype=torch.uint8, device=dev)
    himg[:40] = torch.frombuffer(bytearray(bytes(sb)), dtype=torch.uint8).to(dev)
    himg[40:] = d_hint[:hint_bytes]
    torch.cuda.synchronize()
    hres = decode_checked(himg.data_ptr(), L.DecodeParams(40 + hint_bytes, dst_base, 40, 20, 0, L.MODE_HINT))
    hint_ok = (hres.err_class == 0 and hres.n_records == kept and int(hres.first_bad_record) == -1
               and bool(torch.equal(cols["aux0"][:kept], offs_kept)))
    del himg
    keep.fill_(1)  # (the identity encode's mask, for any later user)
    alg = seg_len + wal_bytes + hint_bytes
    wr = kern.get("k_write")
    return {"encode_ms": round(enc_ms, 3), "records_in": n_rec, "records_kept": kept, "split_records": split,
            "wal_bytes": wal_bytes, "hint_bytes": hint_bytes, "dst_base_time": dst_base,
            "GBs": round(alg / (enc_ms * 1e-3) / 1e9, 1),
            "writer_TBs": round(alg / (wr * 1e-3) / 1e12, 3) if wr else None, "kernel_ms": kern,
            "layout_events": {"wal": int(res.wal_events), "hint": int(res.hint_events)},
            "parity": {"dst_decodes_to_kept_rows": wal_ok, "hint_decodes_to_offsets": hint_ok}}


if __name__ == "__main__":
    main()
