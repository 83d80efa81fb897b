#!/usr/bin/env python3
"""WAL record decode+CRC throughput (device-resident) on 1..8 MI355X, one process per GPU.

Workload (BASELINE.json configs[1], "B"): a synthetic 1 GiB bitcaskDB WAL segment, NsSize 20,
100 B keys / 4 KiB values, no etag/expire/meta, built by the product's host writer
(bcw_synth_segment) and copied to HBM before timing. One "step" = one full decode of the
segment through the C-ABI (bcw_decode_segment_async): header chase, CRC-32C verify of every
fragment, record assembly and RecordFromBytes for every record into the device record table.
An extra `pipelined` key times the same K steps rotating over --inflight (default 2) independent
segments, each with its own context (stream, scratch, record table), as a scan over many WAL files
runs: one segment's latency-bound kernels overlap the next one's CRC pass.
Multi-GPU = config D: every rank decodes its own independent segment (seed 42 + rank) with no
collective on the data path ("scaling": "weak"); the barrier + max-over-ranks timing follows the
driver contract. Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "WAL record decode+CRC GiB/s (device-resident), 4 KiB values, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
BASE_TIME = 1_700_000_000


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # untimed steps right before the timed ones (the driver's own value). After an idle period the chip lowers its
    # shader clock under this load over the first ~10-60 back-to-back decodes (in-kernel clock 2.1 -> 1.3-1.5 GHz and
    # back, profiles/r05_clock): with 5 warmup steps the timed ones sit in that dip, as a one-file
    # compaction scan does
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--seg-bytes", type=int, default=1 << 30)
    ap.add_argument("--config", default="B", choices=["B", "C"], help="B: 4 KiB values; C: Zipf 128 B-64 KiB")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the extra legs (config C, all-core / pread CPU baselines, file-to-file end-to-end rates)")
    ap.add_argument("--encode-records", type=int, default=10_000_000,
                    help="records of the extra encode_e leg (BASELINE.json configs[4], config E: 10 M); 0 skips it")
    ap.add_argument("--cpu-threads", type=int, default=16, help="threads of the all-core CPU baseline")
    ap.add_argument("--inflight", type=int, default=2,
                    help="segments in flight for the extra pipelined leg: steps rotate over this many contexts "
                         "(own stream, segment, record table); the headline value is one segment at a time")
    ap.add_argument("--event-every", type=int, default=4,
                    help="HIP events bracket every N-th k_crc launch of the timed region")
    ap.add_argument("--launcher-selftest", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r06", "k_crc_pmc.json"),
                    help="PMC traffic summary (tools/pmc_summary.py over rocprofv3 --pmc passes of this command) to "
                         "report as roofline.traffic; used only when its decode_src_sha16 matches this build's "
                         "decode sources (bitcaskdb_amd/build.py decode_src_sha16)")
    return ap.parse_args()


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_all_cores(O, hb, n_rec, seconds, threads):
    """the restated decode loop on `threads` host threads at once, each over the same segment (ctypes releases
    the GIL inside the C call); returns (GiB/s, passes, seconds)"""
    import threading
    seg_len = int(hb.size)
    counts = [0] * threads
    t0 = time.perf_counter()
    stop = t0 + seconds

    def run(i):
        while time.perf_counter() < stop:
            got, ec, _ = O.decode_fast(hb, 40, BASE_TIME, 20, 20)
            assert got == n_rec and ec == 0
            counts[i] += 1

    th = [threading.Thread(target=run, args=(i,)) for i in range(threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    return seg_len * sum(counts) / 2 ** 30 / dt, sum(counts), dt


def cpu_pread_config_a(O, L, seconds):
    """config A: a 64 MiB 4 KiB-value segment on disk (page cache), decoded with a pread per 32 KiB block as
    the reference iterator does (wal_iterator.go:55 -> utils.go:32-48), 1 thread"""
    import tempfile
    n, r = C.c_uint64(), C.c_uint64()
    assert L.lib.bcw_synth_segment(64 << 20, 0, 7, 20, 100, 4096, 0, BASE_TIME, None, 0, C.byref(n), C.byref(r)) == 0
    buf = np.zeros(n.value, dtype=np.uint8)
    assert L.lib.bcw_synth_segment(64 << 20, 0, 7, 20, 100, 4096, 0, BASE_TIME, C.c_void_p(buf.ctypes.data),
                                   n.value, C.byref(n), C.byref(r)) == 0
    with tempfile.NamedTemporaryFile(dir="/tmp", suffix=".wal") as fh:
        fh.write(buf.tobytes())
        fh.flush()
        fd = os.open(fh.name, os.O_RDONLY)
        try:
            passes, t = 0, time.perf_counter()
            while True:
                got, ec, _ = O.decode_fast_pread(fd, int(n.value), 40, BASE_TIME, 20, 20)
                assert got == r.value and ec == 0
                passes += 1
                if time.perf_counter() - t >= seconds:
                    break
            dt = time.perf_counter() - t
        finally:
            os.close(fd)
    return int(n.value) * passes / 2 ** 30 / dt, passes, dt, int(n.value)


def _fs_of(path: str) -> str:
    """filesystem type and device of the mount holding `path` (/proc/mounts: the longest matching mount point)"""
    best, out = "", "unknown"
    try:
        with open("/proc/mounts") as fh:
            for ln in fh:
                dev, mnt, fs = ln.split()[:3]
                if path.startswith(mnt) and len(mnt) > len(best):
                    best, out = mnt, f"{fs} ({dev} on {mnt})"
    except OSError:
        pass
    return out


def end_to_end(L, ctx, stream, host, d_seg, step, table, d_res, seg_len, n_rec, reps=3):
    """file -> pinned slices -> HBM -> decode, and file -> decode -> re-encode (all kept) -> dst WAL + hint
    files, through bcw_stage (f3); the files sit in the page cache (written just before)"""
    import tempfile
    import torch
    from bitcaskdb_amd import Stage
    dev = d_seg.device
    st = Stage(ctx, 8 << 20, 16)
    cap = table.capacity
    keep = torch.ones(cap, dtype=torch.uint8, device=dev)
    d_wal = torch.empty(seg_len + (seg_len >> 6) + (1 << 20), dtype=torch.uint8, device=dev)
    d_hint = torch.empty(n_rec * 200 + (1 << 20), dtype=torch.uint8, device=dev)
    e_res = torch.zeros(C.sizeof(L.EncodeResult), dtype=torch.uint8, device=dev)
    ep = L.EncodeParams(seg_len, BASE_TIME, 2, 40, 40, 40, L.ENC_COMPACT, 20, 20)
    out = L.EncodeOut(C.cast(C.c_void_p(d_wal.data_ptr()), L.u8p), d_wal.numel(),
                      C.cast(C.c_void_p(d_hint.data_ptr()), L.u8p), d_hint.numel(), None, 0)
    res = {}
    with tempfile.TemporaryDirectory(dir="/tmp") as tmp:
        src = os.path.join(tmp, "1.wal")
        host.numpy().tofile(src)
        fd = os.open(src, os.O_RDONLY)
        try:
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(reps):
                st.read(fd, 0, seg_len, d_seg.data_ptr(), stream.cuda_stream, threads=8)
                step()
                torch.cuda.synchronize()
            res["decode_file_GiBs"] = round(seg_len / 2 ** 30 / ((time.perf_counter() - t) / reps), 2)
            # from the storage device: the file's pages written back and dropped from the page cache before every
            # read (posix_fadvise DONTNEED), and through an O_DIRECT descriptor (no page cache at all)
            os.fsync(fd)
            t_cold = 0.0
            for _ in range(reps):
                os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
                torch.cuda.synchronize()
                t = time.perf_counter()
                st.read(fd, 0, seg_len, d_seg.data_ptr(), stream.cuda_stream, threads=8)
                step()
                torch.cuda.synchronize()
                t_cold += time.perf_counter() - t
            res["decode_file_cold_GiBs"] = round(seg_len / 2 ** 30 / (t_cold / reps), 2)
            try:
                dfd = os.open(src, os.O_RDONLY | os.O_DIRECT)
            except OSError as e:
                res["decode_file_odirect_GiBs"] = f"O_DIRECT open refused: {e.strerror}"
            else:
                try:
                    torch.cuda.synchronize()
                    t = time.perf_counter()
                    for _ in range(reps):
                        st.read(dfd, 0, seg_len, d_seg.data_ptr(), stream.cuda_stream, threads=8)
                        step()
                        torch.cuda.synchronize()
                    res["decode_file_odirect_GiBs"] = round(seg_len / 2 ** 30 / ((time.perf_counter() - t) / reps), 2)
                except OSError as e:
                    res["decode_file_odirect_GiBs"] = f"O_DIRECT read failed: {e}"
                finally:
                    os.close(dfd)
            res["tmp_fs"] = _fs_of(tmp)
            t = time.perf_counter()
            for i in range(reps):
                st.read(fd, 0, seg_len, d_seg.data_ptr(), stream.cuda_stream, threads=8)
                step()
                rc = L.lib.bcw_encode_segment_async(ctx.handle, C.c_void_p(d_seg.data_ptr()), C.byref(ep),
                                                    C.byref(table), C.c_void_p(d_res.data_ptr()),
                                                    C.c_void_p(keep.data_ptr()), C.byref(out),
                                                    C.c_void_p(e_res.data_ptr()))
                assert rc == 0
                stream.synchronize()
                r = L.EncodeResult.from_buffer_copy(bytes(e_res.cpu().numpy()))
                assert r.err_class == 0 and r.fits and r.n_written == n_rec
                for name, dbuf, nb in (("2.merge", d_wal, r.wal_need), ("2.tmp", d_hint, r.hint_need)):
                    ofd = os.open(os.path.join(tmp, f"{i}.{name}"), os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
                    try:
                        st.write(ofd, 40, dbuf.data_ptr(), int(nb), stream.cuda_stream, threads=8)
                    finally:
                        os.close(ofd)
            res["compaction_file_to_file_GiBs"] = round(seg_len / 2 ** 30 / ((time.perf_counter() - t) / reps), 2)
        finally:
            os.close(fd)
    st.close()
    res["note"] = ("decode_file / compaction: source and output files in the page cache; decode_file_cold: the source "
                   "written back and dropped from the page cache (posix_fadvise DONTNEED) before every read; "
                   "decode_file_odirect: read through an O_DIRECT descriptor; 16 pinned 8 MiB slices, 8 pread / pwrite "
                   "threads; compaction = read + decode + re-encode + hint rebuild + dst WAL and hint written back")
    return res


def config_c_leg(L, Context, torch, dev, args, make_table, roof_name, kernel_names):
    """BASELINE.json configs[2] (C): a 1 GiB segment of Zipf(1.1) 128 B-64 KiB values, decoded exactly like the
    headline (W untimed steps, then K timed, HIP events around every --event-every-th k_crc); an extra key, never
    `value`"""
    n, r = C.c_uint64(), C.c_uint64()
    assert L.lib.bcw_synth_segment(args.seg_bytes, 0, 42, 20, 100, 4096, 1, BASE_TIME, None, 0, C.byref(n),
                                   C.byref(r)) == 0
    host = torch.empty(n.value, dtype=torch.uint8).pin_memory()
    assert L.lib.bcw_synth_segment(args.seg_bytes, 0, 42, 20, 100, 4096, 1, BASE_TIME, C.c_void_p(host.data_ptr()),
                                   n.value, C.byref(n), C.byref(r)) == 0
    seg_len, n_rec = int(n.value), int(r.value)
    d_seg = host.to(dev)
    del host
    table, cols = make_table(n_rec + 64)
    d_res = torch.zeros(C.sizeof(L.DecodeResult), dtype=torch.uint8, device=dev)
    params = L.DecodeParams(seg_len, BASE_TIME, 40, 20, 20, L.MODE_RECORD)
    ctx = Context(torch.cuda.current_device())
    stream = torch.cuda.Stream()
    ctx.set_stream(stream.cuda_stream)

    def step():
        assert L.lib.bcw_decode_segment_async(ctx.handle, C.c_void_p(d_seg.data_ptr()), C.byref(params),
                                              C.byref(table), C.c_void_p(d_res.data_ptr())) == 0
    step()
    torch.cuda.synchronize()
    res = L.DecodeResult.from_buffer_copy(bytes(d_res.cpu().numpy()))
    assert res.err_class == 0 and res.n_records == n_rec and res.first_bad_record == -1, "config C decode check"
    n_frags = int(res.n_frags)
    roof_k = kernel_names.index(roof_name)
    for _ in range(args.warmup):
        step()
    L.lib.bcw_ctx_set_profiling(ctx.handle, 1 << roof_k)
    L.lib.bcw_ctx_set_profiling_sample(ctx.handle, args.event_every)
    nk = len(kernel_names)
    L.lib.bcw_ctx_kernel_times(ctx.handle, None, None, nk)  # reset
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    tot = (C.c_double * nk)()
    cnt = (C.c_uint64 * nk)()
    L.lib.bcw_ctx_kernel_times(ctx.handle, tot, cnt, nk)
    L.lib.bcw_ctx_set_profiling(ctx.handle, 0)
    crc_ms = tot[roof_k] / max(1, cnt[roof_k])
    alg = seg_len + 17 * n_frags + 48 * n_rec
    ctx.close()
    return {"value": round(seg_len * args.steps / 2 ** 30 / wall, 2), "unit": "GiB/s",
            "ms_per_step": round(wall / args.steps * 1e3, 4), "steps": args.steps, "warmup": args.warmup,
            "seg_bytes": seg_len, "records": n_rec, "fragments": n_frags,
            "k_crc_ms": round(crc_ms, 4), "k_crc_frac": round(alg / (crc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "note": "configs[2]: Zipf(s=1.1) values 128 B-64 KiB (numpy default_rng(42) semantics), same "
                    "warmup/steps as the headline, measured after it in the same process"}


def encode_e_leg(args):
    """BASELINE.json configs[4] (E): the compaction re-encode (compactOneWal: Record.Encode + WriteRecord + hint
    append, every record kept) of --encode-records records of the config-E shape, device-resident; the same warmup
    and steps as the headline, timed with HIP events on the codec's stream (tools/bench_encode.py measure); an
    extra key, never `value`. Its parity: the dst WAL equals the source from byte 40 and the hint decodes back to the
    returned offsets."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_encode  # noqa: E402
    m = bench_encode.measure(args.encode_records, args.steps, args.warmup, realistic=True)
    alg = m["src_bytes"] + m["wal_bytes"] + m["hint_bytes"]
    wr = m["kernel_ms"].get("k_write")
    return {"value": m["value"], "unit": m["unit"], "encode_ms": m["encode_ms"], "records": m["records"],
            "src_bytes": m["src_bytes"], "steps": args.steps, "warmup": args.warmup,
            "decode_plus_encode_ms": m["decode_plus_encode_ms"], "kernel_ms": m["kernel_ms"],
            "writer_TBs": round(alg / (wr * 1e-3) / 1e12, 3) if wr else None, "parity": m["parity"],
            "realistic": m["realistic"],
            "note": "writer_TBs: algorithmic bytes (src read + dst WAL + hint written) / the writer phase (k_wcopy + "
                    "k_write + k_write_general + k_hwrite, one profiling slot named k_write); realistic: the same "
                    "source with a seeded 70 % keep mask and a dst baseTime 500,000 s lower (tools/bench_encode.py "
                    "realistic_leg)"}


def main():
    args = parse()
    from bitcaskdb_amd import shard
    # --gpus N without a launcher: start the N rank processes here (before anything touches a GPU) and exit with
    # their status; under torch.distributed.run WORLD_SIZE must equal N
    try:
        plans = shard.launch_plan(args.gpus, os.environ)
    except ValueError as e:
        raise SystemExit(f"bench.py: {e}")
    if plans is not None:
        sys.exit(shard.spawn_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], plans))
    if args.launcher_selftest:  # CPU test of the launcher: report the rank environment, touch no GPU
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")}),
              flush=True)
        return
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    share = world > ndev  # more ranks than GPUs (the 1-GPU box's two-rank test): RCCL needs one GPU per rank
    torch.cuda.set_device(shard.rank_device(local, ndev))
    if world > 1:
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
    dev = torch.device("cuda", torch.cuda.current_device())
    red_dev = None if share else dev  # max-over-ranks tensor: host memory under gloo

    from bitcaskdb_amd import _lib as L
    from bitcaskdb_amd import Context

    # ---- this rank's segments: built on the host with the product writer, then copied to HBM ----
    # A scan over many WAL files (recovery, compaction of every wal, config D) keeps `inflight` segments in
    # flight on independent contexts, so one segment's latency-bound header chase / record emission and the
    # kernel boundaries overlap another segment's CRC pass. Every step is still one complete decode of one
    # whole segment; the steps rotate over the contexts.
    vmode = 0 if args.config == "B" else 1
    nslot = max(1, args.inflight)

    def build_segment(seed):
        n, r = C.c_uint64(), C.c_uint64()
        rc = L.lib.bcw_synth_segment(args.seg_bytes, 0, seed, 20, 100, 4096, vmode, BASE_TIME, None, 0, C.byref(n),
                                     C.byref(r))
        assert rc == 0
        host = torch.empty(n.value, dtype=torch.uint8).pin_memory()
        rc = L.lib.bcw_synth_segment(args.seg_bytes, 0, seed, 20, 100, 4096, vmode, BASE_TIME,
                                     C.c_void_p(host.data_ptr()), n.value, C.byref(n), C.byref(r))
        assert rc == 0
        return host, int(n.value), int(r.value)

    ptr_t = {"u8": L.u64p, "u4": L.u32p, "u1": L.u8p}

    def make_table(cap):
        # a record-mode table: aux0 / aux1 are hint-mode columns and stay NULL (bcw.h), as a record-mode caller passes them
        cols = {}
        for name, dt in L.TABLE_COLUMNS:
            if name in ("aux0", "aux1"):
                continue
            tdt = {"u8": torch.int64, "u4": torch.int32, "u1": torch.uint8}[dt]
            cols[name] = torch.empty(cap, dtype=tdt, device=dev)
        return L.RecordTable(cap, *[C.cast(C.c_void_p(cols[name].data_ptr()), ptr_t[dt]) if name in cols else None
                                    for name, dt in L.TABLE_COLUMNS]), cols
    slots = []
    for j in range(nslot):
        host, seg_len, n_rec = build_segment(shard.segment_seed(42 + 1000 * j, rank))
        d_seg = host.to(dev, non_blocking=True)
        # ---- device record table + result ----
        table, cols = make_table(n_rec + 64)
        d_res = torch.zeros(C.sizeof(L.DecodeResult), dtype=torch.uint8, device=dev)
        params = L.DecodeParams(seg_len, BASE_TIME, 40, 20, 20, L.MODE_RECORD)
        sctx = Context(torch.cuda.current_device())
        sstream = torch.cuda.Stream()  # dedicated stream: the codec's kernels and the timing events share it
        sctx.set_stream(sstream.cuda_stream)
        slots.append(dict(host=host, seg_len=seg_len, n_rec=n_rec, d_seg=d_seg, cols=cols, table=table, d_res=d_res,
                          params=params, ctx=sctx, stream=sstream))
        if j == 0:
            del host  # slot 0's host copy is kept in its slot (end-to-end and CPU legs)
    torch.cuda.synchronize()
    s0 = slots[0]
    host, seg_len, n_rec, d_seg = s0["host"], s0["seg_len"], s0["n_rec"], s0["d_seg"]
    table, d_res, ctx, stream = s0["table"], s0["d_res"], s0["ctx"], s0["stream"]

    def decode(sl):
        rc = L.lib.bcw_decode_segment_async(sl["ctx"].handle, C.c_void_p(sl["d_seg"].data_ptr()),
                                            C.byref(sl["params"]), C.byref(sl["table"]),
                                            C.c_void_p(sl["d_res"].data_ptr()))
        if rc != 0:
            raise RuntimeError(L.lib.bcw_strerror(rc).decode())

    def step():  # slot 0 alone (end-to-end legs)
        decode(s0)

    rot = [0]

    def step_rot():
        decode(slots[rot[0] % nslot])
        rot[0] += 1

    # ---- correctness gate (not timed): one decode of every in-flight segment, checked ----
    for sl in slots:
        decode(sl)
    torch.cuda.synchronize()
    n_frags = 0
    for j, sl in enumerate(slots):
        res = L.DecodeResult.from_buffer_copy(bytes(sl["d_res"].cpu().numpy()))
        nr, cols = sl["n_rec"], sl["cols"]
        ok = (res.err_class == 0 and res.n_records == nr and res.first_bad_record == -1
              and int((cols["status"][:nr] != 0).sum().item()) == 0
              and int((cols["size"][:nr] <= 0).sum().item()) == 0)
        if not ok:
            raise SystemExit(f"rank {rank} slot {j}: decode check failed: err={res.err_class} n={res.n_records}/{nr} "
                             f"bad={res.first_bad_record}")
        if j == 0:
            n_frags = int(res.n_frags)

    # kernel ids by name (the pipeline's kernel list is the library's)
    nk = int(L.lib.bcw_ctx_kernel_times(ctx.handle, None, None, 0))
    names = [L.lib.bcw_kernel_name(k).decode() for k in range(nk)]
    # the dominant kernel: k_crc (the CRC stream + record emission)
    roof_name = "k_crc"
    roof_k = names.index(roof_name)

    def kernel_times(ctxs):
        """per-kernel average over the given contexts (reading resets their accumulators)"""
        agg_t, agg_c = [0.0] * nk, [0] * nk
        for cx in ctxs:
            tot = (C.c_double * nk)()
            cnt = (C.c_uint64 * nk)()
            L.lib.bcw_ctx_kernel_times(cx.handle, tot, cnt, nk)
            for k in range(nk):
                agg_t[k] += tot[k]
                agg_c[k] += cnt[k]
        return {names[k]: (agg_t[k] / agg_c[k], agg_c[k]) for k in range(nk) if agg_c[k]}

    all_ctx = [sl["ctx"] for sl in slots]
    # ---- timed region: K steps, barrier + synchronize on both sides, max over ranks ----
    # HIP events bracket only the roofline kernel (k_crc) on each codec stream
    # (every --event-every-th launch: an event pair idles that stream for a few microseconds)
    # ---- warmup: W untimed steps back to back, right before the timed ones ----
    for _ in range(args.warmup):
        step()
    for cx in all_ctx:
        L.lib.bcw_ctx_set_profiling(cx.handle, 1 << roof_k)
        L.lib.bcw_ctx_set_profiling_sample(cx.handle, args.event_every)
    kernel_times(all_ctx)  # reset (synchronises the codec streams)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    wall = shard.timed_steps(step, args.steps, 0, torch.cuda.synchronize, dist.barrier if world > 1 else None)
    ev1.record(stream)
    torch.cuda.synchronize()
    ev_ms = ev0.elapsed_time(ev1)
    crc_ms, crc_samples = kernel_times(all_ctx)[roof_name]
    bytes_total = seg_len * args.steps
    # pipelined: the same K steps rotating over the in-flight segments (an extra key, never `value`: with two
    # streams a k_crc event pair also spans the other segment's kernels)
    pipelined = None
    if nslot > 1:
        for cx in all_ctx:
            L.lib.bcw_ctx_set_profiling(cx.handle, 0)
        wall_p = shard.timed_steps(step_rot, args.steps, 0, torch.cuda.synchronize,
                                   dist.barrier if world > 1 else None)
        wall_p = shard.max_over_ranks(wall_p, dist, red_dev)
        bytes_p = sum(slots[i % nslot]["seg_len"] for i in range(args.steps))
        pipelined = {"inflight": nslot, "value": round(shard.aggregate_gib_s([bytes_p / args.steps] * world, wall_p,
                                                                               args.steps), 2),
                     "unit": "GiB/s", "ms_per_step": round(wall_p / args.steps * 1e3, 4),
                     "note": "steps rotate over independent segments on their own contexts/streams (a multi-file "
                             "scan): one segment's k_chase and the kernel boundaries overlap the next one's k_crc"}
    # every kernel's average, one segment at a time (untimed repeat, events around each kernel)
    L.lib.bcw_ctx_set_profiling_sample(ctx.handle, 1)
    L.lib.bcw_ctx_set_profiling(ctx.handle, -1)
    for _ in range(min(args.steps, 10)):
        step()
    kern = {k: v[0] for k, v in kernel_times([ctx]).items()}
    for cx in all_ctx:
        L.lib.bcw_ctx_set_profiling(cx.handle, 0)

    wall_max = shard.max_over_ranks(wall, dist, red_dev)
    ms_per_step = wall_max / args.steps * 1e3
    # whole job: this rank's bytes per step (segments of equal size on every rank, to a record) x ranks
    value = shard.aggregate_gib_s([bytes_total / args.steps] * world, wall_max, args.steps)

    # end-to-end PCIe-inclusive rate (pinned H2D of the segment + decode), rank 0 only, not `value`
    pcie = None
    if rank == 0:
        torch.cuda.synchronize()
        t = time.perf_counter()
        reps = 3
        with torch.cuda.stream(stream):
            for _ in range(reps):
                d_seg.copy_(host, non_blocking=True)
                step()
        torch.cuda.synchronize()
        pcie = seg_len / 2 ** 30 / ((time.perf_counter() - t) / reps)

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    # ---- roofline of the dominant kernel (k_crc): algorithmic bytes per launch / avg duration ----
    # segment read once + per fragment its descriptor (16 B read) and verdict (1 B written) + per record its row of
    # the record table (48 B written: k_crc emits the records)
    alg_bytes = seg_len + 17 * n_frags + 48 * n_rec
    achieved = alg_bytes / (crc_ms * 1e-3) / 1e9
    # traffic: HBM bytes per launch from a committed PMC summary measured on THIS build's k_crc (same decode-source
    # hash, same segment), else null
    traffic, traffic_src = None, None
    if args.pmc and os.path.exists(args.pmc):
        from bitcaskdb_amd.build import decode_src_sha16
        try:
            pm = json.load(open(args.pmc))
            if (pm.get("seg_bytes") == seg_len and pm.get("kernel") == roof_name
                    and pm.get("decode_src_sha16") == decode_src_sha16()):
                traffic = pm.get("hbm_bytes_per_launch")
                traffic_src = os.path.relpath(args.pmc, ROOT)
        except Exception:
            traffic = None
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_src": traffic_src,
                "kernel": roof_name,
                "kernel_ms": round(crc_ms, 4), "kernel_launches_timed": crc_samples, "alg_bytes": alg_bytes,
                "pipeline_GBs": round(bytes_total / args.steps / (ms_per_step * 1e-3) / 1e9, 1),
                "kernel_ms_all": {k: round(v, 4) for k, v in kern.items()}}

    # ---- config C and end-to-end through the host I/O staging (rank 0, N=1) ----
    extras = {}
    if world == 1 and not args.no_extras and args.config == "B":
        extras["config_c"] = config_c_leg(L, Context, torch, dev, args, make_table, roof_name, names)
    if world == 1 and not args.no_extras and args.config == "B" and args.encode_records > 0:
        extras["encode_e"] = encode_e_leg(args)
    if world == 1 and not args.no_extras:
        extras["e2e"] = end_to_end(L, ctx, stream, host, d_seg, step, table, d_res, seg_len, n_rec)

    # ---- CPU baseline: restated reference decode loop (oracle/, hardware CRC, 1 thread) ----
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import _oracle as O  # noqa: E402  (cpu_baseline leg only)
        hb = host.numpy()
        passes, t = 0, time.perf_counter()
        while True:
            got, ec, _ = O.decode_fast(hb, 40, BASE_TIME, 20, 20)
            assert got == n_rec and ec == 0
            passes += 1
            if time.perf_counter() - t >= args.cpu_seconds:
                break
        dt = time.perf_counter() - t
        model = cpu_model()
        cpu = {"value": round(seg_len * passes / 2 ** 30 / dt, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
               "sample": f"{passes} full decode passes over the same {seg_len} B config-{args.config} segment "
                         f"(host copy), restated wal_iterator.go Next + RecordFromBytes with SSE4.2 CRC, 1 thread, "
                         f"{dt:.1f} s, {model}"}
        if not args.no_extras:
            thr = max(1, min(args.cpu_threads, os.cpu_count() or 1))
            v, p, d = cpu_all_cores(O, hb, n_rec, args.cpu_seconds, thr)
            extras["cpu_all_cores"] = {"value": round(v, 3), "unit": "GiB/s", "cores": thr, "kind": "port",
                                       "sample": f"{p} passes over the config-{args.config} segment on {thr} "
                                                 f"threads in {d:.1f} s, {model}"}
            v, p, d, a_len = cpu_pread_config_a(O, L, min(args.cpu_seconds, 5.0))
            extras["cpu_config_a_pread"] = {"value": round(v, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
                                            "sample": f"config A: {p} passes over a {a_len} B segment file (page "
                                                      f"cache), one pread per 32 KiB block, {d:.1f} s, {model}"}

    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"config {args.config}: {seg_len} B WAL segment per GPU, NsSize 20, 100 B keys, "
                               + ("4 KiB values" if args.config == "B" else "Zipf(1.1) 128 B-64 KiB values")
                               + ", device-resident decode+CRC+record parse",
                   "seg_bytes": seg_len, "records": n_rec, "fragments": n_frags,
                   "parallelism": f"one independent segment per GPU x{world}" + (" (ranks sharing GPUs)" if share else ""),
                   },
        "roofline": roofline, "cpu_baseline": cpu,
        "pcie_inclusive_GiBs": round(pcie, 2) if pcie else None,
        "event_ms_per_step": round(ev_ms / args.steps, 4),
    }
    if pipelined:
        line["pipelined"] = pipelined
    line.update(extras)
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
