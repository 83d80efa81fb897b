#!/usr/bin/env python3
"""WAL record decode+CRC throughput (device-resident) on 1..8 MI355X, one process per GPU.

Workload (BASELINE.json configs[1], "B"): a synthetic 1 GiB bitcaskDB WAL segment, NsSize 20,
100 B keys / 4 KiB values, no etag/expire/meta, built by the product's host writer
(bcw_synth_segment) and copied to HBM before timing. One "step" = one full decode of the
segment through the C-ABI (bcw_decode_segment_async): header chase, CRC-32C verify of every
fragment, record assembly and RecordFromBytes for every record into the device record table.
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
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--seg-bytes", type=int, default=1 << 30)
    ap.add_argument("--config", default="B", choices=["B", "C"], help="B: 4 KiB values; C: Zipf 128 B-64 KiB")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--event-every", type=int, default=4,
                    help="HIP events bracket every N-th k_crc launch of the timed region")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r01_k_crc_pmc.json"),
                    help="PMC traffic summary (rocprofv3 --pmc of this command) to report as roofline.traffic")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from bitcaskdb_amd import _lib as L
    from bitcaskdb_amd import Context
    from bitcaskdb_amd import shard

    # ---- build this rank's segment on the host with the product writer, then copy to HBM ----
    seed = shard.segment_seed(42, rank)
    vmode = 0 if args.config == "B" else 1
    n, r = C.c_uint64(), C.c_uint64()
    rc = L.lib.bcw_synth_segment(args.seg_bytes, 0, seed, 20, 100, 4096, vmode, BASE_TIME, None, 0, C.byref(n),
                                 C.byref(r))
    assert rc == 0
    host = torch.empty(n.value, dtype=torch.uint8).pin_memory()
    rc = L.lib.bcw_synth_segment(args.seg_bytes, 0, seed, 20, 100, 4096, vmode, BASE_TIME,
                                 C.c_void_p(host.data_ptr()), n.value, C.byref(n), C.byref(r))
    assert rc == 0
    seg_len, n_rec = int(n.value), int(r.value)
    d_seg = host.to(dev, non_blocking=True)
    torch.cuda.synchronize()

    # ---- device record table + result ----
    cap = n_rec + 64
    cols = {}
    for name, dt in L.TABLE_COLUMNS:
        tdt = {"u8": torch.int64, "u4": torch.int32, "u1": torch.uint8}[dt]
        cols[name] = torch.empty(cap, dtype=tdt, device=dev)
    ptr_t = {"u8": L.u64p, "u4": L.u32p, "u1": L.u8p}
    table = L.RecordTable(cap, *[C.cast(C.c_void_p(cols[name].data_ptr()), ptr_t[dt]) for name, dt in L.TABLE_COLUMNS])
    d_res = torch.zeros(C.sizeof(L.DecodeResult), dtype=torch.uint8, device=dev)
    params = L.DecodeParams(seg_len, BASE_TIME, 40, 20, 20, L.MODE_RECORD)

    ctx = Context(torch.cuda.current_device())
    stream = torch.cuda.Stream()  # dedicated stream: the codec's kernels and the timing events share it
    ctx.set_stream(stream.cuda_stream)

    def step():
        rc = L.lib.bcw_decode_segment_async(ctx.handle, C.c_void_p(d_seg.data_ptr()), C.byref(params),
                                            C.byref(table), C.c_void_p(d_res.data_ptr()))
        if rc != 0:
            raise RuntimeError(L.lib.bcw_strerror(rc).decode())

    # ---- warmup + correctness gate (not timed) ----
    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize()
    res = L.DecodeResult.from_buffer_copy(bytes(d_res.cpu().numpy()))
    ok = (res.err_class == 0 and res.n_records == n_rec and res.first_bad_record == -1
          and int((cols["status"][:n_rec] != 0).sum().item()) == 0
          and int((cols["size"][:n_rec] <= 0).sum().item()) == 0)
    if not ok:
        raise SystemExit(f"rank {rank}: decode check failed: err={res.err_class} n={res.n_records}/{n_rec} "
                         f"bad={res.first_bad_record}")
    n_frags = int(res.n_frags)

    # kernel ids by name (the pipeline's kernel list is the library's)
    nk = int(L.lib.bcw_ctx_kernel_times(ctx.handle, None, None, 0))
    names = [L.lib.bcw_kernel_name(k).decode() for k in range(nk)]
    roof_k = names.index("k_crc")

    def kernel_times():
        tot = (C.c_double * nk)()
        cnt = (C.c_uint64 * nk)()
        L.lib.bcw_ctx_kernel_times(ctx.handle, tot, cnt, nk)
        return {names[k]: (tot[k] / cnt[k]) for k in range(nk) if cnt[k]}

    # ---- timed region: K steps, barrier + synchronize on both sides, max over ranks ----
    # HIP events bracket only the roofline kernel (k_crc) on the codec's stream
    # (every --event-every-th launch: an event pair idles the GPU for a few microseconds)
    L.lib.bcw_ctx_set_profiling(ctx.handle, 1 << roof_k)
    L.lib.bcw_ctx_set_profiling_sample(ctx.handle, args.event_every)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    kernel_times()  # reset (synchronises the codec's stream)
    ev0.record(stream)
    # warmup already ran above (with the correctness gate)
    wall = shard.timed_steps(step, args.steps, 0, torch.cuda.synchronize, dist.barrier if world > 1 else None)
    ev1.record(stream)
    torch.cuda.synchronize()
    ev_ms = ev0.elapsed_time(ev1)
    tot = (C.c_double * nk)()
    cnt = (C.c_uint64 * nk)()
    L.lib.bcw_ctx_kernel_times(ctx.handle, tot, cnt, nk)
    crc_ms, crc_samples = tot[roof_k] / cnt[roof_k], int(cnt[roof_k])
    # every kernel's average (untimed repeat, events around each kernel)
    L.lib.bcw_ctx_set_profiling_sample(ctx.handle, 1)
    L.lib.bcw_ctx_set_profiling(ctx.handle, -1)
    for _ in range(min(args.steps, 10)):
        step()
    kern = kernel_times()
    L.lib.bcw_ctx_set_profiling(ctx.handle, 0)

    wall_max = shard.max_over_ranks(wall, dist, dev)
    ms_per_step = wall_max / args.steps * 1e3
    value = shard.aggregate_gib_s([seg_len] * world, wall_max, args.steps)  # same-size segment per rank

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
    alg_bytes = seg_len + 17 * n_frags  # segment read once + fragment descriptors (16 B read, 1 B verdict)
    achieved = alg_bytes / (crc_ms * 1e-3) / 1e9
    traffic = None
    if args.pmc and os.path.exists(args.pmc):
        try:
            pm = json.load(open(args.pmc))
            if pm.get("seg_bytes") == seg_len:
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": "k_crc",
                "kernel_ms": round(crc_ms, 4), "kernel_launches_timed": crc_samples, "alg_bytes": alg_bytes,
                "pipeline_GBs": round(seg_len / (ms_per_step * 1e-3) / 1e9, 1),
                "kernel_ms_all": {k: round(v, 4) for k, v in kern.items()}}

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
        cpu = {"value": round(seg_len * passes / 2 ** 30 / dt, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
               "sample": f"{passes} full decode passes over the same {seg_len} B config-{args.config} segment "
                         f"(host copy), restated wal_iterator.go Next + RecordFromBytes with SSE4.2 CRC, 1 thread, "
                         f"{dt:.1f} s, {platform.processor() or platform.machine()}"}

    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"config {args.config}: {seg_len} B WAL segment per GPU, NsSize 20, 100 B keys, "
                               + ("4 KiB values" if args.config == "B" else "Zipf(1.1) 128 B-64 KiB values")
                               + ", device-resident decode+CRC+record parse",
                   "seg_bytes": seg_len, "records": n_rec, "fragments": n_frags,
                   "parallelism": f"one independent segment per GPU x{world}"},
        "roofline": roofline, "cpu_baseline": cpu,
        "pcie_inclusive_GiBs": round(pcie, 2) if pcie else None,
        "event_ms_per_step": round(ev_ms / args.steps, 4),
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
