"""Multi-rank path on CPU: world_size-2 gloo processes run the same sharding/timing code as bench.py
(bitcaskdb_amd.shard), each decoding its own synthetic segment with the CPU oracle standing in for
the device decode (the GPU path is covered by test_gpu_*)."""
from __future__ import annotations

import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from bitcaskdb_amd import shard

SEG = 1 << 20


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import _oracle as O
        seed = shard.segment_seed(42, rank)
        seg = O.synth(SEG, 0, seed)
        result = {}

        def step():
            d = O.decode(seg, 40, 1_700_000_000, 20, 20)
            result["n"] = len(d.recs)
            result["err"] = d.err_class
            result["first_foff"] = int(d.recs["foff"][0])
            result["sizes"] = int(d.recs["size"].sum())
            result["digest"] = int(d.frags["stored_crc"].astype("uint64").sum())

        wall = shard.timed_steps(step, 2, 1, lambda: None, dist.barrier)
        wall_max = shard.max_over_ranks(wall, dist)
        gathered = [None] * world
        dist.all_gather_object(gathered, dict(result, seed=seed, wall=wall, wall_max=wall_max, seg=len(seg)))
        if rank == 0:
            out.put(gathered)
    finally:
        dist.destroy_process_group()


def test_assign_segments_covers_each_once():
    for n in (0, 1, 7, 64):
        for world in (1, 2, 3, 8):
            got = sorted(i for r in range(world) for i in shard.assign_segments(n, world, r))
            assert got == list(range(n))
    with pytest.raises(ValueError):
        shard.assign_segments(4, 2, 2)


def test_aggregate_rate():
    assert shard.aggregate_gib_s([1 << 30, 1 << 30], 2.0, 4) == pytest.approx(4.0)
    with pytest.raises(ValueError):
        shard.aggregate_gib_s([1], 0.0, 1)


def test_gloo_world2_independent_segments():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [g["seed"] for g in gathered] == [42, 43]
    # every rank decoded its own segment cleanly; the segments differ
    assert all(g["err"] == 0 and g["n"] > 0 for g in gathered)
    assert gathered[0]["digest"] != gathered[1]["digest"]
    # max-over-ranks: both ranks agree and it bounds each rank's own time
    wm = {g["wall_max"] for g in gathered}
    assert len(wm) == 1
    wall_max = wm.pop()
    assert all(g["wall"] <= wall_max + 1e-9 for g in gathered)
    value = shard.aggregate_gib_s([g["seg"] for g in gathered], wall_max, 2)
    assert value > 0
