"""Multi-GPU sharding of the WAL decode: one process per GPU, no collective on the data path.

bitcaskDB decodes WAL segments independently of each other (compaction.go:294-327 scans one wal file
per compactOneWal call; NewHintByWal, hint.go:123-161, likewise one file at a time), so the unit of
parallelism across GPUs is the segment: rank r takes segments r, r + world, r + 2*world, ... and
decodes them on its own device. The only cross-rank traffic is the benchmark's barrier and the
max-over-ranks of the timed region (bench.py); throughput therefore scales weakly with the number of
GPUs. These helpers hold that logic so that the CPU tests (gloo, world_size 2) exercise the same
code the GPU benchmark runs.
"""
from __future__ import annotations

import os
import socket
import subprocess
import time
from typing import Callable, Mapping, Optional, Sequence


def segment_seed(base: int, rank: int) -> int:
    """Seed of the synthetic segment a rank decodes in the benchmark (independent per rank)."""
    return base + rank


def assign_segments(n_segments: int, world: int, rank: int) -> list[int]:
    """Round-robin assignment of segment indices to ranks (every segment exactly once)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    return list(range(rank, n_segments, world))


def timed_steps(step: Callable[[], None], steps: int, warmup: int, sync: Callable[[], None],
                barrier: Optional[Callable[[], None]] = None) -> float:
    """Run `warmup` untimed steps, then time exactly `steps` steps bracketed by barrier + sync on
    both sides. Returns this rank's wall time in seconds."""
    for _ in range(warmup):
        step()
    sync()
    if barrier is not None:
        barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if barrier is not None:
        barrier()
    return time.perf_counter() - t0


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """MAX of a float over all ranks (identity without an initialised process group)."""
    if dist is None or not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_gib_s(bytes_per_rank: Sequence[int], wall_max_s: float, steps: int) -> float:
    """Whole-job throughput: every rank's bytes per step, over the slowest rank's time per step."""
    if wall_max_s <= 0 or steps <= 0:
        raise ValueError("empty timing")
    return sum(bytes_per_rank) / 2 ** 30 / (wall_max_s / steps)


def launch_plan(gpus: int, env: Mapping[str, str]) -> Optional[list[dict]]:
    """How `bench.py --gpus N` runs: None when this process is already the job (N = 1, or a rank started by
    torch.distributed.run with WORLD_SIZE = N); otherwise the environments of the N rank processes to start,
    one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1). A WORLD_SIZE that disagrees
    with --gpus is an error: the job would silently run on the wrong number of GPUs."""
    if gpus < 1:
        raise ValueError(f"--gpus {gpus}: need at least one GPU")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise ValueError(f"--gpus {gpus} but WORLD_SIZE={world}: launch with --nproc-per-node {gpus} "
                             f"or drop the launcher")
        return None
    if gpus == 1:
        return None
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    plans = []
    for r in range(gpus):
        e = dict(env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        plans.append(e)
    return plans


def spawn_ranks(argv: Sequence[str], plans: Sequence[Mapping[str, str]], timeout: Optional[float] = None) -> int:
    """Start one child process per plan (never an exec of this process: the children are new programs, started
    before this process touches a GPU) and wait for all of them; returns the first nonzero exit code, else 0.
    A rank that fails takes the others down (they would wait at the rendezvous or a barrier)."""
    procs = [subprocess.Popen(list(argv), env=dict(e)) for e in plans]
    rc = 0
    deadline = None if timeout is None else time.monotonic() + timeout
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:
                    q.terminate()
        if deadline is not None and time.monotonic() > deadline:
            for q in pending:
                q.kill()
            return rc or 124
        time.sleep(0.05)
    return rc


def rank_device(local_rank: int, device_count: int) -> int:
    """The GPU of a local rank: its own when the node has enough, else ranks share devices round-robin (the
    1-GPU box's multi-rank test)."""
    if device_count <= 0:
        raise RuntimeError("no GPU")
    return local_rank % device_count
