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

import time
from typing import Callable, Optional, Sequence


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
