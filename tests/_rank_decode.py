"""One rank of tests/test_gpu_multirank.py (test infrastructure): started as a child process with RANK /
WORLD_SIZE / MASTER_* in its environment, it decodes its own segment (seed 42 + rank) through libbcw on its
GPU (ranks share device 0 on a 1-GPU box, gloo for the barrier and the gathers), compares every column with
the CPU oracle, and rank 0 prints the gathered verdicts as one JSON line.

BCW_RANK_CONFIG=D: BASELINE.json config D's per-rank workload instead of the small mixed segments -- a 1 GiB
config-B segment (100 B keys / 4 KiB values, seed 42 + rank) per rank, checked by tests/_parity.full_parity
(every fragment and record column and every payload's hash against oc_decode_segment)."""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    import _oracle as O
    from bitcaskdb_amd import Context, shard

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = shard.rank_device(int(os.environ.get("LOCAL_RANK", rank)), torch.cuda.device_count())
    seed = shard.segment_seed(42, rank)
    config_d = os.environ.get("BCW_RANK_CONFIG") == "D"
    ctx = Context(dev)
    verdict = {}
    if config_d:  # compaction.go's full scan: one 1 GiB segment per rank (compaction.go:203-211)
        import cases
        from _parity import full_parity
        seg = O.synth(1 << 30, 0, seed, value_mode=0)

        def step_d():
            try:
                got, ref = full_parity(ctx, seg, cases.params(), f"D rank {rank}")
                verdict.update(ok=got.result.err_class == 0, n=int(got.n_records), frags=len(ref.frags),
                               seg_bytes=len(seg))
            except AssertionError as e:
                verdict.update(ok=False, n=-1, err=str(e)[:500])
        wall = shard.timed_steps(step_d, 1, 0, torch.cuda.synchronize, dist.barrier)
        wall_max = shard.max_over_ranks(wall, dist)
        out = [None] * world
        dist.all_gather_object(out, dict(verdict, rank=rank, device=dev, seed=seed, wall=wall, wall_max=wall_max))
        ctx.close()
        if rank == 0:
            print(json.dumps(out), flush=True)
        dist.destroy_process_group()
        return
    seg = O.synth(48 << 20, 0, seed, value_mode=rank % 2)  # rank 1: config-C record sizes
    ref = O.decode(seg, 40, 1_700_000_000, 20, 20, want_bytes=False)

    def step():
        got = ctx.decode(np.frombuffer(seg, dtype=np.uint8), 40, 1_700_000_000, 20, 20, with_frags=True)
        ok = got.result.err_class == ref.err_class and got.n_records == len(ref.recs)
        for col in ("foff", "size", "first_frag", "emit_frag", "status", "key_len", "val_len"):
            ok = ok and bool((got.table[col].astype(np.uint64) == ref.recs[col].astype(np.uint64)).all())
        nf = len(ref.frags)
        ok = ok and bool((got.frags["crc_ok"][:nf] == ref.frags["crc_ok"]).all())
        verdict.update(ok=ok, n=int(got.n_records))

    wall = shard.timed_steps(step, 2, 1, torch.cuda.synchronize, dist.barrier)
    wall_max = shard.max_over_ranks(wall, dist)
    out = [None] * world
    dist.all_gather_object(out, dict(verdict, rank=rank, device=dev, seed=seed, wall=wall, wall_max=wall_max))
    ctx.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
