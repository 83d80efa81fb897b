"""The multi-rank path on the GPU: libbcw driven from two rank processes at once (on a 1-GPU box both share
device 0), each decoding its own segment against the oracle, and bench.py --gpus 2 starting its own ranks."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

from bitcaskdb_amd import shard

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _clean_env():
    return {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}


def test_two_ranks_decode_vs_oracle():
    plans = shard.launch_plan(2, _clean_env())
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "_rank_decode.py")], env=e,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for e in plans]
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    got = json.loads([ln for ln in outs[0][0].splitlines() if ln.startswith("[")][-1])
    assert [g["rank"] for g in got] == [0, 1] and [g["seed"] for g in got] == [42, 43]
    assert all(g["ok"] and g["n"] > 0 for g in got), got
    assert len({g["wall_max"] for g in got}) == 1


def test_config_d_two_ranks_full_size():
    """BASELINE.json config D's per-rank workload through the sharded launcher: two rank processes started by
    shard.launch_plan (sharing device 0 on the 1-GPU box), each decoding its own 1 GiB config-B segment (seed
    42 + rank), every column and payload hash against the oracle (compaction.go:203-211, db_impl.go:274-281:
    one wal file per scan step, files independent)"""
    plans = shard.launch_plan(2, _clean_env())
    for e in plans:
        e["BCW_RANK_CONFIG"] = "D"
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "_rank_decode.py")], env=e,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for e in plans]
    outs = [p.communicate(timeout=600) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    got = json.loads([ln for ln in outs[0][0].splitlines() if ln.startswith("[")][-1])
    assert [g["rank"] for g in got] == [0, 1] and [g["seed"] for g in got] == [42, 43]
    assert all(g["ok"] for g in got), got
    assert all(g["seg_bytes"] >= 1 << 30 and g["n"] > 250_000 and g["frags"] > 280_000 for g in got), got


def test_bench_gpus2_config_d():
    """bench.py --gpus 2 at config D's full 1 GiB per rank: the driver's multi-GPU line (n_gpus 2, one
    independent segment per rank, every rank's decode checked by bench.py itself before timing)"""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--seg-bytes", str(1 << 30),
                          "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-extras", "--inflight", "1"],
                         env=_clean_env(), capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(ln) for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["scaling"] == "weak" and ln["value"] > 0
    assert ln["config"]["seg_bytes"] >= 1 << 30 and ln["config"]["records"] > 250_000
    assert "x2" in ln["config"]["parallelism"]


def test_bench_gpus2_self_launch():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--seg-bytes", str(64 << 20),
                          "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-extras", "--inflight", "1"],
                         env=_clean_env(), capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(ln) for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 alone prints
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["value"] > 0 and ln["scaling"] == "weak"
