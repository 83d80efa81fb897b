"""The bounded-index oracle (oracle/bcw_oracle.c oc_smap_*: map.go's SimpleMap / ShardMap with the sampled
approximate-LRU eviction, Rand / WallTime injected) pinned by the reference's own map and index tests,
restated scenario by scenario (map_test.go, index_test.go)."""
from __future__ import annotations

import struct

import pytest

import _oracle as O


def u64(i: int) -> bytes:
    return struct.pack("<Q", i)


def simple_map(rand_vals):
    # map_test.go mockSimpleMapOperator: Hash(k) = k, Rand(n) = fixedValues[i] % n (cycled), one SimpleMap
    return O.SMap(100, 80, 16, 3, nshards=1, hash_mode=1, rand_vals=rand_vals)


def test_options_validate():
    """MapOptions.validate (map.go:102-120): Limited <= Capacity, 16 <= EvictionPoolCapacity <= Limited,
    SampleKeys >= 1"""
    for args in ((100, 120, 16, 3), (100, 80, 90, 3), (100, 80, 16, 0), (100, 80, 15, 3)):
        with pytest.raises(ValueError):
            O.SMap(*args, nshards=1)
    O.SMap(100, 80, 16, 3, nshards=1)


def test_simple_map_basic_operations():
    """map_test.go TestMap_SimpleMapBasicOperations"""
    m = simple_map([1, 2, 3])
    for k in (1, 2, 3):
        assert m.set(u64(k), (k,))[0] == 0
    assert m.get(u64(1))[0] == 1 and m.get(u64(2))[0] == 2
    r, old = m.set(u64(1), (11,))
    assert r == 1 and old[0] == 1 and m.get(u64(1))[0] == 11
    for i in range(4, 82):
        m.set(u64(i), (i,))
    assert m.get(u64(1)) is None  # the first evicted key (evictionOrder[0])
    old = m.delete(u64(2))
    assert old is not None and old[0] == 2
    assert m.get(u64(2)) is None


def test_simple_map_eviction_order():
    """map_test.go TestMap_SimpleMapEvictionOrder: Rand 1..6 samples buckets 1, 2, 3 then 4, 5, 6; equal
    expires keep the sample order in the pool, so key 1 is evicted first, then key 2 (the pool keeps its
    stale duplicate, map.go:338-339)"""
    m = simple_map([1, 2, 3, 4, 5, 6])
    for i in range(1, 81):
        r, _ = m.set(u64(i), (i,))
        assert r == 0
    r, old = m.set(u64(81), (81,))
    assert r == 2 and old[0] == 1
    assert m.get(u64(1)) is None
    for i in range(2, 82):
        assert m.get(u64(i))[0] == i
    r, old = m.set(u64(82), (82,))
    assert r == 2 and old[0] == 2
    assert m.get(u64(2)) is None
    for i in range(3, 83):
        assert m.get(u64(i))[0] == i
    assert m.size() == 80


def test_shard_map_basic():
    """map_test.go TestMap_ShardMapBasic (murmur3 hash, 16 shards)"""
    m = O.SMap(1000, 800, 16, 3)
    for k in (b"123", b"456", b"789"):
        m.set(k, (int(k),))
    assert m.get(b"123")[0] == 123 and m.get(b"456")[0] == 456
    r, old = m.set(b"123", (111,))
    assert r == 1 and old[0] == 123 and m.get(b"123")[0] == 111
    assert m.delete(b"456")[0] == 456 and m.get(b"456") is None


def test_shard_map_lru_eviction():
    """map_test.go TestMap_ShardMapLRUEviction: 999 999 keys into Limited 800 000; the clock advances while
    they are written (about 1 s per 100 k sets here), so the older first half is evicted more (> 100 000)"""
    m = O.SMap(1_000_000, 800_000, 32, 5, seed=7)
    n = 1_000_000
    for i in range(1, n):
        if i % 100_000 == 0:
            m.set_now(i // 100_000)
        m.set(str(i).encode(), (i,))
    assert m.size() == 800_000
    missing = sum(1 for i in range(1, 500_001) if m.get(str(i).encode()) is None)
    assert missing > 100_000
    for i in range(1, n, 997):  # survivors hold their own values
        v = m.get(str(i).encode())
        assert v is None or v[0] == i


def test_index_eviction_write_stats():
    """index_test.go TestIndexEviction: Capacity 1000 / Limited 800 (16 shards of 62 / 50 entries), every
    Put past the limit evicts one entry and reports its valueSize as freed: total = 100 * (N - 800)"""
    m = O.SMap(1000, 800, 32, 5, seed=3)
    ns = b"ns1"
    total = 0
    n = 200_000
    for i in range(1, n + 1):
        _, fb = m.index_op(ns, b"key%d" % i, 0, 1, i * 100, 100)
        total += fb
    assert total == 100 * (n - 800)
    assert m.size() == 800


def test_index_basic_and_delete_operations():
    """index_test.go TestIndexBasicOperations / TestIndexDeleteOperations over the bounded map"""
    m = O.SMap(1000, 800, 32, 5)
    ns = b"ns1"
    m.index_op(ns, b"key1", 0, 1, 100, 100)
    m.index_op(ns, b"key2", 0, 2, 200, 100)
    assert m.index_get(ns, b"key1") == (0, (1, 100, 100))
    assert m.index_get(ns, b"key2") == (0, (2, 200, 100))
    assert m.index_op(ns, b"key1", 0, 3, 300, 100) == (1, 100)  # WriteStat of the replaced value
    assert m.index_get(ns, b"key1") == (0, (3, 300, 100))
    assert m.index_op(ns, b"key1", 1) == (3, 100)
    assert m.index_get(ns, b"key1")[0] == 1
    assert m.index_op(ns, b"key1", 1) == (0, 0)  # ErrKeyNotFound: no stat
    assert m.index_op(ns, b"key2", 2) == (2, 100)
    assert m.index_get(ns, b"key2")[0] == 2  # ErrKeySoftDeleted
