"""GPU parity of the device index against the index oracle (oracle/bcw_oracle.c
oc_index_*, itself pinned by murmur3 known answers and a Python model in test_index_oracle.py):
Put/Delete/SoftDelete batches with the reference's sequential last-op-wins order, Get, growth, export,
the recovery Put loops over hint / data WALs, and the device compaction filter feeding the re-encode."""
from __future__ import annotations

import random

import numpy as np
import pytest

import _oracle as O
import cases
from bitcaskdb_amd import _lib as L
from bitcaskdb_amd import index as IX
from bitcaskdb_amd import wal as W

pytestmark = pytest.mark.gpu
BASE = cases.BASE


def _keyset(rng, n, ns=20):
    out = []
    for i in range(n):
        nsb = bytes([65 + i % 5]) * ns
        k = bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 7, 8, 15, 16, 17, 31, 100, 250])))
        out.append((nsb, k + b"%d" % i))
    return out


def check_against_oracle(ix, oc, keys):
    st, fid, off, size = ix.get_many([ns + k for ns, k in keys])
    for j, (ns, k) in enumerate(keys):
        ost, (of, oo, osz) = oc.get(ns, k)
        assert st[j] == ost, (j, st[j], ost)
        if ost != 1:
            assert (fid[j], off[j], size[j]) == (of, oo, osz), j


def test_index_batches_vs_oracle(ctx):
    rng = random.Random(1)
    keys = _keyset(rng, 3000)
    ix = IX.Index(ctx, keys=1024, arena_bytes=1 << 16)  # small: the batches force growth (rehash)
    oc = O.Index()
    for batch in range(12):
        n = rng.choice([1, 50, 2000, 9000])
        ops, ks, fids, offs, sizes = [], [], [], [], []
        for _ in range(n):
            ns, k = rng.choice(keys)  # duplicates inside a batch: the last op wins
            op = rng.choice([0, 0, 0, 0, 1, 2])
            f, o, z = rng.randrange(1, 50), rng.randrange(40, 1 << 40), rng.randrange(5, 1 << 20)
            ops.append(op)
            ks.append(ns + k)
            fids.append(f)
            offs.append(o)
            sizes.append(z)
            oc.set(ns, k, op, f, o, z)
        ix.apply(ops, ks, fids, offs, sizes)
        check_against_oracle(ix, oc, keys + _keyset(random.Random(99), 50))
    s = ix.stats()
    assert s.live == oc.live() and s.overflow == 0 and s.slot_capacity > 1024
    exp = ix.export()
    assert len(exp) == oc.live()
    for mk, v in exp.items():
        st, ov = oc.get(mk[:20], mk[20:])
        assert st != 1 and ov == v
    # the reference's single-key interface and errors
    ns, k = keys[0]
    ix.put(ns, k, 7, 1234, 99)
    assert ix.get(ns, k) == (7, 1234, 99)
    ix.soft_delete(ns, k)
    with pytest.raises(IX.ErrKeySoftDeleted):
        ix.get(ns, k)
    ix.delete(ns, k)
    with pytest.raises(IX.ErrKeyNotFound):
        ix.get(ns, k)
    ix.close()


def _wal_set(seed, nfiles=3, n=400, nkeys=500, vlens=(10, 300, 5000, 40000)):
    rng = random.Random(seed)
    files = {}
    for fid in range(1, nfiles + 1):
        payloads = [cases.rec(rng.randrange(0, nkeys), vlen=rng.choice(vlens)) for _ in range(n)]
        data, _ = cases.wal_of(payloads)
        ec, _, _, hint = O.hint_by_wal(data, fid, 40, BASE, 20, 20)
        assert ec == 0
        files[fid] = (data, hint)
    return files


def test_recover_from_hints_and_wals(ctx):
    """recoverFromWals (db_impl.go:268-314): ascending fids, hint files preferred; a corrupted hint is
    followed by its data WAL with the hint's earlier puts kept; the result equals the oracle's index."""
    files = _wal_set(2)
    fid2_data, fid2_hint = files[2]
    bad = bytearray(fid2_hint)
    bad[len(bad) // 2] ^= 0x21  # CRC failure mid-hint -> fall back to the WAL of fid 2
    oc = O.Index()
    for fid in sorted(files):
        data, hint = files[fid]
        h = bytes(bad) if fid == 2 else hint
        ec, _ = oc.put_segment(h, 40, BASE, 20, 0, 1, fid)
        if ec != 0:
            assert fid == 2
            assert oc.put_segment(data, 40, BASE, 20, 20, 0, fid)[0] == 0
    ix = IX.Index(ctx)
    IX.recover_from_wals(ix, {fid: (W.load_wal(d, fid), W.load_wal(bytes(bad) if fid == 2 else h, fid))
                              for fid, (d, h) in files.items()})
    exp = ix.export()
    assert len(exp) == oc.live() == ix.stats().live
    for mk, v in exp.items():
        st, ov = oc.get(mk[:20], mk[20:])
        assert st == 0 and ov == v


def test_recover_onephase_record_fid(ctx):
    """onePhase (compaction.go:248-251) puts hint.fid (the compaction output fid), recovery the file fid."""
    data, _ = cases.wal_of([cases.rec(i, vlen=30) for i in range(100)])
    ec, _, _, hint = O.hint_by_wal(data, 77, 40, BASE, 20, 20)
    ix = IX.Index(ctx)
    dres, ires = ix.recover_segment(hint, L.MODE_HINT, 5, 40, BASE, 20, 0, use_record_fid=True)
    assert ires.err_class == 0 and ires.n_in == 100 == ires.n_done
    assert {v[0] for v in ix.export().values()} == {77}
    dres, ires = ix.recover_segment(hint, L.MODE_HINT, 5, 40, BASE, 20, 0)
    assert {v[0] for v in ix.export().values()} == {5}


def test_compaction_filter_fused(ctx):
    """the device doFilter (compaction.go:329-348) over the oldest WAL after recovery: keep mask == the
    oracle's, and the fused decode -> filter -> encode writes the same bytes as oc_compact_append with
    that mask; soft-deleted and deleted keys are dropped."""
    files = _wal_set(3, nfiles=3, n=600)
    ix = IX.Index(ctx)
    oc = O.Index()
    for fid in sorted(files):
        data, hint = files[fid]
        ix.recover_segment(hint, L.MODE_HINT, fid, 40, BASE, 20, 0)
        oc.put_segment(hint, 40, BASE, 20, 0, 1, fid)
    # later writes: soft-delete / delete some keys (DBImpl.writeIndex, db_impl.go:433-452)
    rng = random.Random(4)
    ns = cases.sha1("ns")[:20]
    ops, ks = [], []
    for i in rng.sample(range(500), 60):
        op = rng.choice([L.IDX_DELETE, L.IDX_SOFT_DELETE])
        ops.append(op)
        ks.append(ns + b"key-%06d" % i)
        oc.set(ns, b"key-%06d" % i, op)
    ix.apply(ops, ks)
    src = files[1][0]
    keep_ref, nv = oc.compact_filter(src, 40, BASE, 20, 20, 1, 600)
    assert 0 < int(keep_ref.sum()) < 600
    dst, hint = W.WalFile(9, BASE), W.WalFile(9, BASE)
    offs, kept = IX.compact_one_wal_filtered(dst, hint, W.load_wal(src, 1), ix)
    assert kept == int(keep_ref.sum())
    rd, rh = O.Writer(BASE, BASE), O.Writer(BASE, BASE)
    ec, _, nin, roffs = O.compact_append(rd, rh, 9, src, 40, BASE, BASE, 20, 20, keep_ref)
    assert ec == 0 and bytes(dst.data) == rd.data() and bytes(hint.data) == rh.data()
    np.testing.assert_array_equal(offs[:nin], roffs[:nin])


def test_filter_zero_length_first_drops_live_record(ctx):
    """a record whose First fragment is zero-length is indexed (Put at write time)
    at its First header, but the iterator reports the next block -> doFilter drops the live record."""
    first = cases.rec(0, vlen=0, klen=8)
    target = 32768 - 7 - 7
    filler = cases.rec(0, vlen=target - len(first) - 2, klen=8)  # the value-length varint grows by 2
    assert len(filler) == target
    payloads = [filler] + [cases.rec(i, vlen=300, klen=8) for i in range(1, 30)]
    data, offs = cases.wal_of(payloads)
    ix, oc = IX.Index(ctx), O.Index()
    ns = cases.sha1("ns")[:20]
    keys = [p[p[0]:p[0] + 8] for p in payloads]
    ix.apply([L.IDX_PUT] * len(payloads), [ns + k for k in keys], [1] * len(payloads), offs,
             [len(p) for p in payloads])
    for k, o, p in zip(keys, offs, payloads):
        oc.put(ns, k, 1, o, len(p))
    keep_ref, _ = oc.compact_filter(data, 40, BASE, 20, 20, 1, len(payloads))
    assert keep_ref[1] == 0 and keep_ref.sum() == len(payloads) - 1
    dst, hint = W.WalFile(9, BASE), W.WalFile(9, BASE)
    _, kept = IX.compact_one_wal_filtered(dst, hint, W.load_wal(data, 1), ix)
    assert kept == len(payloads) - 1


def test_index_config_b_scale(ctx):
    """the hint WAL of a 1 GiB config-B segment (~254 k keys) rebuilt into the device index, then the
    device filter over the data WAL keeps every record (each key's latest copy is in this file)."""
    data = O.synth(1 << 30, 0, 42)
    ec, _, n, hint = O.hint_by_wal(data, 1, 40, BASE, 20, 20)
    assert ec == 0
    ix = IX.Index(ctx)
    dres, ires = ix.recover_segment(hint, L.MODE_HINT, 1, 40, BASE, 20, 0)
    assert ires.err_class == 0 and ires.n_done == n
    assert ix.stats().live == n
    dst, hint_w = W.WalFile(2, BASE), W.WalFile(2, BASE)
    _, kept = IX.compact_one_wal_filtered(dst, hint_w, W.load_wal(data, 1), ix)
    assert kept == n
    assert bytes(dst.data)[40:] == data[40:]  # every record kept, same base time: the same bytes


def test_write_stats_vs_oracle(ctx):
    """bcw_index_apply_stat: every op's WriteStat (index.go:100-165) equals the reference index's -- the oracle's
    SimpleMap/ShardMap restatement with a Limited above the key count (no eviction, the device's regime) --
    including ops on keys an earlier op of the same batch touched; writeIndex's per-fid sums follow."""
    rng = random.Random(11)
    keys = _keyset(rng, 400)
    ix = IX.Index(ctx, keys=1024, arena_bytes=1 << 16)
    om = O.SMap(1 << 20, 1 << 19, 32, 5)
    for batch in range(8):
        n = rng.choice([1, 64, 700, 3000])
        ops, ks, fids, offs, sizes, want = [], [], [], [], [], []
        for _ in range(n):
            ns, k = rng.choice(keys)
            op = rng.choice([0, 0, 0, 1, 2])
            f, o, z = rng.randrange(1, 9), rng.randrange(40, 1 << 40), rng.randrange(5, 1 << 20)
            ops.append(op)
            ks.append(ns + k)
            fids.append(f)
            offs.append(o)
            sizes.append(z)
            want.append(om.index_op(ns, k, op, f, o, z))
        if batch % 2:
            ref = {}
            for wf, wb in want:  # writeStats[stat.FreeWalFid] += stat.FreeBytes (db_impl.go:450)
                ref[wf] = ref.get(wf, 0) + wb
            assert ix.write_index(ops, ks, fids, offs, sizes) == ref
            continue
        found, ffid, fbytes = ix.apply(ops, ks, fids, offs, sizes, stats=True)
        for i, (wf, wb) in enumerate(want):
            assert (int(ffid[i]), int(fbytes[i])) == (wf, wb), (batch, i, ops[i])
            if found[i] == 0:
                assert wb == 0 and wf == 0
    # the device agrees with the oracle map on every key afterwards
    st, fid, off, size = ix.get_many([ns + k for ns, k in keys])
    for j, (ns, k) in enumerate(keys):
        ost, ov = om.index_get(ns, k)
        assert st[j] == ost and (ost == 1 or (int(fid[j]), int(off[j]), int(size[j])) == ov), j
    ix.close()


def test_rebuild_over_existing_keys_takes_no_arena(ctx):
    """only keys new to the index take arena space: a rebuild over the same keys (recovery of a WAL whose keys
    are indexed) leaves the arena as it was (round-2 rebuild regression: every op appended its key)"""
    data, _ = cases.wal_of([cases.rec(i, vlen=100) for i in range(3000)])
    ix = IX.Index(ctx, keys=4096, arena_bytes=1 << 20)
    ix.recover_segment(data, L.MODE_RECORD, 1, 40, BASE, 20, 20)
    a0 = ix.stats().arena_used
    assert a0 > 0
    for _ in range(4):
        dres, ires = ix.recover_segment(data, L.MODE_RECORD, 2, 40, BASE, 20, 20)
        assert ires.n_done == 3000
    s = ix.stats()
    assert s.arena_used == a0 and s.live == 3000
    assert {v[0] for v in ix.export().values()} == {2}
    ix.close()


def test_bounded_index_snapshot_filter(ctx):
    """A bounded Go index (IndexLimited below the key count, db.go:70-72): recovery evicts keys
    (map.go:185-187), doFilter drops their records ("deleted or evicted", compaction.go:330-333). The device
    filter runs against a snapshot of the Go index's live entries (bcw_index_clear + apply): keep masks and
    the re-encoded dst / hint bytes equal the oracle's over the evicting map."""
    files = _wal_set(5, nfiles=3, n=500, nkeys=1500, vlens=(10, 300, 5000))
    om = O.SMap(1024, 512, 32, 5, seed=9)  # 16 shards of 64 buckets / 32 entries
    for fid in sorted(files):
        om.set_now(fid)
        data, hint = files[fid]
        ec, n = om.put_segment(hint, 40, BASE, 20, 0, 1, fid)
        assert ec == 0 and n == 500
    assert om.size() == 512
    snap = om.export()
    assert len(snap) == 512
    ix = IX.Index(ctx)
    ix.apply([L.IDX_PUT], [b"x" * 20 + b"stale"], [9], [99], [9])  # cleared by the snapshot load
    ix.load_snapshot(snap)
    assert ix.stats().live == 512 and ix.export() == snap
    for src_fid in (1, 3):
        src = files[src_fid][0]
        keep_ref, nv = om.compact_filter(src, 40, BASE, 20, 20, src_fid, 500)
        assert nv == 500 and 0 < int(keep_ref.sum()) < 500
        dst, hint = W.WalFile(9, BASE), W.WalFile(9, BASE)
        offs, kept = IX.compact_one_wal_filtered(dst, hint, W.load_wal(src, src_fid), ix)
        assert kept == int(keep_ref.sum())
        rd, rh = O.Writer(BASE, BASE), O.Writer(BASE, BASE)
        ec, _, nin, roffs = O.compact_append(rd, rh, 9, src, 40, BASE, BASE, 20, 20, keep_ref)
        assert ec == 0 and bytes(dst.data) == rd.data() and bytes(hint.data) == rh.data()
        np.testing.assert_array_equal(offs[:nin], roffs[:nin])
    ix.close()


def test_hint_recovery_wide_namespace(ctx):
    """NsSize 300: the hint key offset (NsSize + len(uvarint keyLen), hint.go:62-66) exceeds the table's u8
    column; the device index recomputes it from the payload"""
    ns = bytes(i % 256 for i in range(300))
    w = O.Writer(BASE, BASE)
    offs = [1000 + 37 * i for i in range(300)]
    for i in range(300):  # HintRecord.Encode (hint.go:32-48); a data WAL cannot carry NsSize 300 (byte(headerSize))
        w.write(O.hint_encode(ns, b"k%05d" % i + bytes(i % 200), 4, offs[i], 60 + i))
    hint = w.data()
    oc = O.Index()
    assert oc.put_segment(hint, 40, BASE, 300, 0, 1, 4)[0] == 0
    ix = IX.Index(ctx)
    dres, ires = ix.recover_segment(hint, L.MODE_HINT, 4, 40, BASE, 300, 0)
    assert ires.err_class == 0 and ires.n_done == 300
    exp = ix.export()
    assert len(exp) == oc.live() == 300
    for mk, v in exp.items():
        assert oc.get(mk[:300], mk[300:]) == (0, v)
    got = []
    W.iterate_hint(W.load_wal(hint, 4), lambda h: got.append((h.ns, h.key, h.off)), ns_size=300)
    assert got == [(ns, b"k%05d" % i + bytes(i % 200), offs[i]) for i in range(300)]


class _BoundModel:
    """the device's capacity policy (bcw_index_set_limit) restated: ops in order on a logical clock (an entry's
    stamp is its last Put / SoftDelete), and after every batch each of the 16 shards (murmur3 Sum64 % 16,
    map.go:395-428's ShardMap) holding more than limited / 16 keys evicts its least recently set ones"""

    def __init__(self, limited):
        self.lim = limited // 16
        self.d = {}
        self.t = 0
        self.evicted = self.evicted_bytes = 0

    def op(self, op, k, f=0, o=0, z=0):
        self.t += 1
        if op == L.IDX_DELETE:
            self.d.pop(k, None)
        elif op == L.IDX_SOFT_DELETE:
            self.d[k] = (0, 0, 0, self.t)
        else:
            self.d[k] = (f, o, z, self.t)

    def bound(self):
        by = {}
        for k, v in self.d.items():
            by.setdefault(O.murmur3_sum64(k) & 15, []).append((v[3], k))
        for lst in by.values():
            if len(lst) > self.lim:
                for _, k in sorted(lst)[:len(lst) - self.lim]:
                    self.evicted += 1
                    self.evicted_bytes += self.d[k][2]
                    del self.d[k]

    def export(self):
        return {k: v[:3] for k, v in self.d.items()}


def _shard_counts(entries):
    c = [0] * 16
    for k in entries:
        c[O.murmur3_sum64(k) & 15] += 1
    return c


@pytest.mark.parametrize("limited", [16 * 8, 16 * 40])
def test_index_capacity_bound_batches(ctx, limited):
    """IndexLimited (db.go:71, db_impl.go:165) on the device index: random Put / Delete / SoftDelete batches over a
    key space several times the bound. After every batch the index equals the policy model (entries, evicted count
    and bytes) and no shard holds more than limited / 16 keys (map.go:185-187's bound; the least-recently-set order
    stands in for the reference's Rand-sampled pool, map.go:319-370)"""
    rng = random.Random(limited)
    keys = [ns + k for ns, k in _keyset(rng, 4 * limited)]
    ix = IX.Index(ctx, keys=1024)
    ix.set_limit(limited)
    m = _BoundModel(limited)
    for batch in range(25):
        n = rng.choice([1, 7, 60, 400])
        ops, ks, fs, os_, zs = [], [], [], [], []
        for _ in range(n):
            op = rng.choice([0, 0, 0, 0, 0, 1, 2])
            k = rng.choice(keys)
            f, o, z = rng.randrange(1, 50), rng.randrange(40, 1 << 40), rng.randrange(5, 1 << 20)
            ops.append(op)
            ks.append(k)
            fs.append(f)
            os_.append(o)
            zs.append(z)
            m.op(op, k, f, o, z)
        ix.apply(ops, ks, fs, os_, zs)
        m.bound()
        exp = ix.export()
        assert exp == m.export(), batch
        assert max(_shard_counts(exp)) <= limited // 16
        s = ix.stats()
        assert (s.live, s.limited, s.evicted, s.evicted_bytes, s.overflow) == (len(exp), limited, m.evicted,
                                                                              m.evicted_bytes, 0), batch
    assert m.evicted > 0
    # a Get of an evicted key fails like a deleted one's (ErrKeyNotFound)
    gone = [k for k in keys if k not in m.d][:50]
    st, _, _, _ = ix.get_many(gone)
    assert all(int(x) == 1 for x in st)
    ix.close()


def test_index_capacity_bound_recovery(ctx):
    """recovery (recoverFromWal's Put loop, db_impl.go:286-313) into a bounded index: each hint / WAL is one batch;
    the index equals the policy model after every file and never holds more than the bound; set_limit on a fuller
    index applies the bound at once; the fan-out recovery (bcw_recover_wals) into a bounded index respects it too
    (its per-file batches hold each file's last put per key, so which keys survive may differ from the serial
    path's: the bound, not the set, is the property there)"""
    files = _wal_set(8, nfiles=4, n=500, nkeys=1500, vlens=(10, 300, 5000))
    limited = 16 * 20
    ix = IX.Index(ctx)
    ix.set_limit(limited)
    m = _BoundModel(limited)
    for fid in sorted(files):
        data, _ = files[fid]
        dec = O.decode(data, 40, BASE, 20, 20, want_bytes=True)
        dres, ires = ix.recover_segment(data, L.MODE_RECORD, fid, 40, BASE, 20, 20)
        assert dres.err_class == 0 and ires.n_done == len(dec.recs) == 500
        for r, pay in zip(dec.recs, dec.payloads):
            ko, kl = int(r["hdr_size"]), int(r["key_len"])
            m.op(L.IDX_PUT, bytes(pay[1:21]) + bytes(pay[ko:ko + kl]), fid, int(r["foff"]) - 7, int(r["size"]))
        m.bound()
        exp = ix.export()
        assert exp == m.export(), fid
        assert len(exp) <= limited and max(_shard_counts(exp)) <= limited // 16
    # an unbounded index, bounded afterwards
    un = IX.Index(ctx)
    for fid in sorted(files):
        un.recover_segment(files[fid][0], L.MODE_RECORD, fid, 40, BASE, 20, 20)
    assert un.stats().live > limited
    un.set_limit(limited)
    assert max(_shard_counts(un.export())) <= limited // 16 and un.stats().evicted > 0
    # the fan-out into a bounded index
    ctx2 = W.Context(0)
    fan = IX.Index(ctx)
    fan.set_limit(limited)
    wals = {fid: (W.load_wal(d, fid), W.load_wal(h, fid)) for fid, (d, h) in files.items()}
    IX.recover_from_wals(fan, wals, contexts=[ctx2])
    exp = fan.export()
    assert 0 < len(exp) <= limited and max(_shard_counts(exp)) <= limited // 16
    assert all(f in files for f, _, _ in exp.values())
    ctx2.close()
    for x in (ix, un, fan):
        x.close()
