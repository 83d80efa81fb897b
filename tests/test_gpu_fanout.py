"""GPU parity of the one-process, several-context fan-outs (bcw_recover_wals, bcw_compact_wals) against the
oracle's sequential loops: recoverFromWals (db_impl.go:268-314) puts file by file in ascending fid, and
doCompactionWork (compaction.go:201-211) appends source by source. Two contexts on device 0 stand in for two
devices (the box has one GPU): the decodes run concurrently, the puts / appends keep the reference's order."""
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
NS = cases.sha1("ns")[:20]


@pytest.fixture(scope="module")
def ctx2():
    c = W.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def ctx3():
    c = W.Context(0)
    yield c
    c.close()


def _files(seed, nfiles, n=300, nkeys=400, vlens=(10, 300, 5000, 40000)):
    """nfiles data WALs over a shared key space (later fids override earlier ones) with their hint files"""
    rng = random.Random(seed)
    files = {}
    for fid in rng.sample(range(1, 1000), nfiles):  # fids not in creation order: the call sorts them
        payloads = [cases.rec(rng.randrange(0, nkeys), vlen=rng.choice(vlens)) for _ in range(n)]
        data, _ = cases.wal_of(payloads)
        ec, _, _, hint = O.hint_by_wal(data, fid, 40, BASE, 20, 20)
        assert ec == 0
        files[fid] = (data, hint)
    return files


def _corrupt(b: bytes, at: float) -> bytes:
    x = bytearray(b)
    x[int(len(x) * at)] ^= 0x21
    return bytes(x)


def _oracle_recover(files):
    """the reference's serial loop: (oracle index, fid it stopped at or None)"""
    oc = O.Index()
    for fid in sorted(files):
        data, hint = files[fid]
        if hint is not None and oc.put_segment(hint, 40, BASE, 20, 0, 1, fid)[0] == 0:
            continue
        if oc.put_segment(data, 40, BASE, 20, 20, 0, fid)[0] != 0:
            return oc, fid
    return oc, None


def _wals(files):
    return {fid: (W.load_wal(d, fid), W.load_wal(h, fid) if h is not None else None) for fid, (d, h) in files.items()}


def _same_as_oracle(ix, oc):
    exp = ix.export()
    assert len(exp) == oc.live() == ix.stats().live
    for mk, v in exp.items():
        st, ov = oc.get(mk[:20], mk[20:])
        assert st == 0 and ov == v, (mk, v, ov)


@pytest.mark.parametrize("with_index_ctx", [True, False])
def test_recover_fanout_two_contexts(ctx, ctx2, ctx3, with_index_ctx):
    """7 files, round-robin over two contexts: a corrupted hint (falls back to its WAL, keeping the hint's
    earlier puts), a file without a hint, overlapping keys across files. The index equals the oracle's serial
    result and the device's own serial result (entries, live count, slots and arena used)."""
    files = _files(11, 7)
    fids = sorted(files)
    d, h = files[fids[2]]
    files[fids[2]] = (d, _corrupt(h, 0.6))
    files[fids[4]] = (files[fids[4]][0], None)
    oc, stop = _oracle_recover(files)
    assert stop is None
    ix = IX.Index(ctx)
    IX.recover_from_wals(ix, _wals(files), contexts=[ctx, ctx2] if with_index_ctx else [ctx2, ctx3])
    _same_as_oracle(ix, oc)
    ser = IX.Index(ctx)
    IX.recover_from_wals(ser, _wals(files))
    assert ser.export() == ix.export()
    a, b = ser.stats(), ix.stats()
    assert (a.live, a.slots_used, a.arena_used, a.overflow) == (b.live, b.slots_used, b.arena_used, 0)


def test_fanout_refuses_a_context_listed_twice(ctx, ctx2):
    """each worker thread owns its context's decode scratch: a context named twice is BCW_E_INVAL, for
    recovery and compaction alike, and nothing is applied"""
    files = _files(13, 3)
    ix = IX.Index(ctx)
    with pytest.raises(RuntimeError, match="invalid"):
        IX.recover_from_wals(ix, _wals(files), contexts=[ctx2, ctx2])
    assert ix.export() == {}
    srcs, _, _, _ = _compaction_setup(14, 2)
    dst, hint = W.WalFile(77, BASE), W.WalFile(77, BASE)
    n0, h0 = dst.size(), hint.size()
    with pytest.raises(RuntimeError, match="invalid"):
        IX.compact_wals_filtered(dst, hint, [W.load_wal(d, fid) for fid, d in srcs], ix, contexts=[ctx, ctx2, ctx])
    assert (dst.size(), hint.size()) == (n0, h0)


def test_recover_fanout_into_populated_index(ctx, ctx2):
    """recovery into an index that already holds entries: recovered keys override them, the others stay"""
    files = _files(12, 4)
    pre = [(NS, b"key-%06d" % i) for i in range(0, 800, 3)]
    oc = O.Index()
    for ns, k in pre:
        oc.put(ns, k, 5000, 77, 99)
    for fid in sorted(files):
        oc.put_segment(files[fid][1], 40, BASE, 20, 0, 1, fid)
    ix = IX.Index(ctx)
    ix.apply([L.IDX_PUT] * len(pre), [ns + k for ns, k in pre], [5000] * len(pre), [77] * len(pre), [99] * len(pre))
    IX.recover_from_wals(ix, _wals(files), contexts=[ctx2, ctx])
    _same_as_oracle(ix, oc)


@pytest.mark.parametrize("bad_at", [1, 3, 5])
def test_recover_fanout_stops_at_failing_wal(ctx, ctx2, bad_at):
    """a file whose hint and data WAL are both corrupted stops recovery: its puts before the bad fragment are
    applied, later fids are not, and the error is the serial path's"""
    files = _files(13, 6)
    fids = sorted(files)
    d, h = files[fids[bad_at]]
    files[fids[bad_at]] = (_corrupt(d, 0.5), _corrupt(h, 0.3))
    oc, stop = _oracle_recover(files)
    assert stop == fids[bad_at]
    ser = IX.Index(ctx)
    with pytest.raises(Exception) as e_ser:
        IX.recover_from_wals(ser, _wals(files))
    ix = IX.Index(ctx)
    with pytest.raises(Exception) as e_fan:
        IX.recover_from_wals(ix, _wals(files), contexts=[ctx, ctx2])
    assert type(e_fan.value) is type(e_ser.value) and str(e_fan.value) == str(e_ser.value)
    _same_as_oracle(ix, oc)
    assert ix.export() == ser.export()


def test_recover_fanout_many_files_three_contexts(ctx, ctx2, ctx3):
    """more files than the look-ahead window (2 per context): the workers wait for the ordered apply"""
    files = _files(14, 13, n=120, nkeys=200, vlens=(10, 300, 3000))
    oc, stop = _oracle_recover(files)
    assert stop is None
    ix = IX.Index(ctx)
    IX.recover_from_wals(ix, _wals(files), contexts=[ctx2, ctx3, ctx])
    _same_as_oracle(ix, oc)


def _compaction_setup(seed, nsrc, n=400):
    """nsrc source WALs recovered into the device index and the oracle's, then deletes / soft deletes / newer
    puts of some keys (so each source keeps only part of its rows)"""
    rng = random.Random(seed)
    srcs = []
    ix_entries = []
    oc = O.Index()
    for fid in range(1, nsrc + 1):
        payloads = [cases.rec(rng.randrange(0, 600), vlen=rng.choice((10, 300, 5000, 40000))) for _ in range(n)]
        data, _ = cases.wal_of(payloads)
        srcs.append((fid, data))
        oc.put_segment(data, 40, BASE, 20, 20, 0, fid)
        ix_entries.append((fid, data))
    ops, ks, fs = [], [], []
    for i in rng.sample(range(600), 120):
        op = rng.choice([L.IDX_DELETE, L.IDX_SOFT_DELETE, L.IDX_PUT])
        f = 900 if op == L.IDX_PUT else 0
        ops.append(op)
        ks.append(NS + b"key-%06d" % i)
        fs.append(f)
        oc.set(NS, b"key-%06d" % i, op, f, 4000 if f else 0, 10 if f else 0)
    return srcs, ix_entries, oc, (ops, ks, fs)


def _device_index(ctx, ix_entries, later):
    ix = IX.Index(ctx)
    for fid, data in ix_entries:
        ix.recover_segment(data, L.MODE_RECORD, fid, 40, BASE, 20, 20)
    ops, ks, fs = later
    ix.apply(ops, ks, fs, [4000 if f else 0 for f in fs], [10 if f else 0 for f in fs])
    return ix


def _oracle_compact(srcs, oc, dst_base):
    rd, rh = O.Writer(dst_base, dst_base), O.Writer(dst_base, dst_base)
    outs = []
    for fid, data in srcs:
        n = len(O.decode(data, 40, BASE, 20, 20, want_bytes=False).recs)
        keep, _ = oc.compact_filter(data, 40, BASE, 20, 20, fid, n)
        ec, _, nin, offs = O.compact_append(rd, rh, 77, data, 40, BASE, dst_base, 20, 20, keep)
        outs.append((ec, nin, offs, int(keep.sum())))
        if ec != 0:
            break
    return rd, rh, outs


@pytest.fixture
def snapshot_ctx(ctx2, ctx3):
    """sets BCW_OPT_FILTER_SNAPSHOT on ctx2 / ctx3 for one test: they then filter against a staging snapshot of the
    index, the path of a context on another device (the box has one GPU), and back to the direct filter after"""
    def use(on: bool):
        for c in (ctx2, ctx3):
            c.set_option(L.OPT_FILTER_SNAPSHOT, int(on))
    yield use
    use(False)


@pytest.mark.parametrize("nctx,snapshot", [(2, False), (3, False), (2, True), (3, True)])
def test_compact_fanout_vs_oracle(ctx, ctx2, ctx3, nctx, snapshot, snapshot_ctx):
    """5 sources appended to one dst / hint pair: the same bytes, offsets and kept counts as the oracle's serial
    doCompactionWork, and as the device's serial compact_one_wal_filtered loop; the contexts filter against the index
    itself (on its device) or against a staging snapshot of it (the path of another device)"""
    snapshot_ctx(snapshot)
    srcs, ents, oc, later = _compaction_setup(21, 5)
    rd, rh, outs = _oracle_compact(srcs, oc, BASE + 10)
    assert all(o[0] == 0 for o in outs)
    ix = _device_index(ctx, ents, later)
    dst, hint = W.WalFile(77, BASE + 10), W.WalFile(77, BASE + 10)
    res = IX.compact_wals_filtered(dst, hint, [W.load_wal(d, fid) for fid, d in srcs], ix,
                                   contexts=[ctx, ctx2, ctx3][:nctx])
    assert bytes(dst.data) == rd.data() and bytes(hint.data) == rh.data()
    assert len(res) == len(srcs)
    for (offs, kept), (ec, nin, roffs, rkept) in zip(res, outs):
        assert kept == rkept
        np.testing.assert_array_equal(offs[:nin], roffs[:nin])
    dst2, hint2 = W.WalFile(77, BASE + 10), W.WalFile(77, BASE + 10)
    ser = IX.compact_wals_filtered(dst2, hint2, [W.load_wal(d, fid) for fid, d in srcs], ix)
    assert bytes(dst2.data) == bytes(dst.data) and bytes(hint2.data) == bytes(hint.data)
    assert [k for _, k in ser] == [k for _, k in res]


@pytest.mark.parametrize("snapshot", [False, True])
def test_compact_fanout_source_error(ctx, ctx2, snapshot, snapshot_ctx):
    """a CRC failure in the third source: the sources before it and its rows before the bad fragment are
    appended, the error is the serial path's, the later sources are not appended (ctx2 filtering directly or
    against a snapshot)"""
    snapshot_ctx(snapshot)
    srcs, ents, oc, later = _compaction_setup(22, 5)
    fid, data = srcs[2]
    srcs[2] = (fid, _corrupt(data, 0.5))
    rd, rh, outs = _oracle_compact(srcs, oc, BASE)
    assert outs[-1][0] != 0 and len(outs) == 3
    ix = _device_index(ctx, ents, later)
    wals = [W.load_wal(d, f) for f, d in srcs]
    dst, hint = W.WalFile(77, BASE), W.WalFile(77, BASE)
    with pytest.raises(Exception) as e_fan:
        IX.compact_wals_filtered(dst, hint, wals, ix, contexts=[ctx2, ctx])
    dst2, hint2 = W.WalFile(77, BASE), W.WalFile(77, BASE)
    with pytest.raises(Exception) as e_ser:
        IX.compact_wals_filtered(dst2, hint2, wals, ix)
    assert type(e_fan.value) is type(e_ser.value)
    assert bytes(dst.data) == rd.data() == bytes(dst2.data)
    assert bytes(hint.data) == rh.data() == bytes(hint2.data)


def test_export_fids(ctx):
    """bcw_index_export_fids: the slice of the index pointing into the given fids"""
    ix = IX.Index(ctx)
    keys = [NS + b"k%05d" % i for i in range(3000)]
    fids = [i % 7 for i in range(3000)]
    ix.apply([L.IDX_PUT] * 3000, keys, fids, [100 + i for i in range(3000)], [9] * 3000)
    ix.apply([L.IDX_DELETE] * 10, keys[:10])
    want = {k: v for k, v in ix.export().items() if v[0] in (2, 5)}
    got = ix.export(fids=[5, 2, 5])
    assert got == want and len(got) > 800
