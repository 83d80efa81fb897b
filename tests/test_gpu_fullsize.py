"""Full-size GPU parity: the benchmark configurations themselves (BASELINE.json configs A, B, C and E),
decoded / encoded on the MI355X through the C-ABI and compared with the CPU oracle column by column.

At these sizes every k_crc wave owns many 32 KiB blocks (config B: ~10.7 per wave), the k_chase
look-back crosses many workgroups and the last-workgroup scans run over all 256 aggregates -- the
regimes the small parity tests never reach. Record payloads are compared through a 64-bit hash of the
bytes gathered from the device fragment table (oracle/bcw_oracle.c oc_gather_payload_hashes) against
the same hash of the oracle's own payloads."""
from __future__ import annotations

import numpy as np
import pytest

import _oracle as O
import cases
from _parity import full_parity
from bitcaskdb_amd import _lib as L

pytestmark = pytest.mark.gpu
BASE = cases.BASE


def test_config_a_64mib(ctx):
    """config A: one 64 MiB segment, 100 B keys / 4 KiB values (15,866 records)."""
    data = O.synth(64 << 20, 0, 0x5EED)
    got, _ = full_parity(ctx, data, cases.params(), "A")
    assert got.n_records > 15000 and got.result.err_class == 0


@pytest.fixture(scope="module")
def config_b():
    return O.synth(1 << 30, 0, 42)


def test_config_b_1gib(ctx, config_b):
    """config B: 1 GiB, 4 KiB values (~254 k records, 32,769 blocks, ~10.7 blocks per k_crc wave)."""
    got, ref = full_parity(ctx, config_b, cases.params(), "B")
    assert got.n_records > 250000 and got.result.err_class == 0
    assert got.result.n_blocks == (len(config_b) - 40 + 32767) // 32768


@pytest.mark.parametrize("where", [0.5, 0.97, 0.9999])
def test_config_b_corruption(ctx, config_b, where):
    """one flipped byte in the middle / last workgroups' ranges of a 1 GiB segment: the same first failing
    fragment, error class, delivered records and their payloads."""
    bad = bytearray(config_b)
    pos = int(len(bad) * where)
    bad[pos] ^= 0x5A
    got, ref = full_parity(ctx, bytes(bad), cases.params(), f"B flip@{pos}")
    assert got.result.err_class in (L.ERR_CRC, L.ERR_TYPE)
    assert 0 < got.n_records < len(ref.recs) + 1 and got.n_records < 260000


def test_config_c_1gib_zipf(ctx):
    """config C: 1 GiB, Zipf(1.1) 128 B - 64 KiB values (spanning records, zero-length Firsts, pads)."""
    data = O.synth(1 << 30, 0, 42, value_mode=1)
    got, ref = full_parity(ctx, data, cases.params(), "C")
    assert got.result.err_class == 0 and got.n_records > 100000


def test_dense_fragments_256mib(ctx):
    """~230 fragments per block over 256 MiB (1.9 M fragments, several blocks per k_crc wave, a
    fragment-table retry)."""
    data = O.synth(256 << 20, 0, 21, 20, 100, 10, 0)
    got, _ = full_parity(ctx, data, cases.params(), "dense256")
    assert got.result.err_class == 0


def test_hint_wal_fullsize(ctx):
    """the hint WAL of a 1 GiB config-C data WAL, decoded in hint mode (IterateHint)."""
    data = O.synth(1 << 30, 0, 43, value_mode=1)
    ec, _, _, hint = O.hint_by_wal(data, 3, 40, BASE, 20, 20)
    assert ec == 0
    full_parity(ctx, hint, cases.params(mode=1), "hint-C")


def test_config_e_compaction_200k(ctx):
    """config E shape at 200,000 records (845 MB source): compaction re-encode and hint rebuild,
    dst WAL + hint WAL bytes and the returned offsets bit-exact against oc_compact_append /
    oc_hint_by_wal; a dst baseTime below the source's re-bases every expire-less record identically."""
    n = 200000
    src = O.synth(1 << 40, n, 42)
    rng = np.random.default_rng(3)
    keep = (rng.random(n) < 0.9).astype(np.uint8)
    dst, hint = O.Writer(BASE, BASE), O.Writer(BASE, BASE)
    ec, er, nin, offs = O.compact_append(dst, hint, 9, src, 40, BASE, BASE, 20, 20, keep)
    assert ec == 0 and nin == n
    res, wal, hb, goffs = ctx.encode(src, L.ENC_COMPACT, 40, BASE, 9, 40, 40, 20, 20, keep)
    assert res.err_class == 0 and res.n_in == n and res.n_written == int(keep.sum())
    assert wal == dst.data()[40:], "dst WAL differs"
    assert hb == hint.data()[40:], "hint WAL differs"
    np.testing.assert_array_equal(goffs[:n], offs[:n])
    # hint rebuild of the same source (NewHintByWal)
    ec2, _, nin2, ref_hint = O.hint_by_wal(src, 5, 40, BASE, 20, 20)
    res2, _, hb2, _ = ctx.encode(src, L.ENC_HINT, 40, BASE, 5, 40, 40, 20, 20)
    assert res2.err_class == ec2 == 0 and res2.n_in == nin2 == n
    assert hb2 == ref_hint[40:], "hint-by-wal bytes differ"


@pytest.fixture
def lookback_ctx():
    """a context whose k_chase takes the decoupled look-back at every size (BCW_OPT_CHASE_DIRECT 0)"""
    from bitcaskdb_amd import Context
    c = Context(0)
    c.set_option(L.OPT_CHASE_DIRECT, 0)
    yield c
    c.close()


@pytest.mark.parametrize("where", [None, 0.3, 0.999])
def test_chase_lookback_branch_256mib(lookback_ctx, where):
    """k_chase's decoupled look-back (the > 1024-workgroup branch, bcw_decode.hip k_chase) forced on a 256 MiB
    config-B shape (128 workgroups chaining inclusive prefixes), clean and with a flipped byte: every column
    equals the oracle's."""
    data = bytearray(O.synth(256 << 20, 0, 44))
    if where is not None:
        data[int(len(data) * where)] ^= 0x11
    got, ref = full_parity(lookback_ctx, bytes(data), cases.params(), f"lookback flip@{where}")
    assert (got.result.err_class == 0) == (where is None)


def test_chase_lookback_config_c(lookback_ctx):
    """the look-back over config C's divergent per-block fragment counts (256 MiB Zipf)"""
    data = O.synth(256 << 20, 0, 45, value_mode=1)
    got, _ = full_parity(lookback_ctx, data, cases.params(), "lookback C")
    assert got.result.err_class == 0


@pytest.mark.parametrize("flip", [False, True])
def test_segment_beyond_2gib(ctx, flip):
    """a 2.25 GiB config-B-shape segment: 1,153 k_chase workgroups, past the direct-sum limit (1024), so the
    product's default path takes the decoupled look-back; with a flipped byte beyond workgroup 1024 (past
    2 GiB) the first failing fragment, delivered records and payloads still equal the oracle's."""
    data = O.synth(9 << 28, 0, 46)
    nwg = ((len(data) - 40 + 32767) // 32768 + 63) // 64
    assert nwg > 1024
    if flip:
        b = bytearray(data)
        pos = (2 << 30) + 40 + 12345 * 7
        assert (pos - 40) // 32768 // 64 >= 1024
        b[pos] ^= 0x40
        data = bytes(b)
    got, ref = full_parity(ctx, data, cases.params(), f"2.25GiB flip={flip}")
    assert (got.result.err_class != 0) == flip
    assert got.n_records > 500000


def test_config_e_compaction_2m_rebase(ctx):
    """config-E-scale compaction: 2,000,000 records carrying expires (a third with etags, every 17th a
    tombstone), a random keep mask (70 %), and a dst baseTime 500,000 s below the source's, so every kept
    record's expire delta grows and its varint lengthens (Record.Encode, record.go:57-138): the dst WAL, the
    hint WAL and every returned offset equal oc_compact_append's (compaction.go:294-327)."""
    n = 2_000_000
    src = O.synth(1 << 40, n, 77, 20, 24, 0, 2)
    rng = np.random.default_rng(5)
    keep = (rng.random(n) < 0.7).astype(np.uint8)
    dst_base = BASE - 500_000
    dst, hint = O.Writer(dst_base, dst_base), O.Writer(dst_base, dst_base)
    ec, er, nin, offs = O.compact_append(dst, hint, 11, src, 40, BASE, dst_base, 20, 20, keep)
    assert ec == 0 and nin == n
    res, wal, hb, goffs = ctx.encode(src, L.ENC_COMPACT, 40, dst_base, 11, 40, 40, 20, 20, keep)
    assert res.err_class == 0 and res.n_in == n and res.n_written == int(keep.sum())
    ref_wal, ref_hint = dst.data()[40:], hint.data()[40:]
    assert len(wal) == len(ref_wal) and len(hb) == len(ref_hint)
    w, rw = np.frombuffer(wal, np.uint8), np.frombuffer(ref_wal, np.uint8)
    bad = np.nonzero(w != rw)[0]
    assert bad.size == 0, f"dst WAL differs from byte {bad[:1]}"
    assert hb == ref_hint, "hint WAL differs"
    np.testing.assert_array_equal(goffs[:n], offs[:n])


@pytest.mark.timeout(600)
def test_config_e_full_size_realistic_chunks(ctx):
    """config E at its full size, the realistic compaction: 10,000,000 config-E records (NsSize
    20, 100 B keys, 4 KiB values) in ten source WALs of 1,000,000, each re-encoded with a seeded 70 % keep mask
    against a dst baseTime 500,000 s below the source's and appended at the running wal_pos / hint_pos (one dst WAL
    of ~29.6 GB, one hint WAL of ~0.9 GB, as doCompactionWork's loop appends source after source,
    compaction.go:201-211). Every chunk's appended dst bytes, hint bytes and returned offsets equal
    oc_compact_append's on writers opened at the same positions (compaction.go:294-327, hint.go:32-48). The device
    encodes run in order; the oracle's checks run on 4 host threads beside them (ctypes releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor

    dst_base = BASE - 500_000

    def check(k, src, keep, wal_pos, hint_pos, res, wal, hb, goffs):
        dst, hint = O.Writer(dst_base, dst_base, at=wal_pos), O.Writer(dst_base, dst_base, at=hint_pos)
        ec, er, nin, offs = O.compact_append(dst, hint, 31, src, 40, BASE, dst_base, 20, 20, keep)
        assert ec == 0 and nin == 1_000_000, (k, ec, er, nin)
        assert res.n_in == nin and res.n_written == int(keep.sum()), k
        assert (res.wal_end, res.hint_end) == (dst.size(), hint.size()), k
        ref = dst.data()
        assert len(wal) == len(ref), (k, len(wal), len(ref))
        bad = np.nonzero(np.frombuffer(wal, np.uint8) != np.frombuffer(ref, np.uint8))[0]
        assert bad.size == 0, f"chunk {k}: dst WAL differs at file offset {wal_pos + int(bad[0])}"
        assert hb == hint.data(), f"chunk {k}: hint WAL differs"
        np.testing.assert_array_equal(goffs[:nin], offs[:nin])
        return nin, int(keep.sum())

    wal_pos = hint_pos = 40
    rng = np.random.default_rng(2026)
    futs = []
    with ThreadPoolExecutor(4) as pool:
        for k in range(10):
            src = np.frombuffer(O.synth(1 << 40, 1_000_000, 900 + k, 20, 100, 4096, 0, BASE), dtype=np.uint8)
            keep = (rng.random(1_000_000) < 0.7).astype(np.uint8)
            res, wal, hb, goffs = ctx.encode(src, L.ENC_COMPACT, 40, dst_base, 31, wal_pos, hint_pos, 20, 20, keep)
            assert res.err_class == 0, (k, res.err_class)
            futs.append(pool.submit(check, k, src, keep, wal_pos, hint_pos, res, wal, hb, goffs))
            wal_pos, hint_pos = res.wal_end, res.hint_end
            del src, wal, hb
            if len(futs) >= 4:  # (at most 4 chunks' buffers alive at once)
                futs[-4].result()
        done = [f.result() for f in futs]
    assert sum(d[0] for d in done) == 10_000_000 and wal_pos > 29_000_000_000


def test_config_b_second_context(ctx_path, config_b):
    """config B decoded by a second context (its own scratch and tables): every column equals the oracle's"""
    got, _ = full_parity(ctx_path, config_b, cases.params(), "B second context")
    assert got.result.err_class == 0 and got.n_records > 250000


@pytest.mark.parametrize("where", [0.0001, 0.5])
def test_config_c_corruption(ctx, where):
    """config C with a flipped byte near the start (workgroup 0) and in the middle: the stream verify's masked
    chunks decide the same first failing fragment as the oracle."""
    data = bytearray(O.synth(1 << 30, 0, 42, value_mode=1))
    data[int(len(data) * where)] ^= 0x24
    got, ref = full_parity(ctx, bytes(data), cases.params(), f"C flip@{where}")
    assert got.result.err_class in (L.ERR_CRC, L.ERR_TYPE)


@pytest.mark.parametrize("direct", [True, False])
def test_forced_wait_abort(direct):
    """a k_chase predecessor wait that gives up (BCW_OPT_TEST_ABORT_WAIT makes workgroup 5 of a 64 MiB segment give
    up at its first step, as a wait past its 200 ms bound would; its bases are then computed from zeroed words):
    the decode reports BCW_ERR_INTERNAL at the wait site with no row, k_crc reads no fragment over the bad bases,
    and the next decode on the same context is bit-exact against the oracle (wal_iterator.go:44,79-82: no partial
    result is ever delivered as valid)."""
    from bitcaskdb_amd import Context
    c = Context(0)
    try:
        if not direct:
            c.set_option(L.OPT_CHASE_DIRECT, 0)
        data = O.synth(64 << 20, 0, 46)
        p = cases.params()
        seg = np.frombuffer(data, dtype=np.uint8)
        c.set_option(L.OPT_TEST_ABORT_WAIT, 6)
        got = c.decode(seg, p["start_off"], p["base_time"], p["ns_size"], p["etag_size"], p["mode"], with_frags=True)
        r = got.result
        assert r.err_class == L.ERR_INTERNAL
        # the aborted decode's fragment table and verdicts are stale: the export delivers no row
        assert all(len(v) == 0 for v in got.frags.values())
        assert r.err_frag == 9 if direct else r.err_frag in (10, 11)  # the site (the largest one that gave up)
        assert r.n_records == 0 and r.n_records_total == 0 and r.retry_frag_capacity == 0
        assert r.first_bad_record == -1 and r.err_file_off == 0
        # one-shot: the next decode on the same context is exact
        full_parity(c, data, p, "after abort")
        # a compaction whose source decode gives up applies nothing (k_enc_prep: BCW_ENC_ERR_TABLE, 0 rows in)
        if direct:
            c.set_option(L.OPT_TEST_ABORT_WAIT, 6)
            res, wal, hb, _ = c.encode(data, L.ENC_COMPACT, 40, BASE, 9, 40, 40, 20, 20,
                                       np.ones(got.result.n_blocks * 8, dtype=np.uint8))
            assert res.err_class == L.ENC_ERR_TABLE and res.n_in == 0 and res.n_written == 0
            assert wal == b"" and hb == b""
            # ... and the wrappers raise instead of returning an empty output as a success: a compaction
            # that wrote nothing must not let its caller drop the source, an empty hint must not look valid
            from bitcaskdb_amd import wal as W
            src = W.load_wal(data, fid=4)
            for call in (lambda: W.compact_one_wal(W.WalFile(9, BASE), W.WalFile(9, BASE), src,
                                                    np.ones(got.result.n_blocks * 8, dtype=np.uint8), ctx=c),
                         lambda: W.new_hint_by_wal(src, ctx=c)):
                c.set_option(L.OPT_TEST_ABORT_WAIT, 6)
                with pytest.raises(RuntimeError):
                    call()
        c.sync()
    finally:
        c.close()


@pytest.mark.gpu
def test_abort_hook_needs_opt_in(monkeypatch):
    """BCW_OPT_TEST_ABORT_WAIT is a fault-injection hook: refused (BCW_E_INVAL) unless BCW_TEST_HOOKS=1"""
    from bitcaskdb_amd import Context
    c = Context(0)
    try:
        monkeypatch.delenv("BCW_TEST_HOOKS", raising=False)
        assert L.lib.bcw_ctx_set_option(c.handle, L.OPT_TEST_ABORT_WAIT, 6) == L.E_INVAL
        monkeypatch.setenv("BCW_TEST_HOOKS", "1")
        assert L.lib.bcw_ctx_set_option(c.handle, L.OPT_TEST_ABORT_WAIT, 0) == 0
    finally:
        c.close()
