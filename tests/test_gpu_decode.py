"""GPU decode parity: libbcw.so on the MI355X against the CPU oracle, bit-exact.

Every comparison goes through the C-ABI (bcw_decode_segment / bcw_decode_fragments) on cuda:0; the ctx_path tests
run on a context of their own (k_chase + k_crc)."""
from __future__ import annotations

import random

import numpy as np
import pytest

import _oracle as O
import cases

pytestmark = pytest.mark.gpu


def gpu_decode(ctx, data, p):
    return ctx.decode(np.frombuffer(data, dtype=np.uint8), p["start_off"], p["base_time"], p["ns_size"],
                      p["etag_size"], p["mode"], with_frags=True)


def assert_parity(ctx, data, p, name=""):
    ref = O.decode(data, p["start_off"], p["base_time"], p["ns_size"], p["etag_size"], p["mode"])
    got = gpu_decode(ctx, data, p)
    res = got.result
    # segment level
    assert res.err_class == ref.err_class, (name, res.err_class, ref.err_class)
    if ref.err_class in (1, 2):
        assert res.err_frag == ref.err_frag, (name, res.err_frag, ref.err_frag)
        fr = ref.frags[ref.err_frag]
        assert res.err_file_off == fr["data_off"] - 7
    assert res.n_records == len(ref.recs), (name, res.n_records, len(ref.recs))
    # fragments parsed by the iterator
    nf = len(ref.frags)
    gf = got.frags
    if nf:
        assert len(gf["data_off"]) >= nf
        for col in ("data_off", "len", "stored_crc", "type"):
            np.testing.assert_array_equal(gf[col][:nf], ref.frags[col], err_msg=f"{name}: frag {col}")
        np.testing.assert_array_equal(gf["crc_ok"][:nf], ref.frags["crc_ok"], err_msg=f"{name}: frag crc_ok")
    # records
    t = got.table
    r = ref.recs
    for col in ("foff", "size", "first_frag", "emit_frag", "status", "hdr_size", "flags", "etag_off", "expire"):
        np.testing.assert_array_equal(t[col].astype(np.uint64), r[col].astype(np.uint64), err_msg=f"{name}: {col}")
    if p["mode"] == 0:
        for col in ("key_len", "val_len", "meta_len"):
            np.testing.assert_array_equal(t[col].astype(np.uint64), r[col] & 0xFFFFFFFF, err_msg=f"{name}: {col}")
    else:
        np.testing.assert_array_equal(t["key_len"].astype(np.uint64), r["key_len"] & 0xFFFFFFFF)
        np.testing.assert_array_equal(t["aux0"], r["val_len"], err_msg=f"{name}: hint off")
        np.testing.assert_array_equal(t["aux1"], r["meta_len"], err_msg=f"{name}: hint size")
    # payload bytes of every record
    for i in range(len(r)):
        assert got.record_bytes(i) == ref.payloads[i], (name, i)
    bad = np.nonzero(r["status"] != 0)[0]
    assert res.first_bad_record == (int(bad[0]) if len(bad) else -1)
    return got, ref


@pytest.mark.parametrize("name", list(cases.ALL))
def test_cases(ctx_path, name):
    data, p = cases.ALL[name]()
    assert_parity(ctx_path, data, p, name)


def test_synth_config_a_fragment(ctx):
    """config A shape (64 MiB would take the oracle ~0.3 s; use 8 MiB here)."""
    data = O.synth(8 << 20, 0, 0x5EED)
    got, ref = assert_parity(ctx, data, cases.params(), "synth8m")
    assert got.result.err_class == 0 and (got.table["status"] == 0).all()


def test_synth_zipf(ctx_path):
    data = O.synth(24 << 20, 0, 42, value_mode=1)
    assert_parity(ctx_path, data, cases.params(), "zipf24m")


@pytest.mark.parametrize("seed", range(12))
def test_corruption_fuzz(ctx_path, seed):
    """random bit flips: same first failing fragment, error class and delivered records."""
    rng = random.Random(seed)
    base, p = cases.case_zipf(120, seed) if seed % 2 else cases.case_config_shape(120, 2000)
    data = cases.corrupt(base, rng, nflips=1 + seed % 3)
    assert_parity(ctx_path, data, p, f"fuzz{seed}")


@pytest.mark.parametrize("cut", [0, 1, 6, 7, 39, 40, 41, 47, 48, 100, 32807, 32808, 32809])
def test_truncations(ctx_path, cut):
    data, p = cases.case_config_shape(20, 3000)
    assert_parity(ctx_path, data[:cut] if cut < len(data) else data, p, f"cut{cut}")


def test_empty_and_small(ctx_path):
    for data in (b"", bytes(40), bytes(46), bytes(47)):
        assert_parity(ctx_path, data, cases.params(), f"small{len(data)}")


@pytest.mark.parametrize("vlen,mib,mode", [(10, 24, 0), (0, 24, 0), (300, 16, 0)])
def test_dense_fragments_at_scale(ctx_path, vlen, mib, mode):
    """~230 fragments per block (hint-WAL density) over many workgroups: exercises the fragment-table
    retry (first capacity guess too small) and the multi-window ring of k_crc at full occupancy."""
    seg = O.synth(mib << 20, 0, 11 + vlen, 20, 100, vlen, 0)
    assert_parity(ctx_path, seg, cases.params(), f"dense vlen={vlen}")


def test_hint_wal_at_scale(ctx):
    """a hint WAL rebuilt from a 20 MiB data WAL, decoded in hint mode (IterateHint)."""
    data = O.synth(20 << 20, 0, 5, 20, 100, 4096, 1)
    ec, _, _, hint = O.hint_by_wal(data, 3, 40, 1_700_000_000, 20, 20)
    assert ec == 0
    assert_parity(ctx, hint, cases.params(mode=1), "hint at scale")


def _sweep_segment(step: int, count: int, base_len: int, payload_kind: str):
    """raw payloads whose lengths grow by `step` bytes: the fragment ends (and with them the check word J, the 7-byte
    header gap and the next fragment's start) walk through every byte offset of the 16 B lane pieces and the 1 KiB
    chunks of the stream verify (bcw_decode.hip stream_verify), including J straddling two pieces, two lanes or two
    chunks, headers split across a chunk boundary and several fragment ends in one chunk"""
    rng = random.Random(base_len * 31 + step)
    ps = []
    for k in range(count):
        n = base_len + k * step
        ps.append(bytes(rng.getrandbits(8) for _ in range(n)) if payload_kind == "rand" else bytes(n))
    data, offs = cases.wal_of(ps)
    return data, offs


@pytest.mark.parametrize("step,count,base_len,kind", [(1, 1100, 1, "rand"), (1, 1100, 1000, "rand"),
                                                      (3, 700, 3000, "rand"), (1, 600, 0, "zero"),
                                                      (17, 400, 50, "rand")])
def test_stream_verify_geometry_sweep(ctx_path, step, count, base_len, kind):
    """every fragment-end offset within a chunk, clean: all verdicts and rows equal the oracle's (the records are
    raw payloads, so RecordFromBytes reports them invalid exactly as the reference does)"""
    data, _ = _sweep_segment(step, count, base_len, kind)
    assert_parity(ctx_path, data, cases.params(), f"sweep{step}/{base_len}/{kind}")


@pytest.mark.parametrize("where", ["last_data", "first_data", "crc_byte", "len_byte"])
def test_stream_verify_geometry_corrupt(ctx_path, where):
    """a corrupted byte at a fragment edge (its last data byte, its first data byte, a stored CRC byte, a length byte)
    of every 37th fragment of the sweep in turn: the first failing fragment and the records before it equal the
    oracle's"""
    data, offs = _sweep_segment(1, 1100, 1, "rand")
    ref = O.decode(data, 40, cases.BASE, 20, 20, 0)
    for f in range(5, len(ref.frags), 37):
        fr = ref.frags[f]
        d0, ln = int(fr["data_off"]), int(fr["len"])
        if ln == 0:
            continue
        pos = {"last_data": d0 + ln - 1, "first_data": d0, "crc_byte": d0 - 7 + (f % 4),
               "len_byte": d0 - 3}[where]
        bad = bytearray(data)
        bad[pos] ^= 0x41
        assert_parity(ctx_path, bytes(bad), cases.params(), f"corrupt {where} frag {f}")


@pytest.mark.parametrize("size,mode", [(48 << 20, 0), (24 << 20, 1), (300 << 10, 0), (5000, 0)])
def test_xcd_balance_split_changes_no_result(size, mode):
    """the per-XCD split of k_crc's stream (XBal, BCW_OPT_XCD_BALANCE): six decodes in a row with the weights adapting
    after each, then with equal bytes per workgroup, then again with the weights -- every decode bit-exact against the
    oracle (sizes from a few hundred boundaries per block to several blocks per wave); other values are refused"""
    from bitcaskdb_amd import Context
    from bitcaskdb_amd import _lib as L
    seg = O.synth(size, 0, 5 + size % 97, value_mode=mode) if size > 10000 else cases.wal_of(
        [cases.rec(i, vlen=100 + i) for i in range(30)])[0]
    c = Context(0)
    try:
        for on in (1, 1, 1, 1, 1, 1, 0, 1):
            c.set_option(L.OPT_XCD_BALANCE, on)
            assert_parity(c, seg, cases.params(), f"xbal={on} size={size}")
        with pytest.raises(ValueError):
            c.set_option(L.OPT_XCD_BALANCE, 3)
    finally:
        c.close()
