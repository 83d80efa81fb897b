"""Full-table parity check of one device decode against the CPU oracle (test infrastructure): every fragment
column, every record column, the error outcome and a 64-bit hash of every record's payload gathered from the
device fragment table (oracle/bcw_oracle.c oc_gather_payload_hashes) against the oracle's own payloads. Shared by
tests/test_gpu_fullsize.py and the rank processes of tests/test_gpu_multirank.py (tests/_rank_decode.py)."""
from __future__ import annotations

import numpy as np

import _oracle as O
from bitcaskdb_amd import _lib as L


def full_parity(ctx, data, p, name):
    ref = O.decode(data, p["start_off"], p["base_time"], p["ns_size"], p["etag_size"], p["mode"], want_bytes=False,
                   want_hashes=True)
    seg = np.frombuffer(data, dtype=np.uint8)
    got = ctx.decode(seg, p["start_off"], p["base_time"], p["ns_size"], p["etag_size"], p["mode"], with_frags=True)
    res = got.result
    assert res.err_class == ref.err_class, (name, res.err_class, ref.err_class)
    if ref.err_class in (L.ERR_CRC, L.ERR_TYPE):
        assert res.err_frag == ref.err_frag, (name, res.err_frag, ref.err_frag)
    assert res.n_records == len(ref.recs), (name, res.n_records, len(ref.recs))
    nf = len(ref.frags)
    gf = got.frags
    assert len(gf["data_off"]) >= nf
    for col in ("data_off", "len", "stored_crc", "type", "crc_ok"):
        np.testing.assert_array_equal(gf[col][:nf], ref.frags[col], err_msg=f"{name}: frag {col}")
    t, r = got.table, ref.recs
    for col in ("foff", "size", "first_frag", "emit_frag", "status", "hdr_size", "flags", "etag_off", "expire"):
        np.testing.assert_array_equal(t[col].astype(np.uint64), r[col].astype(np.uint64), err_msg=f"{name}: {col}")
    if p["mode"] == 0:
        for col in ("key_len", "val_len", "meta_len"):
            np.testing.assert_array_equal(t[col].astype(np.uint64), r[col] & 0xFFFFFFFF, err_msg=f"{name}: {col}")
    else:
        np.testing.assert_array_equal(t["aux0"], r["val_len"], err_msg=f"{name}: hint off")
        np.testing.assert_array_equal(t["aux1"], r["meta_len"], err_msg=f"{name}: hint size")
    h = O.gather_payload_hashes(seg, gf, t)
    bad = np.nonzero(h != ref.hashes)[0]
    assert bad.size == 0, f"{name}: {bad.size} payloads differ, first at record {bad[:1]}"
    st = np.nonzero(r["status"] != 0)[0]
    assert res.first_bad_record == (int(st[0]) if len(st) else -1)
    return got, ref
