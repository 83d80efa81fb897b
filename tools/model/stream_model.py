"""CPU model of k_crc's stream verify (bcw_decode.hip stream_verify), lane by lane, to check its arithmetic against
the oracle's per-fragment verdicts. Test infrastructure only (slow: pure Python)."""
from __future__ import annotations

import os
import sys

import numpy as np

POLY = 0x82F63B78
T = []
for b in range(256):
    c = b
    for _ in range(8):
        c = (c >> 1) ^ (POLY if c & 1 else 0)
    T.append(c)


def crc_raw(data: bytes, s: int = 0) -> int:
    for b in data:
        s = (s >> 8) ^ T[(s ^ b) & 0xFF]
    return s


_OPS = {}


def shift(x: int, n: int) -> int:  # A_{8n}, by basis images (memoized per n)
    img = _OPS.get(n)
    if img is None:
        img = _OPS[n] = [crc_raw(bytes(n), 1 << i) for i in range(32)]
    r = 0
    i = 0
    while x:
        if x & 1:
            r ^= img[i]
        x >>= 1
        i += 1
    return r


def rotl(x, r):
    return ((x << r) | (x >> (32 - r))) & 0xFFFFFFFF


def check_word(stored: int, ln: int) -> int:
    u = rotl((stored - 0xA282EAD8) & 0xFFFFFFFF, 15)
    return (~u & 0xFFFFFFFF) ^ shift(0xFFFFFFFF, ln)


PIECE, CHUNK = 16, 1024
PW = PIECE // 4


def sbfe(v, j):
    return 0xFFFFFFFF if (v >> j) & 1 else 0


def mask_chunk(w, pa, pb, pc, J, lane):
    """bcw_decode.hip mask_chunk: w (8 words of lane `lane`), chunk-relative pa, pb, pc"""
    u = PW * lane
    ga, gb, gc = pa >> 2, (pb + 7) >> 2, pc >> 2
    lo1, hi1, lo2 = min(max(ga - u, 0), PW), min(max(gb - u, 0), PW), min(max(gc - u, 0), PW)
    keep = (((1 << hi1) - 1) & ~((1 << lo1) - 1)) | (0xFF << lo2)
    x = [w[j] & sbfe(keep, j) for j in range(PW)]

    def fix(wi, f):
        L, jj = wi // PW, wi % PW
        if lane == L:
            x[jj] = f(x[jj]) & 0xFFFFFFFF
    if 0 < pa < CHUNK and pa & 3:
        m = (0xFFFFFFFF << (8 * (pa & 3))) & 0xFFFFFFFF
        fix(pa >> 2, lambda v: v & m)
    r = pb & 3
    if 0 <= pb < CHUNK:
        m, jl = (1 << (8 * r)) - 1, (J << (8 * r)) & 0xFFFFFFFF
        fix(pb >> 2, lambda v: (v & m) | jl)
    if r and -4 <= pb < CHUNK - 4:
        jh = J >> (32 - 8 * r)
        fix((pb >> 2) + 1, lambda v: jh)
    if 0 < pc < CHUNK and pc & 3:
        m = (0xFFFFFFFF << (8 * (pc & 3))) & 0xFFFFFFFF
        fix(pc >> 2, lambda v: v & m)
    return x


def mask_gap(w, pb, J, lane):
    """bcw_decode.hip mask_gap (data on both sides of [pb, pb + 7))"""
    x = list(w)

    def fix(wi, f):
        L, jj = wi // PW, wi % PW
        if lane == L:
            x[jj] = f(x[jj]) & 0xFFFFFFFF
    r = pb & 3
    wb = pb >> 2
    lo, jl = (1 << (8 * r)) - 1, (J << (8 * r)) & 0xFFFFFFFF
    fix(wb, lambda v: (v & lo) | jl)
    if r == 0:
        fix(wb + 1, lambda v: v & 0xFF000000)
    else:
        jh = J >> (32 - 8 * r)
        fix(wb + 1, lambda v: jh)
        if r >= 2:
            keep = ~((1 << (8 * (r - 1))) - 1) & 0xFFFFFFFF
            fix(wb + 2, lambda v: v & keep)
    return x


GAP_CHECKS = [0]


def words_to_bytes(w):
    return b"".join(int(v).to_bytes(4, "little") for v in w)


def verify(seg: bytes, frags) -> list:
    """frags: list of (gs, ge, J) in order; returns verdicts (the kernel's arithmetic, one lane at a time)"""
    nfr = len(frags)
    FAR = 1 << 62
    geo = lambda i: frags[i] if i < nfr else (FAR, FAR, 0)
    seglen = len(seg)
    i = 0
    fc, fn = geo(0), geo(1)
    H = [0] * 64
    out = [None] * nfr
    SH = CHUNK - PIECE

    def piece_words(C0, l):
        o = C0 + PIECE * l
        b = bytes(seg[o:o + PIECE]) if o < seglen else b""
        b = b + bytes(PIECE - len(b))
        return [int.from_bytes(b[4 * j:4 * j + 4], "little") for j in range(PW)]

    def process(C0):
        nonlocal i, fc, fn, H
        C1 = C0 + CHUNK
        W = [piece_words(C0, l) for l in range(64)]
        if fc[0] <= C0 and fc[1] >= C1:
            H = [shift(crc_raw(words_to_bytes(W[l]), H[l]), SH) for l in range(64)]
            return
        while True:
            if fc[0] >= C1:
                return
            closes = fc[1] + 4 <= C1
            next_in = closes and fn[0] < C1 and fn[1] >= C1

            def rel(p):
                r = p - C0
                return -64 if r < -64 else (4096 if r > 4096 else r)
            pb = rel(fc[1])
            X = [mask_chunk(W[l], rel(fc[0]), pb, rel(fn[0]) if next_in else 4096, fc[2], l) for l in range(64)]
            if next_in and rel(fc[0]) <= 0 and fn[0] - fc[1] == 7:
                Y = [mask_gap(W[l], pb, fc[2], l) for l in range(64)]
                assert X == Y, (pb, rel(fc[0]))
                GAP_CHECKS[0] += 1
            if not closes:
                H = [shift(crc_raw(words_to_bytes(X[l]), H[l]), SH) for l in range(64)]
                return
            e = pb + 4
            Lf, K = e // PIECE, ((e % PIECE) + 3) >> 2
            Tt, newH = 0, []
            for l in range(64):
                xb = words_to_bytes(X[l])
                s8 = shift(crc_raw(xb, H[l]), SH)
                if l < Lf or (l == Lf and K == PW):
                    A = s8
                elif l == Lf and K > 0:
                    A = shift(crc_raw(xb[:4 * K], H[l]), 4 * (PW - K) + SH)
                else:
                    A = shift(H[l], PIECE + SH)
                Tt ^= shift(A, PIECE * (63 - l))
                newH.append(s8 ^ A)
            out[i] = 1 if Tt == 0 else 0
            H = newH
            i += 1
            fc, fn = fn, geo(i + 1)
            if next_in:
                return

    ge_last = frags[-1][1]
    c_first = frags[0][0] // CHUNK
    c_end = (ge_last + 4 + CHUNK - 1) // CHUNK
    for c in range(c_first, c_end):
        process(c * CHUNK)
    return out


def random_check(seed: int, nbytes: int, corrupt: int = 0):
    """a synthetic segment of small mixed records (the oracle's writer and decoder), optionally with corrupted bytes"""
    import random
    import _oracle as O
    rnd = random.Random(seed)
    w = O.Writer(1, 1)
    while w.size() < nbytes:
        n = rnd.choice([0, 1, 2, 3, 4, 5, 9, 20, 25, 30, 60, 200, 1000]) if rnd.random() < 0.97 else rnd.choice([3000, 40000])
        w.write(bytes(rnd.getrandbits(8) for _ in range(n)))
    seg = bytearray(w.data())
    for _ in range(corrupt):
        seg[rnd.randrange(40, len(seg))] ^= 1 << rnd.randrange(8)
    d = O.decode(bytes(seg), 40, 1, 20, 20)
    fr = [(int(f["data_off"]), int(f["data_off"]) + int(f["len"]), check_word(int(f["stored_crc"]), int(f["len"])))
          for f in d.frags]
    got = verify(bytes(seg), fr)
    want = [int(f["crc_ok"]) for f in d.frags]
    bad = [k for k in range(len(fr)) if got[k] != want[k]]
    print(f"random seed {seed}: {len(fr)} fragments, {sum(want)} ok; mismatches: {bad[:20]}")
    return not bad


if __name__ == "__main__":
    import json
    if sys.argv[1] == "random":
        sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
        ok = all(random_check(s, int(sys.argv[3]), int(sys.argv[4])) for s in range(int(sys.argv[2])))
        print("mask_gap cases checked:", GAP_CHECKS[0])
        sys.exit(0 if ok else 1)
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
    path = sys.argv[1]
    exp = json.load(open(path))
    seg = open(path[:-5] + ".wal", "rb").read()
    fr = [(f["data_off"], f["data_off"] + f["len"], check_word(f["stored_crc"], f["len"])) for f in exp["frags"]]
    got = verify(seg, fr)
    want = [f["crc_ok"] for f in exp["frags"]]
    bad = [k for k in range(len(fr)) if got[k] != want[k]]
    print(os.path.basename(path), len(fr), "fragments; mismatches:", bad[:20])
