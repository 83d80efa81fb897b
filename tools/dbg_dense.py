"""debug: dense vlen=0 decode vs oracle, the mismatching rows"""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import _oracle as O
import cases
from bitcaskdb_amd import Context

seg = O.synth(24 << 20, 0, 11, 20, 100, 0, 0)
p = cases.params()
ref = O.decode(seg, p["start_off"], p["base_time"], p["ns_size"], p["etag_size"], p["mode"])
ctx = Context(0)
for rep in range(2):
    got = ctx.decode(np.frombuffer(seg, dtype=np.uint8), p["start_off"], p["base_time"], p["ns_size"], p["etag_size"],
                     p["mode"], with_frags=True)
    t, r = got.table, ref.recs
    bad = np.nonzero(t["foff"].astype(np.uint64) != r["foff"].astype(np.uint64))[0]
    print("rep", rep, "n", len(r), "bad", len(bad))
    for i in bad[:12]:
        ff = int(r["first_frag"][i]); ef = int(r["emit_frag"][i])
        print(i, "got foff", int(t["foff"][i]), "ff", int(t["first_frag"][i]), "ef", int(t["emit_frag"][i]), "size", int(t["size"][i]),
              "| ref foff", int(r["foff"][i]), "ff", ff, "ef", ef, "size", int(r["size"][i]),
              "| frag types", [int(x) for x in ref.frags["type"][ff:ef + 1]], "lens", [int(x) for x in ref.frags["len"][ff:ef + 1]],
              "offs", [int(x) for x in ref.frags["data_off"][ff:ef + 1]])
    for col in ("size", "first_frag", "emit_frag", "status"):
        print(col, "mismatches", int(np.count_nonzero(t[col].astype(np.uint64) != r[col].astype(np.uint64))))
