#!/usr/bin/env python3
"""Parity of the experimental 512-thread split kernel (SR_SPLIT=2: halves of up to 1024 taxa, two taxa per
thread) against the CPU oracle: config 5's matrix (8 chains x 1 + 10 calls) and a ragged forced split
(60 x 1500, 30 hard sites).   SR_SPLIT=2 python tools/sp512_check.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import gen_synthetic  # noqa: E402
import oracle_ref  # noqa: E402
import seriation_amd as sa  # noqa: E402
from test_gpu_edge import make_text  # noqa: E402

out = {}
X, hard = gen_synthetic.make(1024, 2048, 20261016)
text = gen_synthetic.to_text(X, hard).encode()
cases = [("config5", text, [1, 2, 3, 4, 5, 6, 7, 8], 1, 10), ("ragged", make_text(60, 1500, 30, seed=60 * 1000 + 1500), [5, 13, 21], 2, 3)]
for name, txt, seeds, bi, sc in cases:
    ds = sa.Dataset.parse(txt, maxs=0)
    with sa.Session(ds, seeds, block_threads=512, columns="hbm") as s:
        kern = s.kernel
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=bi, sample_calls=sc, keep_records=True, block_threads=512,
                                   columns="hbm")
    ok = True
    for k, sd in enumerate(seeds):
        o = oracle_ref.run_chain(txt, sd, bi, sc, maxs=0)
        ok = ok and o["rc"] == 0 and np.array_equal(ri[k], o["rec_int"]) and \
            np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64)) and summ[k]["consistent"] == 0
    out[name] = {"kernel": kern, "chains": len(seeds), "calls": bi + sc, "match": bool(ok)}
print(json.dumps(out))
sys.exit(0 if all(v["match"] and v["kernel"] == "split" for v in out.values()) else 1)
