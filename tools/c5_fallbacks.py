#!/usr/bin/env python3
"""Config 5 (1024 x 2048, split chains): kernel time and the fast paths' fallback counts of a session
(sr_session_fallback_counts: exact deltas, exact Gibbs walks, sequential c/d draws) -- for A/Bs of the
Gibbs checkpoint forms.   SERIATION_LIB=... python tools/c5_fallbacks.py [chains] [calls]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import gen_synthetic  # noqa: E402
import seriation_amd as sa  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 100
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 10
X, hard = gen_synthetic.make(1024, 2048, 20261016)
ds = sa.Dataset(X, hard)
with sa.Session(ds, list(range(1, C + 1)), calls_per_launch=calls, block_threads=1024) as s:
    s.run(2)
    s.sync()
    t = time.perf_counter()
    s.run(calls)
    s.sync()
    wall = time.perf_counter() - t
    ms = s.last_kernel_ms()
    fb = np.array([s.fallback_counts(k) for k in range(C)])
    acc = np.array([s.accept_counts(k) for k in range(C)])
    kern = s.kernel
print(json.dumps({"lib": os.environ.get("SERIATION_LIB", "product"), "kernel": kern, "chains": C, "calls": calls,
                  "kernel_ms": ms, "wall_s": wall, "fallbacks_total": fb.sum(axis=0).tolist(),
                  "exact_walks_per_chain_sweep": float(fb[:, 1].sum()) / (C * (calls + 2) * 10),
                  "accepts_total": acc.sum(axis=0).tolist()}))
