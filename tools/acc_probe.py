#!/usr/bin/env python3
"""Accepted moves per sweep by kind (diagnostic): how often each apply path runs.

  python tools/acc_probe.py SITES TAXA [chains] [calls] [block_threads]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import gen_synthetic  # noqa: E402
import seriation_amd as sa  # noqa: E402

N, M = int(sys.argv[1]), int(sys.argv[2])
C = int(sys.argv[3]) if len(sys.argv) > 3 else 100
calls = int(sys.argv[4]) if len(sys.argv) > 4 else 20
tb = int(sys.argv[5]) if len(sys.argv) > 5 else 0
seed = 20261015 if (N, M) == (256, 512) else 20261016
path = "/tmp/sr_synth_%dx%d_%d.txt" % (N, M, seed)
if not os.path.exists(path):
    gen_synthetic.write(N, M, seed, path)
ds = sa.Dataset.load(path, maxs=0)   # full lines (the bench loads synthetic data the same way)
with sa.Session(ds, list(range(1, C + 1)), calls_per_launch=2, block_threads=tb) as s:
    s.run(2)
    s.sync()
    t = []
    for k in range(calls // 2):
        t0 = time.perf_counter()
        s.run(2)
        s.sync()
        t.append(time.perf_counter() - t0)
    acc = np.array([s.accept_counts(k) for k in range(C)], np.float64)
sweeps = (calls // 2 + 1) * 20
names = ["c", "d", "ab", "pi1", "pi2", "swap", "pi3"]
print("%dx%d chains %d TB %d: launches (2 calls) %.2f ms mean, %.2f max" % (N, M, C, tb, 1e3 * np.mean(t), 1e3 * np.max(t)))
print("accepted per sweep (mean over chains / max chain):")
for k, n in enumerate(names):
    print("  %-5s %8.3f %8.3f" % (n, acc[:, k].mean() / sweeps, acc[:, k].max() / sweeps))
