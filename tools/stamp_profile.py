#!/usr/bin/env python3
"""Phase breakdown of the sweep kernel from an SR_STAMPS build (diagnostic only).

  SERIATION_LIB=<pkg>/build/stamps/libseriation.so python tools/stamp_profile.py [dataset] [chains] [calls]
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd"))
import numpy as np  # noqa: E402
import seriation_amd as sa  # noqa: E402

PH = ["totals+c,d", "sampleab", "logl", "prop draws", "terms pi1", "terms pi2/swap", "terms pi3", "decide/apply/tail"]
if os.environ.get("SR_FINE"):   # SR_STAMP_FINE builds (tools/build_variant.sh fine "-DSR_STAMPS -DSR_STAMP_FINE")
    PH = ["misc (K, T4, logl, tail)", "sampleab", "C scan+scalar", "C terms", "C dpp sums", "C barrier", "C decide",
          "C apply taxa", "rng generation", "hard tables", "C apply rpi/hp", "A totals + sweep barriers",
          "A c,d draws", "C setup + hard bits", "C ring words", "C lane-par draws"]
path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tests/golden/datasets/synth_256x512.txt")
C = int(sys.argv[2]) if len(sys.argv) > 2 else 100
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 10
tbk = int(sys.argv[4]) if len(sys.argv) > 4 else 0
ds = sa.Dataset.load(path, maxs=0)   # full lines (the bench loads synthetic data the same way)
s = sa.Session(ds, list(range(1, C + 1)), calls_per_launch=calls, block_threads=tbk)
s.run(calls)
s.sync()
t0 = time.perf_counter()
s.run(calls)
s.sync()
wall = time.perf_counter() - t0
out = np.zeros((C, 17, 8), np.uint64)
sa.lib().sr_session_debug_counters(s.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)))
sweeps = calls * 10
nw = s.block_threads // 64
per = out[:, 1:1 + nw, :].astype(np.float64) / 2.0 / sweeps   # [chain, wave, phase] cycles per sweep
if os.environ.get("SR_FINE") and nw <= 8:
    per = np.concatenate([per, out[:, 9:9 + nw, :].astype(np.float64) / 2.0 / sweeps], axis=2)[:, :, :len(PH)]
print("dataset %s  chains %d  TB %d  launch wall %.2f ms  (%.1f us/sweep)" % (os.path.basename(path), C, s.block_threads,
                                                                          wall * 1e3, wall * 1e6 / sweeps))
print("  %-24s %12s %12s %12s" % ("phase (cycles/sweep)", "wave0", "mean wave", "max wave"))
for k, name in enumerate(PH):
    print("  %-24s %12.0f %12.0f %12.0f" % (name, per[:, 0, k].mean(), per[:, :, k].mean(), per[:, :, k].mean(0).max()))
print("  total wave0 %.0f; exact-sum fallbacks/sweep %.3f; sampleab fallbacks/sweep %.3f" % (
    per[:, 0, :].sum(1).mean(), out[:, 0, 0].astype(np.float64).mean() / 2 / sweeps,
    out[:, 0, 1].astype(np.float64).mean() / 2 / sweeps))
print("  sampleab fallback reasons/sweep: prev %.3f here %.3f S0 %.3f (rest = no crossing in segment)" % tuple(
    out[:, 0, 2 + q].astype(np.float64).mean() / 2 / sweeps for q in range(3)))
ev = out[:, 0, 5:8].astype(np.float64).mean(0) / 2 / sweeps
print("  term evaluations/sweep: pi1 %.2f pi2/swap %.2f pi3 %.2f" % tuple(ev))
print("  cycles per evaluation (wave-mean): pi1 %.0f pi2/swap %.0f pi3 %.0f" % tuple(per[:, :, 4 + k].mean() / max(ev[k], 1e-9) for k in range(3)))
if os.environ.get("SR_GIBBS_STATS"):
    h = out[:, 0, :].astype(np.float64).sum(0)
    nd = max(h[4], 1)
    print("  gibbs draws %d: window words/draw %.2f, wave-max window/draw %.2f, walk words/draw %.2f" % (
        h[4], h[5] / nd, h[6] / (nd / 64), h[7] / nd))
