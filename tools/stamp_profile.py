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
warm = int(os.environ.get("SR_WARM", "0"))   # extra calls before the profiled ones (a chain's steady state)
s.run(calls)
s.sync()
out0 = np.zeros((C, 17, 8), np.uint64)
if warm:   # steady state: the counters of the profiled launch alone (they accumulate over launches)
    s.run(warm)
    s.sync()
    sa.lib().sr_session_debug_counters(s.h, out0.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)))
acc0 = np.array([s.accept_counts(c) for c in range(C)], np.float64)
t0 = time.perf_counter()
s.run(calls)
s.sync()
wall = time.perf_counter() - t0
acc = (np.array([s.accept_counts(c) for c in range(C)], np.float64) - acc0).mean(0) / (calls * 10)
out = np.zeros((C, 17, 8), np.uint64)
sa.lib().sr_session_debug_counters(s.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)))
if warm:   # x / 2 / sweeps below: the profiled launch's counters, doubled
    out = (out - out0) * np.uint64(2)
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
if not os.environ.get("SR_FINE") and not os.environ.get("SR_GIBBS_STATS"):
    bs = np.concatenate([out[:, 9, 0:1], out[:, 0, 5:8]], axis=1).astype(np.float64).mean(0) / 2 / sweeps   # coarse builds
    print("  phase-C batches/sweep %.3f; proposals drawn into batches/sweep %.2f (16 needed); proposal-table refills/sweep "
          "%.3f; scalar-path proposals/sweep %.3f" % (bs[1], bs[2], bs[3], bs[0]))
print("  accepted per sweep (profiled launch, chain mean): pi1 %.3f pi2 %.3f swap %.3f pi3 %.3f" % tuple(acc[3:7]))
if os.environ.get("SR_BAR") and nw <= 8:   # SR_STAMPS + SR_STAMP_BAR builds: cycles inside the sweep loop's barriers
    bar = out[:, 9:9 + nw, 7].astype(np.float64) / 2.0 / sweeps
    tot = per[:, :, :8].sum(2)
    print("  barrier wait (cycles/sweep): wave0 %.0f, mean wave %.0f = %.1f %% of the mean wave's sweep" % (
        bar[:, 0].mean(), bar.mean(), 100.0 * bar.mean() / tot.mean()))
if os.environ.get("SR_GIBBS_STATS"):
    h = out[:, 0, :].astype(np.float64).sum(0)
    nd = max(h[4], 1)
    print("  gibbs draws %d: window words/draw %.2f, wave-max window/draw %.2f, walk words/draw %.2f" % (
        h[4], h[5] / nd, h[6] / (nd / 64), h[7] / nd))
