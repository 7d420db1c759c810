#!/usr/bin/env python3
"""Parity of the forced-fallback build (tests/test_gpu_fallbacks.py runs this in a child process
with SERIATION_LIB=<pkg>/build/force/libseriation.so, built with -DSR_FORCE_EXACT).

In that build every fast path is replaced by the computation it certifies against: each Gibbs
draw takes the exact three-pass walk (draw_exact: mcmc_auxa + mcmc_logtop + mcmc_randompick,
mcmc.c:711-748, 828-915), each non-vetoed proposal the exact sequential delta (mcmc.c:1214,
1435, 1630) and each c/d update the sequential GSL beta/gamma/ziggurat path (mcmc.c:751-825).
The records must still equal the CPU oracle's bit for bit, and the fallback counters must show
that the fallbacks ran.  Exit status 0 = pass; the first failure is printed."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "seriation-in-paleontological-data-using-mcmc_amd"))

import numpy as np  # noqa: E402

import oracle_ref  # noqa: E402
import seriation_amd as sa  # noqa: E402
from test_gpu_edge import make_text  # noqa: E402


def check(name, text, seeds, tb, ts, columns="auto", block_threads=0):
    ds = sa.Dataset.parse(text, maxs=0)
    with sa.Session(ds, seeds, calls_per_launch=max(tb, ts, 1), block_threads=block_threads, columns=columns) as s:
        s.run(tb, save=False)
        s.run(ts, save=True)
        ab, cdl = s.fetch_records()
        fb = np.array([s.fallback_counts(k) for k in range(len(seeds))])
    for k, seed in enumerate(seeds):
        o = oracle_ref.run_chain(text, seed, tb, ts, maxs=0)
        assert o["rc"] == 0
        if not np.array_equal(ab[k].astype(np.int32), o["rec_int"]):
            raise AssertionError("%s seed %d: integer state differs from the oracle" % (name, seed))
        if not np.array_equal(cdl[k].view(np.uint64), o["rec_dbl"].view(np.uint64)):
            raise AssertionError("%s seed %d: c/d/loglik differ from the oracle" % (name, seed))
    sweeps = (tb + ts) * 10
    tot = fb.sum(0)
    # every c/d update and every Gibbs draw went through its fallback; exact deltas ran
    assert (fb[:, 2] == sweeps).all(), (name, fb)
    assert (fb[:, 1] == 2 * ds.M * sweeps).all(), (name, fb)
    assert tot[0] > 0, (name, fb)
    print("%-22s %d chains x %d calls: bit-exact; fallbacks per chain (exact deltas, exact walks, "
          "sequential c/d) = %s" % (name, len(seeds), tb + ts, fb[0].tolist()), flush=True)


def main():
    ds_dir = os.path.join(HERE, "golden", "datasets")

    def rd(n):
        with open(os.path.join(ds_dir, n), "rb") as fh:
            return fh.read()

    check("g10s10", rd("g10s10.txt"), [1, 2, 3], 2, 4)
    check("g2s2", rd("g2s2.txt"), [1], 2, 3)
    check("synth_256x512", rd("synth_256x512.txt"), [1, 2], 0, 2)
    check("many-hard", make_text(60, 100, 30, seed=60 * 1000 + 100), [1, 7], 2, 3)
    check("lds-walk", make_text(600, 80, 7, seed=600 * 1000 + 80), [1, 7], 1, 2)
    check("tb256-2-per-thread", make_text(96, 512, 5, seed=96 * 1000 + 512), [1, 7], 1, 2, block_threads=256)
    check("hbm-g10s10", rd("g10s10.txt"), [4, 5], 1, 3, columns="hbm")
    print("fallback parity: all cases bit-exact", flush=True)


if __name__ == "__main__":
    main()
