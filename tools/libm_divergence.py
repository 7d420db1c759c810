#!/usr/bin/env python3
"""How much does the libm matter?  Runs config 2 (g10s10, chains with seeds 1..C, tb burn-in +
ts saved mcmc_sample calls) through two builds of the CPU oracle -- the current one
(glibc exp/log restated, bit-identical to libm.so.6) and an alternative build given by path
(e.g. the round-1 oracle with its own ~0.51-ulp exp/log) -- and reports how many chains
diverge on integers, the first diverging call, and the largest relative difference of
exp_loglik (north_star tolerance: 1e-6).  Diagnostic, CPU only:

    python tools/libm_divergence.py /tmp/oldor/liboracle_old.so [chains] [tb] [ts]
"""
import ctypes
import json
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_ref  # noqa: E402

DS = os.path.join(ROOT, "tests", "golden", "datasets", "g10s10.txt")


def run_with(libpath, text, seed, tb, ts):
    if libpath:
        alt = ctypes.CDLL(libpath)
        alt.oracle_run_chain.restype = ctypes.c_int
        alt.oracle_run_chain.argtypes = oracle_ref.lib().oracle_run_chain.argtypes
        alt.oracle_parse.restype = ctypes.c_int
        alt.oracle_parse.argtypes = oracle_ref.lib().oracle_parse.argtypes
        saved = oracle_ref._L
        oracle_ref._L = alt
        try:
            return oracle_ref.run_chain(text, seed, tb, ts)
        finally:
            oracle_ref._L = saved
    return oracle_ref.run_chain(text, seed, tb, ts)


def one(args):
    alt, seed, tb, ts = args
    with open(DS, "rb") as fh:
        text = fh.read()
    a = run_with(None, text, seed, tb, ts)
    b = run_with(alt, text, seed, tb, ts)
    diff = [t for t in range(ts) if not np.array_equal(a["rec_int"][t], b["rec_int"][t])]
    rel = abs(a["exp"][0] - b["exp"][0]) / abs(a["exp"][0])
    return seed, (diff[0] if diff else None), float(rel)


def main():
    alt = sys.argv[1]
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    tb = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    ts = int(sys.argv[4]) if len(sys.argv) > 4 else 1000
    oracle_ref.lib()
    with mp.get_context("fork").Pool(min(8, os.cpu_count() or 1)) as pool:
        res = pool.map(one, [(alt, s, tb, ts) for s in range(1, C + 1)])
    div = [r for r in res if r[1] is not None]
    print(json.dumps({"dataset": "g10s10", "chains": C, "burnin_calls": tb, "sample_calls": ts,
                      "chains_diverging_on_integers": len(div),
                      "first_divergent_saved_call": sorted(r[1] for r in div)[:10],
                      "max_rel_exp_loglik_diff": max(r[2] for r in res),
                      "median_rel_exp_loglik_diff": float(np.median([r[2] for r in res]))}))


if __name__ == "__main__":
    main()
