"""Parity fuzz over random shapes (GPU): random N, M, hard sites, block size, column placement and c/d mode, each run against
the CPU oracle (2 burn-in + 3 saved calls, 2 seeds).  Prints one line per shape and exits 1 on the first mismatch.
    python tools/fuzz_shapes.py [count] [seed] [--lds | --mid]"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "seriation-in-paleontological-data-using-mcmc_amd"))
import oracle_ref                      # noqa: E402  (the checker)
import seriation_amd as sa             # noqa: E402
from test_gpu_edge import make_text    # noqa: E402


def main():
    lds = "--lds" in sys.argv   # LDS-column shapes (register and LDS walks; with SR_JIT unset, specialised kernels)
    mid = "--mid" in sys.argv   # the planner's mid-size shapes (N 64-320, M 513-1024: 512-thread LDS columns, round 6)
    argv = [a for a in sys.argv[1:] if a not in ("--lds", "--mid")]
    count = int(argv[0]) if argv else 12
    rng = np.random.default_rng(int(argv[1]) if len(argv) > 1 else 2026)
    for t in range(count):
        N = int(rng.integers(64, 321)) if mid else int(rng.integers(8, 544 if lds else 1500))
        M = int(rng.integers(513, 1025)) if mid else int(rng.integers(2, 1025 if lds else 2600))
        nh = int(min(N - 2, rng.choice([0, 3, 12, 40, 70])))
        tb = 0 if mid else int(rng.choice([0, 256, 512, 1024]))
        cols = "auto" if (lds or mid) else str(rng.choice(["auto", "hbm"]))
        mcd = 0 if mid else int(rng.random() < 0.2)   # manycd: per-taxon c, d (1024 threads)
        if mcd:
            tb = int(rng.choice([0, 1024]))
        if tb and M > tb and cols == "auto" and rng.random() < 0.5:
            tb = 0
        text = make_text(N, M, nh, seed=int(rng.integers(1 << 30)))
        ds = sa.Dataset.parse(text, maxs=0)
        seeds = [int(s) for s in rng.integers(1, 1000, 2)]
        try:
            with sa.Session(ds, seeds, block_threads=tb, columns=cols, manycd=mcd) as s:
                desc = "%s/%s tb %d" % (s.variant, s.kernel, s.block_threads)
        except sa.SrError as e:
            print("shape %2d N %4d M %4d nh %2d tb %4d %s: refused (%s)" % (t, N, M, nh, tb, cols, e), flush=True)
            continue
        out = sa.run_chains(ds, seeds, burnin_calls=2, sample_calls=3, keep_records=True, block_threads=tb, columns=cols,
                            manycd=mcd)
        summ, recs = out
        ri, rd = recs[0], recs[1]
        ok = True
        for k, sd in enumerate(seeds):
            o = oracle_ref.run_chain(text, sd, 2, 3, maxs=0, manycd=mcd)
            ok = ok and o["rc"] == 0 and np.array_equal(ri[k], o["rec_int"]) and \
                np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64)) and summ[k]["consistent"] == 0
            if mcd:
                ok = ok and np.array_equal(recs[2][k].view(np.uint64), o["rec_cdv"].view(np.uint64))
        print("shape %2d N %4d M %4d nh %2d tb %4d %-4s%s -> %-18s %s" % (t, N, M, nh, tb, cols, " mcd" if mcd else "", desc,
                                                                          "== oracle" if ok else "MISMATCH"), flush=True)
        if not ok:
            sys.exit(1)


if __name__ == "__main__":
    main()
