#!/usr/bin/env python3
"""The reference's only known answers, on the HIP path: Docs/Report.pdf Table 1 (p.7).

Each row runs 100 chains (seeds 1..100) of 1000 burn-in + 1000 saved mcmc_sample calls,
selects chains with choose_chains' one-sigma rule (script.py:70-98) and reports E[c], E[d]
(script.py:101-121) and CORRMN (compute_exp_ages, script.py:124-152) beside the published
numbers.  The band is SURVEY.md §8c's proposal (+-0.002 / +-0.03 / +-0.02);
the reference itself states no tolerance.

    python tools/table1.py [--rows g10s10,g5s5,g10s2] > profiles/r01e_table1.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd"))

# dataset -> (chains selected, E[c], E[d], CORRMN) from Docs/Report.pdf Table 1
TABLE1 = {
    "g10s10": (8, 0.0119, 0.5127, 0.940),
    "g5s5": (2, 0.0066, 0.6699, 0.926),
    "g10s2": (2, 0.0093, 0.6833, 0.669),
}
BAND = (0.002, 0.03, 0.02)


def run_row(name, chains=100, burnin=1000, samples=1000, seed_base=1, rng="mt"):
    import seriation_amd as sa
    from seriation_amd import analysis, launcher
    sel, pc, pd, pr = TABLE1[name]
    ds = sa.Dataset.load(os.path.join(ROOT, "tests", "golden", "datasets", name + ".txt"))
    t0 = time.perf_counter()
    summ, (ri, rd) = sa.run_chains(ds, list(range(seed_base, seed_base + chains)), burnin_calls=burnin,
                                   sample_calls=samples, keep_records=True, rng=rng)
    wall = time.perf_counter() - t0
    vals = {"chain_%02d" % k: s["exp_loglik"] for k, s in enumerate(summ)}
    chosen = launcher.choose_from_values(vals, sel)
    ec, ed = analysis.exp_cd_from_records([rd[k] for k in chosen])
    corr = analysis.corr_mn_from_records([ri[k][:, 2 * ds.M:] for k in chosen])
    got = (float(ec), float(ed), float(corr))
    pub = (pc, pd, pr)
    return {"dataset": name, "rng": rng, "sites": ds.N, "taxa": ds.M, "chains": chains, "seed_base": seed_base, "selected": chosen,
            "E_c": got[0], "E_d": got[1], "CORRMN": got[2], "published": {"E_c": pc, "E_d": pd, "CORRMN": pr},
            "within_band": [bool(abs(g - p) < b) for g, p, b in zip(got, pub, BAND)],
            "wall_s": wall, "chain_iterations": chains * (burnin + samples) * 10}


def run_row_spread(name, blocks=6, chains=100, burnin=1000, samples=1000, rng="mt"):
    """The Table 1 estimator (100 chains -> one-sigma selection -> E[c], E[d], CORRMN) repeated over
    `blocks` disjoint seed blocks (seeds 1..100, 101..200, ...).  The reference's own seeds are not
    published (script.py draws them at random), so its row is one draw of this estimator: with 2
    selected chains (g5s5, g10s2) the draw-to-draw spread exceeds the fixed band, and the row is
    checked against the estimator's measured distribution instead -- the published value must lie
    within max(band, 3 sd) of the block mean."""
    import numpy as np
    rows = [run_row(name, chains, burnin, samples, seed_base=1 + b * chains, rng=rng) for b in range(blocks)]
    sel, pc, pd, pr = TABLE1[name]
    out = {"dataset": name, "blocks": rows, "published": {"E_c": pc, "E_d": pd, "CORRMN": pr}}
    ok = []
    for key, pub, band in zip(("E_c", "E_d", "CORRMN"), (pc, pd, pr), BAND):
        v = np.array([r[key] for r in rows])
        mean, sd = float(v.mean()), float(v.std(ddof=1))
        tol = max(band, 3.0 * sd)
        out[key] = {"mean": mean, "sd": sd, "min": float(v.min()), "max": float(v.max()), "tolerance": tol,
                    "within": bool(abs(pub - mean) < tol)}
        ok.append(out[key]["within"])
    out["within_spread"] = ok
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="g10s10,g5s5,g10s2")
    ap.add_argument("--spread", type=int, default=0, help="repeat each row over this many disjoint seed blocks")
    ap.add_argument("--rng", default="mt", choices=("mt", "philox"), help="philox: the opt-in SR_F_RNG_PHILOX stream")
    args = ap.parse_args()
    if args.spread:
        rows = [run_row_spread(r, args.spread, rng=args.rng) for r in args.rows.split(",")]
    else:
        rows = [run_row(r, rng=args.rng) for r in args.rows.split(",")]
    print(json.dumps({"source": "Docs/Report.pdf Table 1 (p.7)", "band": BAND, "rows": rows}, indent=1), flush=True)


if __name__ == "__main__":
    main()
