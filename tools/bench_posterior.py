#!/usr/bin/env python3
"""Posterior-summary kernels (csrc/sr_post.hip) at the analysis script's own
scale: 8 selected chains x 1000 saved samples of the synthetic 256x512 workload, read straight
from a session's record buffer in HBM (sr_session_posterior), plus the CPU checker
(oracle/om_script.py, numpy) on the same records for reference.

    python tools/bench_posterior.py [--samples 1000] [--selected 8]

Prints one JSON line: per-kind kernel ms, element-samples/s (output elements x samples), the
bytes each kernel must read (algorithmic: the selected chains' record operands, once) and the
numpy checker's time.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=1000)
    ap.add_argument("--selected", type=int, default=8)
    ap.add_argument("--chains", type=int, default=16)
    args = ap.parse_args()
    import numpy as np
    import seriation_amd as sa
    from seriation_amd import analysis
    ds = sa.Dataset.load(os.path.join(ROOT, "tests", "golden", "datasets", "synth_256x512.txt"))
    N, M = ds.N, ds.M
    sel = list(range(args.selected))
    with sa.Session(ds, list(range(1, args.chains + 1)), calls_per_launch=args.samples) as s:
        s.run(args.samples, save=True)
        s.sync()
        analysis.posterior_from_session(s, sel, args.selected)   # warm-up
        res = {}
        for kind in analysis.KINDS:
            r = analysis.posterior_from_session(s, sel, args.selected, kinds=(kind,))
            res[kind] = r["kernel_ms"]
        ab, _ = s.fetch_records()
    rows = [ab[k].astype(np.int64) for k in sel]
    import om_script
    t0 = time.perf_counter()
    om_script.pair_order_matrix(rows, args.selected, N, M)
    cpu_po = time.perf_counter() - t0
    elems = {"pair_order": N * N, "alive": N * M, "false_alive": N * M, "false_ones": N * M, "exp_pi": N, "exp_a": M}
    nsamp = args.selected * args.samples
    out = {"workload": "synthetic 256x512, %d selected chains x %d samples, records in HBM" % (args.selected, args.samples),
           "kernel_ms": res,
           "element_samples_per_s": {k: elems[k] * nsamp / (res[k] / 1e3) for k in res},
           "algorithmic_bytes": {"pair_order": nsamp * N * 2, "alive": nsamp * 2 * M * 2,
                                 "false_alive": nsamp * 2 * M * 2, "false_ones": nsamp * 2 * M * 2 + N * M,
                                 "exp_pi": nsamp * N * 2, "exp_a": nsamp * M * 2},
           "cpu_checker_pair_order_s": cpu_po,
           "note": "each output element is one thread's sequential f64 accumulation (the script's "
                   "operation order); bound by the dependent add chain, records L2-resident"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
