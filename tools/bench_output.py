#!/usr/bin/env python3
"""End-to-end sampling with the reference's file output: sr_run_to_dirs on the
synthetic 256x512 matrix, 100 chains, writing Chains/chain_NN/chain_data.csv (one ~22 KB
mcmc_save_chain line per saved call) while the GPU samples the next launch.

    python tools/bench_output.py [--chains 100] [--calls 200] [--threads 1,16]

Prints one JSON line per writer-thread count: wall seconds, saved lines/s, MB/s of CSV written,
and the GPU-only time of the same sampling (records kept in HBM, no formatting) for reference.
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=100)
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--threads", default="1,16")
    ap.add_argument("--dataset", default=os.path.join(ROOT, "tests", "golden", "datasets", "synth_256x512.txt"))
    args = ap.parse_args()
    import seriation_amd as sa
    ds = sa.Dataset.load(args.dataset)
    seeds = list(range(1, args.chains + 1))
    # GPU-only reference: the same calls, records resident in HBM
    with sa.Session(ds, seeds, calls_per_launch=100) as s:
        s.run(10)
        s.sync()
        t0 = time.perf_counter()
        left = args.calls
        while left > 0:
            k = min(100, left)
            s.reset_records()
            s.run(k, save=True)
            left -= k
        s.sync()
        gpu_s = time.perf_counter() - t0
    for nt in [int(x) for x in args.threads.split(",")]:
        os.environ["SR_WRITER_THREADS"] = str(nt)
        d = tempfile.mkdtemp(prefix="sr_out_")
        try:
            t0 = time.perf_counter()
            sa.run_to_dirs(ds, seeds, root=d, chain_ids=list(range(args.chains)), burnin_calls=0,
                           sample_calls=args.calls)
            wall = time.perf_counter() - t0
            nbytes = sum(os.path.getsize(os.path.join(d, "Chains", c, "chain_data.csv"))
                         for c in os.listdir(os.path.join(d, "Chains")))
        finally:
            shutil.rmtree(d, ignore_errors=True)
        lines = args.chains * args.calls
        print(json.dumps({"writer_threads": nt, "chains": args.chains, "saved_calls": args.calls,
                          "wall_s": wall, "lines_per_s": lines / wall, "csv_MB": nbytes / 1e6,
                          "csv_MB_per_s": nbytes / 1e6 / wall, "gpu_only_s": gpu_s,
                          "note": "wall includes session setup (init, upload), GPU sampling, overlapped "
                                  "formatting + writes, final consistency check and the summary files"}),
              flush=True)


if __name__ == "__main__":
    main()
