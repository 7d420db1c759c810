#!/usr/bin/env python3
"""Planner A/B for mid-size shapes (round-5 review item 8): shapes whose one-thread-per-taxon
block (1024 threads) does not fit its layout in LDS ran HBM columns; a 512-thread block with two taxa per thread
keeps the columns in LDS.  Same box, interleaved: bench.py on the synthetic N x M (gen_synthetic seed 20261016),
100 chains, each variant with its parity leg (2 selected chains x 2 saved calls against the oracle).

    python tools/ab_planner.py OUTDIR        -> OUTDIR/ab_planner.json"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = [(256, 600), (200, 800), (128, 1000)]
VARIANTS = {"lds512": ["--block-threads", "512", "--columns", "lds"],
            "hbm1024": ["--block-threads", "1024", "--columns", "hbm"]}
COMMON = ["--no-cpu-baseline", "--legs", "none", "--parity-chains", "2", "--parity-rejected", "0", "--parity-calls", "2",
          "--steps", "5", "--warmup", "3", "--calls-per-step", "10", "--total-chains", "100"]


def main():
    out_dir = sys.argv[1]
    res = {}
    for N, M in SHAPES:
        key = "%dx%d" % (N, M)
        res[key] = {v: [] for v in VARIANTS}
        for rep in range(2):
            for v, extra in VARIANTS.items():
                cmd = [sys.executable, "bench.py", "--sites", str(N), "--taxa", str(M)] + COMMON + extra
                p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
                if p.returncode != 0:
                    print(p.stderr[-2000:])
                    raise SystemExit("%s %s failed" % (key, v))
                b = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
                assert b["parity"]["match"], b["parity"]
                res[key][v].append({"value": b["value"], "kernel_ms": b["roofline"]["kernel_ms"],
                                    "columns": b["config"]["columns"], "block_threads": b["config"]["block_threads"],
                                    "kernel_build": b["config"]["kernel_build"]})
                print(key, v, rep, "%.0f chain-iter/s, kernel %.3f ms" % (b["value"], b["roofline"]["kernel_ms"]),
                      flush=True)
    with open(os.path.join(out_dir, "ab_planner.json"), "w") as fh:
        json.dump({"note": "bench.py --sites N --taxa M, 100 chains, 5 steps of 10 calls after 3 warm-up steps; "
                           "interleaved, same box", "shapes": res}, fh, indent=1)


if __name__ == "__main__":
    main()
