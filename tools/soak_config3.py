#!/usr/bin/env python3
"""Parity soak of config 3 (GPU + CPU oracle): 100 chains (seeds 1..100) on the synthetic 256 x 512 matrix under the
reference CLI's protocol -- 1000 burn-in + 1000 saved calls of 10 sweeps (mcmc.c:140-185) -- every saved record of
every chain against the CPU oracle, bit for bit (a, b, pi; c, d, loglik as f64 bits).  The GPU tests hold 16 chains
to this depth; this run holds all 100 (the oracle needs ~5 min on 16 cores).   python tools/soak_config3.py OUT.json"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench_parity  # noqa: E402
import seriation_amd as sa  # noqa: E402

SYNTH = os.path.join(ROOT, "tests", "golden", "datasets", "synth_256x512.txt")


def main():
    with open(SYNTH, "rb") as fh:
        text = fh.read()
    ds = sa.Dataset.parse(text, maxs=0)
    ids = list(range(100))
    t0 = time.perf_counter()
    with sa.Session(ds, [i + 1 for i in ids], calls_per_launch=1000) as s:
        for _ in range(20):
            s.run(50, save=False)
        for _ in range(20):
            s.run(50, save=True)
        ab, cdl = s.fetch_records()
        kernel = s.kernel, s.specialized
    gpu_s = time.perf_counter() - t0
    # the oracle in chunks of 16 chains (one per core of the box's CPU share), a progress line after each
    out = {"chains": [], "match": True, "mismatch": {}, "oracle_wall_s": 0.0}
    for k0 in range(0, len(ids), 16):
        ch = ids[k0:k0 + 16]
        r = bench_parity.check_selected(text, ch, [i + 1 for i in ch], 1000, ab[k0:k0 + 16], cdl[k0:k0 + 16])
        out["chains"] += r["chains"]
        out["match"] = out["match"] and r["match"]
        out["mismatch"].update(r["mismatch"])
        out["oracle_wall_s"] += r["oracle_wall_s"]
        out["saved_calls_compared"] = r["saved_calls_compared"]
        print("chains %d..%d: %s (%.0f s)" % (ch[0], ch[-1], "match" if r["match"] else r["mismatch"], r["oracle_wall_s"]),
              flush=True)
    out.update({"gpu_wall_s": gpu_s, "kernel": list(kernel), "note": "100 chains x (1000 burn-in + 1000 saved calls), "
                "every saved record of every chain against the CPU oracle"})
    with open(sys.argv[1], "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: out[k] for k in ("match", "saved_calls_compared", "oracle_wall_s", "gpu_wall_s")}))
    sys.exit(0 if out["match"] else 1)


if __name__ == "__main__":
    main()
