#!/usr/bin/env python3
"""Summarise an A/B directory of tools/gpu_ab_par.sh into one profiles/ JSON.

  python tools/ab_summary.py gpurun_out/r05r profiles/r05r_ab_x.json "experiment text"
"""
import glob
import json
import os
import sys

src, dst, text = sys.argv[1], sys.argv[2], sys.argv[3]
runs, means = {}, {}
for f in sorted(glob.glob(os.path.join(src, "*_[0-9].json"))):
    b = json.load(open(f))
    name = os.path.basename(f)
    runs[name] = {"value": b["value"], "kernel_ms": b["roofline"]["kernel_ms"]}
    means.setdefault(name.rsplit("_", 1)[0], []).append(b["roofline"]["kernel_ms"])
par = {}
for f in sorted(glob.glob(os.path.join(src, "parity_*.log"))):
    lines = [l.strip() for l in open(f) if l.strip()]
    par[os.path.basename(f)] = lines[-1] if lines else ""
out = {"experiment": text, "runs": runs, "mean_kernel_ms": {k: sum(v) / len(v) for k, v in means.items()},
       "parity": par}
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out["mean_kernel_ms"]))
