#!/usr/bin/env python3
"""Config 2's wall split (GPU): the reference protocol on g10s10 (100 chains, 1000 + 1000 calls) three ways --
sr_run_chains without a sink, the launcher writing the Chains/ files, and a bare session (2 launches) -- twice.
Round 6 (r06i): 0.45 / 0.50 / 0.43 s: the files add ~0.07 s; the sampling is the per-sweep latency floor (~21 us per
sweep at 124 x 139, against ~24 us at 256 x 512).    python tools/config2_split.py"""
import sys, time, os, tempfile, shutil
sys.path.insert(0, "seriation-in-paleontological-data-using-mcmc_amd")
import seriation_amd as sa
from seriation_amd import launcher
G = "tests/golden/datasets/g10s10.txt"
ds = sa.Dataset.load(G)
for rep in range(2):
    t = time.perf_counter(); sa.run_chains(ds, list(range(1, 101)), burnin_calls=1000, sample_calls=1000); a = time.perf_counter() - t
    d = tempfile.mkdtemp(); t = time.perf_counter()
    launcher.run_all_chains(G, n_chains=100, seeds=list(range(1, 101)), devices=[0], root=d, verbose=False); b = time.perf_counter() - t
    shutil.rmtree(d)
    with sa.Session(ds, list(range(1, 101)), calls_per_launch=1000) as s:
        t = time.perf_counter(); s.run(1000); s.run(1000, save=True); s.sync(); c = time.perf_counter() - t
    print("run_chains(no sink) %.3f s  run_to_dirs(files) %.3f s  session 2000 calls %.3f s" % (a, b, c), flush=True)
