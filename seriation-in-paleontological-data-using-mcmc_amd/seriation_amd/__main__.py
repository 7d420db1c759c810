"""Batched command line: many chains in one GPU session (SURVEY.md §5 "Config / flags").

The reference drives one ``./mcmc i < dataset`` process per chain from ``script.py``
(script.py:25-67, mcmc.c:102-210); ``build/mcmc`` keeps that exact contract.  This entry runs the
whole job at once and writes the same ``Chains/chain_NN`` tree:

    python -m seriation_amd DATASET [--chains 100] [--burnin 1000] [--samples 1000] [--thin 10]
                                    [--seed-base S] [--devices 0,1] [--root .] [--select K]
                                    [--no-save] [--debug-check] [--rng mt|philox] [--manycd]

  --thin        sweeps per saved sample (the reference's mcmc_sample runs 10, mcmc.c:225)
  --seed-base   chain k gets seed S + k; omitted -> unique 1-byte urandom seeds like
                script.py:25-38 (at most 256 chains)
  --select K    after the run, the one-sigma selection of choose_chains (script.py:70-98) over
                the written exp_data.csv files; prints the chosen chain indices
  --no-save     sample without writing files; prints one JSON summary per chain
  --rng         mt: GSL MT19937 as the reference (default); philox: the opt-in counter-based
                Philox4x32-10 stream for sampling (statistically equivalent, not bit-equal)
  --debug-check mcmc_consistent on every chain after every mcmc_sample call (the reference's
                MCMCDEBUG build, mcmc.c:249-255); with --no-save
  --manycd      per-taxon c, d (mcmc_readmodel's manycd = 1, mcmc.c:777-786, 807-816)

Prints the wall time (seconds, 2 decimals) as script.py:67 does.  Exit status 1 when a chain
fails its closing consistency check (mcmc.c:199-204).
"""
import argparse
import json
import sys
import time

from . import core, launcher


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m seriation_amd", description=__doc__.split("\n\n")[0])
    ap.add_argument("dataset")
    ap.add_argument("--chains", type=int, default=100)
    ap.add_argument("--burnin", type=int, default=1000, help="burn-in mcmc_sample calls")
    ap.add_argument("--samples", type=int, default=1000, help="saved mcmc_sample calls")
    ap.add_argument("--thin", type=int, default=10, help="sweeps per mcmc_sample call")
    ap.add_argument("--seed-base", type=int, default=None)
    ap.add_argument("--devices", default="0", help="comma-separated GPU ordinals")
    ap.add_argument("--root", default=".")
    ap.add_argument("--select", type=int, default=0)
    ap.add_argument("--no-save", action="store_true")
    ap.add_argument("--debug-check", action="store_true")
    ap.add_argument("--rng", default="mt", choices=("mt", "philox"))
    ap.add_argument("--manycd", action="store_true")
    a = ap.parse_args(argv)
    if a.chains < 1 or a.burnin < 0 or a.samples < 0 or a.thin < 1:
        ap.error("--chains and --thin must be >= 1, --burnin and --samples >= 0")
    devices = [int(d) for d in a.devices.split(",") if d.strip()]
    if a.seed_base is None:
        if a.chains > 256:
            ap.error("urandom 1-byte seeds (script.py:25-38) allow at most 256 chains; pass --seed-base")
        old = []
        seeds = [launcher._unique_seed(old) for _ in range(a.chains)]
    else:
        seeds = [a.seed_base + k for k in range(a.chains)]
    if a.debug_check and not a.no_save:
        ap.error("--debug-check runs with --no-save")
    if a.no_save:
        ds = core.Dataset.load(a.dataset)
        t0 = time.perf_counter()
        summ, _ = core.run_chains(ds, seeds, burnin_calls=a.burnin, sample_calls=a.samples,
                                  sweeps_per_call=a.thin, devices=devices[:len(seeds)], debug_check=a.debug_check,
                                  rng=a.rng, manycd=int(a.manycd))
        wall = time.perf_counter() - t0
        for s in summ:
            print(json.dumps(s))
        print(round(wall, 2))
    else:
        summ = launcher.run_all_chains(a.dataset, n_chains=a.chains, seeds=seeds, devices=devices,
                                       burnin_calls=a.burnin, sample_calls=a.samples, root=a.root,
                                       sweeps_per_call=a.thin, rng=a.rng, manycd=int(a.manycd))
        if a.select:
            print("selected:", " ".join(str(k) for k in launcher.choose_chains(a.select, a.root)))
    return 1 if any(s.get("consistent", 0) for s in summ) else 0


if __name__ == "__main__":
    sys.exit(main())
