"""Drop-in for the reference's chain launcher (script.py:15-99), backed by the GPU.

The reference runs ``Pool(8).starmap(run_chain, ...)`` over 100 chains, each a
``./mcmc i < dataset`` process seeded through GSL_RNG_SEED (script.py:25-67).  Here the
same functions exist with the same signatures and the same Chains/chain_NN output tree,
but all chains of a call run as one batched GPU session (one workgroup per chain); with
several GPUs the chains are sharded contiguously, one host thread per device.  A chain's
output depends only on (dataset, seed), never on the sharding.
"""
import os
import subprocess
import time

import numpy as np

from . import core


def generate_random_seed():
    """script.py:15-22: one byte from /dev/urandom, as the text `od` prints."""
    try:
        return subprocess.check_output("od -vAn -N1 -tu1 < /dev/urandom", shell=True, text=True)
    except Exception:
        return " %d\n" % (os.urandom(1)[0])


def _unique_seed(old_seeds):
    # script.py:33-39 (the reference's check-then-append is racy; here it is serial)
    while True:
        seed = generate_random_seed()
        if seed not in old_seeds:
            old_seeds.append(seed)
            return int(seed.strip(), 0)


def run_chain(chain_index, old_seeds, dataset, burnin_calls=1000, sample_calls=1000, device=0, root="."):
    """script.py:25-45: run one chain with a fresh unique seed, writing Chains/chain_NN."""
    seed = _unique_seed(old_seeds)
    ds = core.Dataset.load(str(dataset))
    return core.run_to_dirs(ds, [seed], root=root, chain_ids=[chain_index], burnin_calls=burnin_calls,
                            sample_calls=sample_calls, device=device)[0]


def run_all_chains(dataset, n_chains=100, seeds=None, devices=None, burnin_calls=1000, sample_calls=1000,
                   root=".", verbose=True, sweeps_per_call=10, rng="mt", manycd=0):
    """script.py:48-67: run all chains and print the wall time (seconds, 2 decimals).

    seeds: None -> unique 1-byte urandom seeds exactly like the reference (only 256 exist, so
    n_chains <= 256); otherwise an explicit list (deterministic runs).
    devices: list of GPU ordinals to shard over (default: [0]); the sharding is done by the C
    library (sr_run_to_dirs_multi: one host thread and session per device).
    manycd: 1 = per-taxon c, d (mcmc_readmodel's flag, mcmc.c:777-786, 807-816)."""
    if seeds is None:
        old = []
        seeds = [_unique_seed(old) for _ in range(n_chains)]
    seeds = list(seeds)[:n_chains]
    devices = devices or [0]
    ds = core.Dataset.load(str(dataset))
    os.makedirs(os.path.join(root, "Chains"), exist_ok=True)
    start = time.perf_counter()
    devices = devices[:len(seeds)]
    summ = core.run_to_dirs(ds, seeds, root=root, chain_ids=list(range(len(seeds))), burnin_calls=burnin_calls,
                            sample_calls=sample_calls, sweeps_per_call=sweeps_per_call, devices=devices, rng=rng,
                            manycd=manycd)
    finish = time.perf_counter()
    if verbose:
        print(round(finish - start, 2))
    return summ


def _read_exp_loglik(path):
    with open(path) as fh:
        fh.readline()
        return float(fh.readline().split(",")[0])


def choose_chains(chains_selected, root="."):
    """script.py:70-99: chains whose expected negative log-likelihood lies within one
    (population) standard deviation of the best chain; the first `chains_selected` of them
    in ascending value, returned as sorted chain indices.  Quirks kept: strict window,
    ddof=0, mapping back by float equality over the directory listing."""
    chains_dir = os.path.join(root, "Chains")
    dirs = os.listdir(chains_dir)
    vals = [_read_exp_loglik(os.path.join(chains_dir, d, "exp_data.csv")) for d in dirs]
    return choose_from_values(dict(zip(dirs, vals)), chains_selected)


def choose_from_values(dir_to_value, chains_selected):
    """The selection rule of choose_chains on {chain_dir_name: exp_loglik}."""
    vals = list(dir_to_value.values())
    lo = min(vals)
    sd = float(np.std(vals))
    y = sorted(x for x in vals if lo - sd < x < lo + sd)
    chosen = []
    for z in y[:chains_selected]:
        for d, x in dir_to_value.items():
            if x == z:
                chosen.append(int(d.split("_")[1]))
    chosen.sort()
    return chosen
