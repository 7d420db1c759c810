"""Multi-GPU chain sharding and the one collective.

Chains are independent given their seed, so ranks never talk while sampling.  One
process per GPU owns a contiguous block of chains; at the end every rank contributes a
fixed-size summary record per chain (chain_id, exp_loglik, exp_c, exp_d -- the
exp_data.csv payload, mcmc.c:53-67) to ONE all-gather (RCCL over xGMI with the "nccl"
backend, gloo in the CPU tests), after which every rank can run the one-sigma chain
selection of script.py:70-99 locally and identically.
"""
import math

import numpy as np

from .launcher import choose_from_values

SUMMARY_FIELDS = ("chain_id", "exp_loglik", "exp_c", "exp_d")


def shard(n_chains, world, rank):
    """Contiguous block of chain indices owned by `rank`: [r*C/G, (r+1)*C/G)."""
    if world <= 0 or not 0 <= rank < world or n_chains < 0:
        raise ValueError("bad shard arguments")
    return range(rank * n_chains // world, (rank + 1) * n_chains // world)


def summaries_from_records(chain_ids, cdl):
    """Per-chain summary rows from saved-sample records cdl[chain, sample, (c, d, loglik)]
    exactly as compute_exp_data / print_exp_data (mcmc.c:53-67): sums over the saved
    samples in order, divided by 1000 (the reference hard-codes the divisor)."""
    rows = np.asarray(cdl, np.float64).tolist()
    out = np.zeros((len(chain_ids), 4))
    for k, cid in enumerate(chain_ids):
        ls = cs = ds = 0.0
        for c, d, ll in rows[k]:   # math.exp is the C library's exp, as in mcmc.c
            ls += -ll
            cs += math.exp(c)
            ds += math.exp(d)
        out[k] = (cid, ls / 1000, cs / 1000, ds / 1000)
    return out


def gather_summaries(rows, n_total, device="cpu", group=None):
    """All-gather every rank's summary rows [n_local, 4] (float64) into [n_total, 4],
    ordered by chain_id.  Shards may be ragged: each rank pads to the largest shard
    with chain_id = -1 rows, so the collective is a single fixed-size all_gather."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    width = max(len(shard(n_total, world, r)) for r in range(world))
    buf = torch.full((width, 4), -1.0, dtype=torch.float64, device=device)
    if len(rows):
        buf[:len(rows)] = torch.as_tensor(np.asarray(rows, np.float64), device=device)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    allrows = torch.cat(parts).cpu().numpy()
    allrows = allrows[allrows[:, 0] >= 0]
    allrows = allrows[np.argsort(allrows[:, 0], kind="stable")]
    if len(allrows) != n_total or not np.array_equal(allrows[:, 0], np.arange(n_total)):
        raise RuntimeError("gathered summaries do not cover chains 0..%d" % (n_total - 1))
    return allrows


def select_chains(all_rows, chains_selected):
    """script.py choose_chains on gathered rows (chain dirs named as the reference does)."""
    vals = {"chain_%02d" % int(r[0]): float(r[1]) for r in all_rows}
    return choose_from_values(vals, chains_selected)
