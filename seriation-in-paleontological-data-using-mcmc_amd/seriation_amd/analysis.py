"""Posterior summaries over the selected chains (script.py:102-189).

Two forms of each statistic:
  * file form -- reads Chains/chain_NN/chain_data.csv exactly as script.py does (token
    positions, the hard-coded /1000, the pair-order matrix that is not reset between
    chains), for drop-in use after `run_all_chains`;
  * record form -- the same arithmetic on in-memory records (c, d in log scale as the
    sampler keeps them; pi as int arrays), as produced by `run_chains(keep_records=True)`
    or gathered across ranks, without the text round trip.
"""
import os

import numpy as np


def _chain_lines(root, chain):
    with open(os.path.join(root, "Chains", "chain_%02d" % chain, "chain_data.csv")) as fh:
        return fh.readlines()


def compute_exp_cd(chains, chains_selected, root="."):
    """script.py:102-124: mean over chains of (sum over samples of the first c / d token)/1000."""
    c_chain = d_chain = 0.0
    for chain in chains:
        c_sum = d_sum = 0.0
        for line in _chain_lines(root, chain):
            f = line.split(",")
            c_sum += float(f[3].split(" ")[0].strip())
            d_sum += float(f[4].split(" ")[0].strip())
        c_chain += c_sum / 1000
        d_chain += d_sum / 1000
    return c_chain / chains_selected, d_chain / chains_selected


def _pearson_identity(pi):
    x = np.asarray(pi, np.float64)
    y = np.arange(len(x), dtype=np.float64)
    xm, ym = x - x.mean(), y - y.mean()
    return float((xm * ym).sum() / np.sqrt((xm * xm).sum() * (ym * ym).sum()))


def compute_exp_ages(chains, chains_selected, sites, root="."):
    """script.py:127-152 (CORRMN): mean over chains of (sum over samples of
    pearson(pi, 0..N-1))/1000."""
    total = 0.0
    for chain in chains:
        s = 0.0
        for line in _chain_lines(root, chain):
            pi = [int(t.strip()) for t in line.split(",")[2].split(" ")[:sites]]
            s += _pearson_identity(pi)
        total += s / 1000
    return total / chains_selected


def compute_pair_order_matrix(chains, chains_selected, sites, root="."):
    """script.py:155-189 including its quirk: the per-chain accumulator is never reset,
    so chain k's samples are divided by 1000 once per remaining chain."""
    po = np.zeros((sites, sites))
    po_chain = np.zeros((sites, sites))
    for chain in chains:
        for line in _chain_lines(root, chain):
            pi = np.array([int(t.strip()) for t in line.split(",")[2].split(" ")[:sites]])
            po_chain += (pi[:, None] < pi[None, :]).astype(np.float64)
            po_chain[np.diag_indices(sites)] -= 1.0   # i == j contributes -1 (script.py:184-185)
        po_chain /= 1000
        po += po_chain
    return po / chains_selected


# ---------------------------------------------------------------- record forms
def exp_cd_from_records(cdl_per_chain):
    """cdl_per_chain: iterable of [ts, 3] arrays (c, d, loglik) -> (E[c], E[d]) with the
    reference's /1000 per chain and mean over the chains given."""
    cdl_per_chain = list(cdl_per_chain)
    c = sum(np.exp(np.asarray(r)[:, 0]).sum() / 1000 for r in cdl_per_chain)
    d = sum(np.exp(np.asarray(r)[:, 1]).sum() / 1000 for r in cdl_per_chain)
    return c / len(cdl_per_chain), d / len(cdl_per_chain)


def corr_mn_from_records(pi_per_chain):
    """pi_per_chain: iterable of [ts, N] int arrays -> CORRMN as compute_exp_ages."""
    pi_per_chain = list(pi_per_chain)
    tot = 0.0
    for P in pi_per_chain:
        tot += sum(_pearson_identity(p) for p in np.asarray(P)) / 1000
    return tot / len(pi_per_chain)
