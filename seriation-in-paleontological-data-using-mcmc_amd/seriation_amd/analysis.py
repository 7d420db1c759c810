"""Posterior summaries over the selected chains (script.py:102-429).

Scalar statistics (E[c], E[d], CORRMN: per-chain sums of ~1000 values) are host Python, in
two forms with identical results:
  * file form -- reads Chains/chain_NN/chain_data.csv exactly as script.py does (token
    positions, the hard-coded /1000), for drop-in use after `run_all_chains`;
  * record form -- the same operation sequence on in-memory records (c, d in log scale as
    the sampler keeps them; pi as int arrays), as produced by `run_chains(keep_records=True)`
    or gathered across ranks (dist.gather_selected_records), without writing the files.

The per-sample matrix accumulations (pair-order matrix, taxon alive / false-alive /
false-ones probabilities, E[pi], E[a]) run on the GPU (csrc/sr_post.hip through
sr_posterior / sr_session_posterior), bit for bit as the script computes them; only the
final argsort reorderings are host numpy.  There is no CPU fallback for them.
"""
import ctypes
import math
import os

import numpy as np

from . import _lib as L
from .core import _check


def _chain_lines(root, chain):
    with open(os.path.join(root, "Chains", "chain_%02d" % chain, "chain_data.csv")) as fh:
        return fh.readlines()


def compute_exp_cd(chains, chains_selected, root="."):
    """script.py:100-124: mean over chains of (sum over samples of the first c / d token)/1000,
    divided by chains_selected."""
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
    """script.py:147: scipy.stats.pearsonr(pi_chain, np.arange(0, sites))[0] -- the reference's
    own call (scipy of this image; the reference pinned scipy 1.4.1, whose formula may differ
    from it in the last bits)."""
    from scipy.stats import pearsonr
    return float(pearsonr(pi, np.arange(0, len(pi)))[0])


def compute_exp_ages(chains, chains_selected, sites, root="."):
    """script.py:127-152 (CORRMN): mean over chains of (sum over samples of
    pearson(pi, 0..N-1))/1000, divided by chains_selected."""
    total = 0.0
    for chain in chains:
        s = 0.0
        for line in _chain_lines(root, chain):
            pi = [int(t.strip()) for t in line.split(",")[2].split(" ")[:sites]]
            s += _pearson_identity(pi)
        total += s / 1000
    return total / chains_selected


# ---------------------------------------------------------------- record forms
# The same operation sequences on in-memory records (c, d in log scale as the sampler keeps them;
# pi as int rows), as produced by run_chains(keep_records=True) or gathered across ranks
# (dist.gather_selected_records): each c / d is the value the file form reads back, i.e.
# mcmc_save_chain's "%.14f" of the C library's exp (mcmc.c:82-85), summed sequentially; so the
# record forms equal the file forms bit for bit (tests/test_analysis.py).
def _token(v):
    return float("%.14f" % math.exp(v))


def exp_cd_from_records(cdl_per_chain, chains_selected=None):
    """cdl_per_chain: iterable of [ts, 3] arrays (c, d, loglik) -> (E[c], E[d]) as
    compute_exp_cd; chains_selected defaults to the number of chains given."""
    cdl_per_chain = list(cdl_per_chain)
    c_chain = d_chain = 0.0
    for r in cdl_per_chain:
        c_sum = d_sum = 0.0
        for c, d, _ll in np.asarray(r, np.float64).tolist():
            c_sum += _token(c)
            d_sum += _token(d)
        c_chain += c_sum / 1000
        d_chain += d_sum / 1000
    n = len(cdl_per_chain) if chains_selected is None else chains_selected
    return c_chain / n, d_chain / n


def corr_mn_from_records(pi_per_chain, chains_selected=None):
    """pi_per_chain: iterable of [ts, N] int arrays -> CORRMN as compute_exp_ages."""
    pi_per_chain = list(pi_per_chain)
    tot = 0.0
    for P in pi_per_chain:
        s = 0.0
        for p in np.asarray(P).tolist():
            s += _pearson_identity(p)
        tot += s / 1000
    n = len(pi_per_chain) if chains_selected is None else chains_selected
    return tot / n


# ---------------------------------------------------------------- GPU posterior summaries
KINDS = ("pair_order", "alive", "false_alive", "false_ones", "exp_pi", "exp_a")


def _shape(kind, N, M):
    return {"pair_order": (N, N), "alive": (N, M), "false_alive": (N, M), "false_ones": (N, M),
            "exp_pi": (N,), "exp_a": (M,)}[kind]


def _outs(kinds, N, M):
    arrs = {k: np.zeros(_shape(k, N, M)) for k in kinds}
    out = L.sr_posterior_out()
    for k, a in arrs.items():
        setattr(out, k, a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return out, arrs


def posterior_from_records(dataset, ab_pi, chains_selected, kinds=KINDS, device=0):
    """sr_posterior: ab_pi [n_sel][count][2M+N] (a | b | pi rows, chains in selection order)
    -> {kind: array}; dataset supplies N, M and X (false_ones)."""
    rec = np.ascontiguousarray(ab_pi, dtype=np.int16)
    assert rec.ndim == 3 and rec.shape[2] == 2 * dataset.M + dataset.N
    out, arrs = _outs(kinds, dataset.N, dataset.M)
    _check(L.lib().sr_posterior(ctypes.byref(dataset.c), rec.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)),
                                rec.shape[0], rec.shape[1], int(chains_selected), device, ctypes.byref(out)),
           "sr_posterior")
    arrs["kernel_ms"] = out.kernel_ms
    return arrs


def posterior_from_session(session, chains, chains_selected, first=0, count=None, kinds=KINDS):
    """sr_session_posterior: the same summaries over a session's records still in HBM.
    chains: session chain indices in selection order."""
    count = session_records(session) - first if count is None else count
    ch = (ctypes.c_int32 * len(chains))(*[int(c) for c in chains])
    out, arrs = _outs(kinds, session.ds.N, session.ds.M)
    _check(L.lib().sr_session_posterior(session.h, ch, len(chains), first, count, int(chains_selected),
                                        ctypes.byref(out)), "sr_session_posterior")
    arrs["kernel_ms"] = out.kernel_ms
    return arrs


def session_records(session):
    return L.lib().sr_session_records(session.h)


def read_chain_rows(root, chains, sites, taxa):
    """chain_data.csv of each chain -> int16 [n][lines][2M+N] (fields 0, 1, 2 tokens as the script
    slices them).  All chains must hold the same number of lines."""
    out = []
    for chain in chains:
        rows = []
        for line in _chain_lines(root, chain):
            f = line.split(",", 3)
            rows.append(np.concatenate([np.array(f[0].split(), np.int64)[:taxa], np.array(f[1].split(), np.int64)[:taxa],
                                        np.array(f[2].split(), np.int64)[:sites]]))
        out.append(np.array(rows, np.int16).reshape(len(rows), 2 * taxa + sites))
    return np.stack(out)


def _file_posterior(chains, chains_selected, sites, taxa, kinds, root, X=None, device=0):
    from .core import Dataset
    rec = read_chain_rows(root, chains, sites, taxa)
    ds = Dataset(np.zeros((sites, taxa), np.uint8) if X is None else np.asarray(X, np.uint8)[:sites, :taxa],
                 np.zeros(sites, bool))
    return posterior_from_records(ds, rec, chains_selected, kinds, device)


def compute_pair_order_matrix(chains, chains_selected, sites, root=".", taxa=None, device=0):
    """script.py:155-189 on the GPU (quirk kept: the per-chain accumulator is never reset).
    taxa: M of the chain files (read from the first line when omitted)."""
    taxa = taxa or _taxa_of(root, chains[0])
    return _file_posterior(chains, chains_selected, sites, taxa, ("pair_order",), root, device=device)["pair_order"]


def compute_exp_pi(chains, sites, chains_selected, root=".", taxa=None, device=0):
    """script.py:230-251 on the GPU (quirk kept: the result is the last per-chain snapshot)."""
    taxa = taxa or _taxa_of(root, chains[0])
    return _file_posterior(chains, chains_selected, sites, taxa, ("exp_pi",), root, device=device)["exp_pi"]


def compute_exp_a(chains, chains_selected, taxa, root=".", sites=None, device=0):
    """script.py:254-275 on the GPU."""
    sites = sites or _sites_of(root, chains[0], taxa)
    return _file_posterior(chains, chains_selected, sites, taxa, ("exp_a",), root, device=device)["exp_a"]


def reorder(mat, exp_pi, exp_a):
    """Rows by the inverse permutation of argsort(exp_pi), columns in argsort(exp_a) order
    (script.py:288-301, 336-347)."""
    rpi = np.argsort(exp_pi)
    idx = np.empty_like(rpi)
    idx[rpi] = np.arange(len(rpi))
    return np.asarray(mat)[idx, :][:, np.argsort(exp_a)]


def taxa_occurence_probability_matrix(chains, chains_selected, sites, taxa, root=".", device=0):
    """plot_taxa_occurence_probability_matrix's return value (script.py:306-347)."""
    r = _file_posterior(chains, chains_selected, sites, taxa, ("alive", "exp_pi", "exp_a"), root, device=device)
    return reorder(r["alive"], r["exp_pi"], r["exp_a"])


def false_taxa_occurence_probability(chains, chains_selected, sites, taxa, root=".", device=0):
    """plot_false_taxa_occurence_probability's return value (script.py:350-389)."""
    r = _file_posterior(chains, chains_selected, sites, taxa, ("false_alive", "exp_pi", "exp_a"), root, device=device)
    return reorder(r["false_alive"], r["exp_pi"], r["exp_a"])


def false_ones_probability(chains, chains_selected, dataset, sites, taxa, root=".", device=0):
    """plot_false_ones_probability's return value (script.py:392-429), N x M (the script
    hard-codes the 124 x 139 shape of g10s10)."""
    from .core import Dataset
    ds = dataset if isinstance(dataset, Dataset) else Dataset.load(str(dataset), maxs=0)
    r = _file_posterior(chains, chains_selected, sites, taxa, ("false_ones", "exp_pi", "exp_a"), root, X=ds.X,
                        device=device)
    return reorder(r["false_ones"], r["exp_pi"], r["exp_a"])


def _taxa_of(root, chain):
    with open(os.path.join(root, "Chains", "chain_%02d" % chain, "chain_data.csv")) as fh:
        return len(fh.readline().split(",", 1)[0].split())


def _sites_of(root, chain, taxa):
    with open(os.path.join(root, "Chains", "chain_%02d" % chain, "chain_data.csv")) as fh:
        return len(fh.readline().split(",")[2].split())
