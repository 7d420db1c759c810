"""Posterior summaries (script.py:102-189) on oracle-written chain files: file form equals
the literal restatement, record form equals file form bit for bit."""
import os
import subprocess

import numpy as np

import oracle_ref
import om_script
from seriation_amd import analysis

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DS = os.path.join(ROOT, "tests", "golden", "datasets", "g10s10.txt")
ORACLE_CLI = os.path.join(ROOT, "oracle", "build", "mcmc_oracle")


def _write_chains(tmp, seeds, tb, ts):
    oracle_ref.lib()
    if not os.path.exists(ORACLE_CLI):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    recs = {}
    text = open(DS, "rb").read()
    for k, s in enumerate(seeds):
        d = os.path.join(tmp, "run%d" % k)
        os.makedirs(os.path.join(d, "Chains", "chain_00"))
        with open(DS, "rb") as fin:
            subprocess.check_call([ORACLE_CLI, "0", str(tb), str(ts)], cwd=d, stdin=fin,
                                  env=dict(os.environ, GSL_RNG_SEED=str(s)), stderr=subprocess.DEVNULL)
        os.makedirs(os.path.join(tmp, "Chains"), exist_ok=True)
        os.rename(os.path.join(d, "Chains", "chain_00"), os.path.join(tmp, "Chains", "chain_%02d" % k))
        recs[k] = oracle_ref.run_chain(text, s, tb, ts)
    return recs


def test_file_and_record_forms_agree(tmp_path):
    recs = _write_chains(str(tmp_path), [3, 8, 11], 3, 6)
    chains = [0, 1, 2]
    N, M = 124, 139
    c, d = analysis.compute_exp_cd(chains, 3, root=str(tmp_path))
    c2, d2 = analysis.exp_cd_from_records([recs[k]["rec_dbl"] for k in chains])
    assert (c, d) == (c2, d2)
    # chains_selected larger than the chains found (the script divides by chains_selected)
    assert analysis.compute_exp_cd(chains[:2], 3, root=str(tmp_path)) == \
        analysis.exp_cd_from_records([recs[k]["rec_dbl"] for k in chains[:2]], 3)
    r = analysis.compute_exp_ages(chains, 3, N, root=str(tmp_path))
    r2 = analysis.corr_mn_from_records([recs[k]["rec_int"][:, 2 * M:] for k in chains])
    assert r == r2
    # the oracle's vectorised pair-order (checker of the GPU kernel) equals the script's literal
    # loops (script.py:155-189 with generate_po_matrix), read back from the chain files
    po_ref = np.zeros((N, N))
    po_chain = np.zeros((N, N))
    for k in chains:
        for p in recs[k]["rec_int"][:, 2 * M:]:
            for i in range(N):
                for j in range(N):
                    po_chain[i][j] += -1 if i == j else int(p[i] < p[j])
        po_chain /= 1000
        po_ref += po_chain
    po_ref /= 3
    rows = [om_script.read_chain_rows(os.path.join(str(tmp_path), "Chains", "chain_%02d" % k, "chain_data.csv"), N, M)
            for k in chains]
    assert np.array_equal(om_script.pair_order_matrix(rows, 3, N, M).view(np.uint64), po_ref.view(np.uint64))
    # the product's chain-file reader gives the same rows
    prod = analysis.read_chain_rows(str(tmp_path), chains, N, M)
    for k in range(3):
        assert np.array_equal(prod[k], rows[k])


def test_pearson_is_the_scripts_call():
    """CORRMN's per-sample coefficient is script.py:147's scipy.stats.pearsonr(pi_chain,
    np.arange(0, sites))[0] (list of ints against an int range), bit for bit."""
    from scipy.stats import pearsonr
    rng = np.random.default_rng(3)
    for n in (124, 273, 256, 2):
        for _ in range(200 if n > 2 else 2):
            pi = [int(v) for v in rng.permutation(n)]
            assert analysis._pearson_identity(pi) == pearsonr(pi, np.arange(0, n))[0]
