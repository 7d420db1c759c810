"""GPU posterior summaries (csrc/sr_post.hip) against the CPU checker oracle/om_script.py, every
f64 bit: pair-order matrix, taxon alive / false-alive / false-ones sums, E[pi], E[a]
(script.py:155-189, 230-275, 306-417), from host records, from a session's records in HBM and
from chain files, plus the script's argsort reorderings."""
import os

import numpy as np
import pytest

import om_script
import oracle_ref
import seriation_amd as sa
from seriation_amd import analysis

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DS = os.path.join(ROOT, "tests", "golden", "datasets")


def same(x, y):
    x, y = np.asarray(x, np.float64), np.asarray(y, np.float64)
    return x.shape == y.shape and np.array_equal(x.view(np.uint64), y.view(np.uint64))


def check_all(res, rows, cs, X, N, M):
    assert same(res["pair_order"], om_script.pair_order_matrix(rows, cs, N, M))
    assert same(res["alive"], om_script.alive_sum(rows, cs, N, M))
    assert same(res["false_alive"], om_script.false_alive_sum(rows, cs, N, M))
    assert same(res["false_ones"], om_script.false_ones_sum(rows, cs, X, N, M))
    assert same(res["exp_pi"], om_script.exp_pi(rows, N, cs, M))
    assert same(res["exp_a"], om_script.exp_a(rows, cs, M))


@pytest.mark.parametrize("N,M,nch,ns,cs", [(124, 139, 3, 1000, 3), (5, 3, 2, 17, 8), (300, 70, 1, 250, 1)])
def test_posterior_random_records(N, M, nch, ns, cs):
    rng = np.random.default_rng(N + M)
    rows = []
    for _ in range(nch):
        a = rng.integers(0, N + 1, (ns, M))
        b = np.minimum(N, a + rng.integers(0, N // 2 + 1, (ns, M)))
        pi = np.argsort(rng.random((ns, N)), axis=1)
        rows.append(np.concatenate([a, b, pi], axis=1))
    X = (rng.random((N, M)) < 0.3).astype(np.uint8)
    ds = sa.Dataset(X, np.zeros(N, bool))
    res = analysis.posterior_from_records(ds, np.stack(rows), cs)
    check_all(res, rows, cs, X, N, M)
    assert res["kernel_ms"] > 0


def test_posterior_from_session_records():
    text = open(os.path.join(DS, "g10s10.txt"), "rb").read()
    ds = sa.Dataset.parse(text)
    seeds = [5, 9, 13, 21]
    with sa.Session(ds, seeds, calls_per_launch=40) as s:
        s.run(5)
        s.reset_records()
        s.run(40, save=True)
        ab, _ = s.fetch_records()
        sel = [2, 0, 3]   # selection order matters (accumulator carried over chains)
        res = analysis.posterior_from_session(s, sel, 8)
    rows = [ab[k].astype(np.int64) for k in sel]
    check_all(res, rows, 8, ds.X, ds.N, ds.M)


def test_posterior_file_forms(tmp_path):
    """Chain files written by the drop-in output path, read back like the script does."""
    text = open(os.path.join(DS, "g10s10.txt"), "rb").read()
    ds = sa.Dataset.parse(text)
    N, M = ds.N, ds.M
    sa.run_to_dirs(ds, [3, 4, 6], root=str(tmp_path), chain_ids=[0, 1, 2], burnin_calls=2, sample_calls=30)
    chains = [0, 2]
    rows = [om_script.read_chain_rows(os.path.join(str(tmp_path), "Chains", "chain_%02d" % k, "chain_data.csv"), N, M)
            for k in chains]
    po = analysis.compute_pair_order_matrix(chains, 2, N, root=str(tmp_path))
    assert same(po, om_script.pair_order_matrix(rows, 2, N, M))
    e_pi = analysis.compute_exp_pi(chains, N, 2, root=str(tmp_path))
    e_a = analysis.compute_exp_a(chains, 2, M, root=str(tmp_path))
    assert same(e_pi, om_script.exp_pi(rows, N, 2, M)) and same(e_a, om_script.exp_a(rows, 2, M))
    t = analysis.taxa_occurence_probability_matrix(chains, 2, N, M, root=str(tmp_path))
    assert same(t, om_script.reorder(om_script.alive_sum(rows, 2, N, M), e_pi, e_a))
    f = analysis.false_taxa_occurence_probability(chains, 2, N, M, root=str(tmp_path))
    assert same(f, om_script.reorder(om_script.false_alive_sum(rows, 2, N, M), e_pi, e_a))
    o = analysis.false_ones_probability(chains, 2, os.path.join(DS, "g10s10.txt"), N, M, root=str(tmp_path))
    assert same(o, om_script.reorder(om_script.false_ones_sum(rows, 2, ds.X, N, M), e_pi, e_a))
    # the records behind the files are the oracle's chain (sampler parity, as elsewhere)
    orc = oracle_ref.run_chain(text, 3, 2, 30)
    assert np.array_equal(rows[0], orc["rec_int"])
