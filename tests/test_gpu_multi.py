"""Several devices from one C call (sr_run_chains_multi / sr_run_to_dirs_multi) and the
per-call consistency mode (SR_F_DEBUG_CHECK, the reference's MCMCDEBUG block, mcmc.c:249-255).

On a one-GPU box the device list repeats ordinal 0: each shard is its own session and host thread
on that GPU, which is the same code path as one shard per GPU."""
import filecmp
import os

import numpy as np
import pytest

import oracle_ref
import seriation_amd as sa

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(HERE, "golden", "datasets")


def _load(name):
    return sa.Dataset.load(os.path.join(DATA, name + ".txt"))


def test_run_chains_multi_equals_single():
    ds = _load("g5s5")
    seeds = [3, 5, 8, 13, 21, 34, 55]
    s1, (r1, d1) = sa.run_chains(ds, seeds, burnin_calls=5, sample_calls=7, keep_records=True)
    s3, (r3, d3) = sa.run_chains(ds, seeds, burnin_calls=5, sample_calls=7, keep_records=True, devices=[0, 0, 0])
    assert np.array_equal(r1, r3)
    assert np.array_equal(d1.view(np.uint64), d3.view(np.uint64))
    for a, b in zip(s1, s3):
        assert a == b


def test_run_to_dirs_multi_byte_identical(tmp_path):
    ds = _load("g10s2")
    seeds = [2, 4, 6, 8, 10]
    one, two = tmp_path / "one", tmp_path / "two"
    one.mkdir()
    two.mkdir()
    sa.run_to_dirs(ds, seeds, root=str(one), burnin_calls=3, sample_calls=4)
    sa.run_to_dirs(ds, seeds, root=str(two), burnin_calls=3, sample_calls=4, devices=[0, 0])
    for k in range(len(seeds)):
        d1, d2 = one / "Chains" / ("chain_%02d" % k), two / "Chains" / ("chain_%02d" % k)
        for f in ("chain_data.csv", "exp_data.csv", "taxa.csv", "sites.csv", "hard_sites.csv"):
            assert filecmp.cmp(str(d1 / f), str(d2 / f), shallow=False), (k, f)


def test_debug_check_every_call_matches_oracle():
    """SR_F_DEBUG_CHECK: one launch per mcmc_sample call, mcmc_consistent after each; the samples are
    the ordinary run's (and the oracle's, which also checks every call)."""
    text = open(os.path.join(DATA, "g10s10.txt"), "rb").read()
    ds = sa.Dataset.parse(text)
    seeds = [1, 2]
    s, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=3, sample_calls=6, keep_records=True, debug_check=True)
    for k, seed in enumerate(seeds):
        o = oracle_ref.run_chain(text, seed, 3, 6, check=1)
        assert o["rc"] == 0
        np.testing.assert_array_equal(ri[k], o["rec_int"])
        assert np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64))
        assert s[k]["consistent"] == 0
    with sa.Session(ds, seeds, calls_per_launch=8, debug_check=True) as sess:
        sess.run(8, save=True)
        assert sa.Session is not None and sess.fetch_records()[0].shape[1] == 8


@pytest.mark.parametrize("columns", ["lds", "hbm"])
def test_checkpoint_resume_both_variants_hard_sites(tmp_path, columns):
    """Checkpoint / restore continues exactly for both kernel variants, on a dataset with hard sites
    (the HBM variant keeps a/b and counts in place in HBM and rebuilds its prefix scratch per launch)."""
    from test_gpu_edge import make_text
    text = make_text(70, 90, 9, seed=4242)
    ds = sa.Dataset.parse(text, maxs=0)
    assert ds.nh == 9
    seeds = [5, 6, 7]
    with sa.Session(ds, seeds, calls_per_launch=24, columns=columns) as s:
        assert s.variant == columns
        s.run(24, save=True)
        ab_full, cdl_full = s.fetch_records()
    ck = str(tmp_path / ("chains_%s.srck" % columns))
    with sa.Session(ds, seeds, calls_per_launch=24, columns=columns) as s:
        s.run(9, save=False)
        s.checkpoint(ck)
    r = sa.Session.restore(ds, ck, calls_per_launch=24, columns=columns)
    try:
        assert r.variant == columns
        r.run(15, save=True)
        ab2, cdl2 = r.fetch_records()
    finally:
        r.close()
    assert np.array_equal(ab_full[:, 9:], ab2)
    assert np.array_equal(cdl_full[:, 9:].view(np.uint64), cdl2.view(np.uint64))
