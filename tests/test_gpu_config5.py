"""BASELINE.json configs[4]: synthetic 1024 sites x 2048 taxa (tools/gen_synthetic.py, seed
20261016, 12 hard sites).  The bit columns (256 KB per chain) exceed the 160 KB LDS, so the
session runs the HBM-column kernel variant; every saved sample must equal the CPU oracle bit for
bit.  The reference parser cannot read its 4096-char lines (MAXS = 2000, mcmc.h:25), so the
dataset is parsed with maxs = 0 on both sides and the oracle is the only reference here."""
import numpy as np
import pytest

import gen_synthetic
import oracle_ref
import seriation_amd as sa

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def config5():
    X, hard = gen_synthetic.make(1024, 2048, 20261016)
    text = gen_synthetic.to_text(X, hard)
    return text if isinstance(text, bytes) else text.encode()


def test_config5_variant_is_hbm(config5):
    ds = sa.Dataset.parse(config5, maxs=0)
    assert (ds.N, ds.M) == (1024, 2048)
    with sa.Session(ds, [1]) as s:
        assert s.variant == "hbm" and s.kernel == "split"   # two workgroups per chain, 1024 taxa each
    with pytest.raises(sa.SrError):
        sa.Session(ds, [1], columns="lds")


def test_config5_parity(config5):
    """8 chains x (1 burn-in + 100 saved calls) = 1010 sweeps each against the oracle, bit for bit
    (oracle on 8 threads, ~25 s)."""
    from concurrent.futures import ThreadPoolExecutor
    ds = sa.Dataset.parse(config5, maxs=0)
    seeds = [1, 2, 3, 4, 5, 6, 7, 8]
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=1, sample_calls=100, keep_records=True)

    def one(s):
        o = oracle_ref.run_chain(config5, s, 1, 100, maxs=0)
        return o["rc"], o["rec_int"].copy(), o["rec_dbl"].copy()

    with ThreadPoolExecutor(8) as ex:
        ref = list(ex.map(one, seeds))
    for k, (s, (rc, oi, od)) in enumerate(zip(seeds, ref)):
        assert rc == 0
        np.testing.assert_array_equal(ri[k], oi, err_msg="seed %d" % s)
        assert np.array_equal(rd[k].view(np.uint64), od.view(np.uint64)), s
        assert summ[k]["consistent"] == 0


def test_config5_parity_one_workgroup(config5, monkeypatch):
    """The one-workgroup HBM-column kernel (two taxa per thread; what more than 128 chains per GPU
    run) on the same data: 8 chains x (1 + 10) calls against the oracle."""
    from concurrent.futures import ThreadPoolExecutor
    monkeypatch.setenv("SR_SPLIT", "0")
    ds = sa.Dataset.parse(config5, maxs=0)
    seeds = [11, 12, 13, 14, 15, 16, 17, 18]
    with sa.Session(ds, seeds[:1]) as s:
        assert s.kernel == "single"
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=1, sample_calls=10, keep_records=True)

    def one(s):
        o = oracle_ref.run_chain(config5, s, 1, 10, maxs=0)
        return o["rc"], o["rec_int"].copy(), o["rec_dbl"].copy()

    with ThreadPoolExecutor(8) as ex:
        ref = list(ex.map(one, seeds))
    for k, (s, (rc, oi, od)) in enumerate(zip(seeds, ref)):
        assert rc == 0
        np.testing.assert_array_equal(ri[k], oi, err_msg="seed %d" % s)
        assert np.array_equal(rd[k].view(np.uint64), od.view(np.uint64)), s
