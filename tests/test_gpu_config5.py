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


def test_config5_100_chains_split_grid(config5):
    """The benched config-5 grid: 100 chains on the split kernel = 13 block groups of 8 chains (blocks
    16 g + 8 h + x hold chain 8 g + x, half h), the last group ragged (4 chains).  (a) Sharded == unsharded:
    the 100-chain session's records equal those of two sessions of 37 and 63 chains (other groups, other
    ragged tails) for every chain; (b) one chain of every block group, the ragged group's first and last
    included, equals the oracle for 10 saved calls (oracle on 14 threads).  mcmc.c:918-996, 1127-1682."""
    from concurrent.futures import ThreadPoolExecutor
    ds = sa.Dataset.parse(config5, maxs=0)
    ids = list(range(100))
    calls = 10
    with sa.Session(ds, [i + 1 for i in ids], chain_ids=ids, calls_per_launch=calls) as s:
        assert s.kernel == "split"
        s.run(calls, save=True)
        ab, cdl = s.fetch_records()
    parts = []
    for lo, hi in ((0, 37), (37, 100)):
        with sa.Session(ds, [i + 1 for i in ids[lo:hi]], chain_ids=ids[lo:hi], calls_per_launch=calls) as s:
            assert s.kernel == "split"
            s.run(calls, save=True)
            parts.append(s.fetch_records())
    np.testing.assert_array_equal(np.concatenate([p[0] for p in parts]), ab)
    assert np.array_equal(np.concatenate([p[1] for p in parts]).view(np.uint64), cdl.view(np.uint64))
    picks = [0, 9, 17, 25, 34, 42, 50, 59, 67, 75, 84, 90, 96, 99]   # groups 0..12; 96 and 99 in the ragged group

    def one(i):
        o = oracle_ref.run_chain(config5, i + 1, 0, calls, maxs=0)
        return o["rc"], o["rec_int"].copy(), o["rec_dbl"].copy()

    with ThreadPoolExecutor(len(picks)) as ex:
        ref = list(ex.map(one, picks))
    assert sorted({i // 8 for i in picks}) == list(range(13))
    for i, (rc, ri, rdb) in zip(picks, ref):
        assert rc == 0
        assert np.array_equal(ab[i].astype(np.int32), ri), "chain %d: integers differ from the oracle" % i
        assert np.array_equal(cdl[i].view(np.uint64), rdb.view(np.uint64)), "chain %d: c/d/loglik differ" % i


def test_config5_converged_regime_equals_oracle_digests(config5):
    """Config 5 in the regime its rates are quoted at: 4 chains (seeds 1-4) under the reference CLI's protocol,
    1000 burn-in + 1000 saved calls (mcmc.c:140-185; 20 000 sweeps per chain), on the product's default config-5
    kernel (split chains, cooperative launch), against the committed oracle digests (tests/golden/config5.json,
    made by tests/golden/make_golden_c5.py: ~28 min of oracle time in the build container).  Every saved call's
    a||b||pi digest, c / d / loglik bits and the exp_data row must match -- the long-walk window trims (SR_QSPAN),
    the grouped f64 Gibbs checkpoints and the LDS checkpoints run at depth here, where the short parity tests
    above (101 calls) do not reach.  mcmc.c:918-996, 1127-1682."""
    import hashlib
    import json
    import os
    from golden.make_golden import record_digest
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "config5.json")) as fh:
        g = json.load(fh)
    assert g["dataset_sha256"] == hashlib.sha256(config5).hexdigest()
    ds = sa.Dataset.parse(config5, maxs=0)
    seeds = [ch["seed"] for ch in g["chains"]]
    with sa.Session(ds, seeds, calls_per_launch=g["saved_calls"]) as s:
        assert s.kernel == "split"
        for _ in range(g["burnin_calls"] // 50):
            s.run(50, save=False)
        for _ in range(g["saved_calls"] // 50):
            s.run(50, save=True)
        ab, cdl = s.fetch_records()
        rows = s.summaries()
    for k, ch in enumerate(g["chains"]):
        dig = [record_digest(r.astype(np.int32)) for r in ab[k]]
        bad = [i for i in range(len(dig)) if dig[i] != ch["sha256"][i]]
        assert not bad, "seed %d: integer state differs from saved call %d on" % (ch["seed"], bad[0])
        assert [[float(v).hex() for v in r] for r in cdl[k]] == ch["cdl_hex"], ch["seed"]
        assert [float(v).hex() for v in rows[k, 1:4]] == ch["exp_hex"], ch["seed"]
