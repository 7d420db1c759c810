"""The opt-in counter-based stream (SR_F_RNG_PHILOX; north_star "Philox state per lane").

Not the reference's generator, so it is pinned two ways: bit-exact against the oracle running the
same Philox4x32-10 stream (tests/oracle_ref.py rng="philox"; the Philox function itself is pinned by
published known answers in tests/test_oracle_rng.py), and statistically against the reference's
only known answer, Docs/Report.pdf Table 1 (g10s10 row, the +-0.002 / +-0.03 / +-0.02 band)."""
import os

import numpy as np
import pytest

import oracle_ref
import seriation_amd as sa

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(HERE, "golden", "datasets")


@pytest.mark.parametrize("name,seeds,tb,ts", [("g10s10.txt", [1, 2, 3], 5, 10), ("g5s5.txt", [4, 0], 3, 8),
                                              ("synth_256x512.txt", [1, 2], 1, 3)])
def test_philox_parity_with_oracle(name, seeds, tb, ts):
    text = open(os.path.join(DATA, name), "rb").read()
    ds = sa.Dataset.parse(text, maxs=0)
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=tb, sample_calls=ts, keep_records=True, rng="philox")
    mt, _ = sa.run_chains(ds, seeds[:1], burnin_calls=tb, sample_calls=ts, rng="mt")
    assert mt[0]["exp_loglik"] != summ[0]["exp_loglik"]
    for k, s in enumerate(seeds):
        o = oracle_ref.run_chain(text, s, tb, ts, maxs=0, rng="philox")
        assert o["rc"] == 0
        np.testing.assert_array_equal(ri[k], o["rec_int"], err_msg="%s seed %d" % (name, s))
        assert np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64)), (name, s)
        assert summ[k]["consistent"] == 0


def test_philox_hbm_columns_and_checkpoint(tmp_path):
    text = open(os.path.join(DATA, "g10s10.txt"), "rb").read()
    ds = sa.Dataset.parse(text)
    seeds = [7, 8]
    with sa.Session(ds, seeds, calls_per_launch=12, columns="hbm", rng="philox") as s:
        s.run(12, save=True)
        ab_full, cdl_full = s.fetch_records()
    for k, seed in enumerate(seeds):
        o = oracle_ref.run_chain(text, seed, 0, 12, rng="philox")
        np.testing.assert_array_equal(ab_full[k].astype(np.int32), o["rec_int"])
    ck = str(tmp_path / "ph.srck")
    with sa.Session(ds, seeds, calls_per_launch=12, rng="philox") as s:
        s.run(4)
        s.checkpoint(ck)
    with pytest.raises(sa.SrError) as e:   # a Philox checkpoint restored as MT19937
        sa.Session.restore(ds, ck, calls_per_launch=12)
    assert e.value.code == sa._lib.SR_EINVAL
    r = sa.Session.restore(ds, ck, calls_per_launch=12, rng="philox")
    try:
        r.run(8, save=True)
        ab2, cdl2 = r.fetch_records()
    finally:
        r.close()
    assert np.array_equal(ab_full[:, 4:], ab2)
    assert np.array_equal(cdl_full[:, 4:].view(np.uint64), cdl2.view(np.uint64))


def test_philox_table1_g10s10_within_band():
    """Statistical gate: the Table 1 g10s10 row (100 chains x (1000 + 1000) calls, 8 selected by the
    one-sigma rule) on the Philox stream lands in the same band as the reference's published row."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
    import table1
    r = table1.run_row("g10s10", rng="philox")
    print({k: r[k] for k in ("E_c", "E_d", "CORRMN", "within_band")})
    assert all(r["within_band"]), r
