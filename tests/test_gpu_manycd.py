"""manycd = 1 (mcmc_readmodel's flag, mcmc.h:40): per-taxon error rates.  Every sweep draws c_m for m = 0..M-1
from Beta(1 + f1_m, 1 + t0_m), then d_m from Beta(1 + f0_m, 1 + t1_m), one after another from the chain's
stream (mcmc.c:777-786, 807-816); every Gibbs draw, logl term and proposal delta then uses the taxon's own
c_m, d_m (mcmc.c:641-642, 949-950, 1212-1213, 1433-1434, 1628-1629).  The MCD kernels run the exact paths;
every saved sample -- a, b, pi, every taxon's c and d, loglik -- must equal the CPU oracle's bit for bit, on
LDS and HBM columns, one and several taxa per thread, through sessions, run_chains and checkpoints."""
import os

import numpy as np
import pytest

import oracle_ref
import seriation_amd as sa
from test_gpu_edge import make_text

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
DS = os.path.join(HERE, "golden", "datasets")


def _text(name):
    with open(os.path.join(DS, name), "rb") as fh:
        return fh.read()


def _check(text, seeds, tb, ts, **kw):
    ds = sa.Dataset.parse(text, maxs=0)
    summ, (ri, rd, rv) = sa.run_chains(ds, seeds, burnin_calls=tb, sample_calls=ts, keep_records=True, manycd=1, **kw)
    for k, s in enumerate(seeds):
        o = oracle_ref.run_chain(text, s, tb, ts, maxs=0, manycd=1)
        assert o["rc"] == 0
        np.testing.assert_array_equal(ri[k], o["rec_int"], err_msg="seed %d: a, b, pi" % s)
        assert np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64)), ("seed %d c0/d0/loglik" % s)
        assert np.array_equal(rv[k].view(np.uint64), o["rec_cdv"].view(np.uint64)), ("seed %d per-taxon c, d" % s)
        assert summ[k]["consistent"] == 0
        np.testing.assert_array_equal(np.array([summ[k]["exp_loglik"], summ[k]["exp_c"], summ[k]["exp_d"]]), o["exp"])
        assert len(np.unique(rv[k][-1][:ds.M])) > 1   # the taxa really carry their own c
    return ds


@pytest.mark.parametrize("name", ["g10s10.txt", "g5s5.txt", "g2s2.txt"])
def test_manycd_reference_datasets(name):
    _check(_text(name), [1, 2], tb=2, ts=4)


def test_manycd_hbm_columns():
    _check(make_text(90, 300, 6, seed=90300), [3, 4], tb=1, ts=3, columns="hbm")


def test_manycd_long_columns():
    """N = 1400 (HBM columns at 1024 threads: a layout that exists since round 5's block-shared hard-site tables)."""
    _check(make_text(1400, 150, 9, seed=1400150), [6], tb=1, ts=2)


def test_manycd_several_taxa_per_thread():
    """M > 1024: two taxa per thread (HBM columns, the one-workgroup kernel; no split chains for manycd)."""
    ds = _check(make_text(48, 1300, 4, seed=481300), [5], tb=1, ts=2)
    with sa.Session(ds, [5], manycd=1) as s:
        assert s.manycd and s.kernel == "single" and s.block_threads == 1024 and not s.specialized


def test_manycd_session_records_and_checkpoint(tmp_path):
    """Session API: fetch_cd_vectors equals the oracle's per-taxon records; a checkpoint (version 8: the per-taxon
    c, d and the buffered records) restores into a session that holds the first 3 records and continues exactly;
    restoring it as manycd = 0 is refused."""
    text = _text("g10s10.txt")
    ds = sa.Dataset.parse(text)
    seeds = [7, 8]
    with sa.Session(ds, seeds, calls_per_launch=6, manycd=1) as s:
        s.run(3, save=True)
        ck = str(tmp_path / "m.ck")
        s.checkpoint(ck)
        s.run(3, save=True)
        ri, rd = s.fetch_records()
        rv = s.fetch_cd_vectors()
    with pytest.raises(sa.SrError):
        sa.Session.restore(ds, ck)
    r = sa.Session.restore(ds, ck, calls_per_launch=6, manycd=1)
    r.run(3, save=True)
    ri2, rd2 = r.fetch_records()
    rv2 = r.fetch_cd_vectors()
    r.close()
    np.testing.assert_array_equal(ri2, ri)   # the checkpoint's 3 records, then the 3 continued ones
    assert np.array_equal(rd2.view(np.uint64), rd.view(np.uint64))
    with sa.Session.restore(ds, ck, calls_per_launch=6, manycd=1) as r3:   # the state API: every taxon's c, d
        st = r3.state(1)
        assert np.array_equal(st["cv"].view(np.uint64), rv[1, 2, :ds.M].view(np.uint64))
        assert np.array_equal(st["dv"].view(np.uint64), rv[1, 2, ds.M:].view(np.uint64))
    assert np.array_equal(rv2.view(np.uint64), rv.view(np.uint64))
    for k, sd in enumerate(seeds):
        o = oracle_ref.run_chain(text, sd, 0, 6, manycd=1)
        np.testing.assert_array_equal(ri[k], o["rec_int"])
        assert np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64))
        assert np.array_equal(rv[k].view(np.uint64), o["rec_cdv"].view(np.uint64))


def test_manycd_debug_check_every_call():
    """SR_F_DEBUG_CHECK (MCMCDEBUG) with per-taxon c, d: mcmc_consistent's loglik recount uses each taxon's own."""
    text = _text("g5s5.txt")
    ds = sa.Dataset.parse(text)
    summ, (ri, rd, rv) = sa.run_chains(ds, [9], burnin_calls=1, sample_calls=3, keep_records=True, manycd=1,
                                       debug_check=True)
    o = oracle_ref.run_chain(text, 9, 1, 3, manycd=1)
    np.testing.assert_array_equal(ri[0], o["rec_int"])
    assert np.array_equal(rv[0].view(np.uint64), o["rec_cdv"].view(np.uint64))
    assert summ[0]["consistent"] == 0


def test_manycd_batched_cli_matches_oracle(tmp_path):
    """python -m seriation_amd --manycd: the Chains tree of 3 chains, chain_data.csv lines with every taxon's
    own c and d, each equal to the oracle's records formatted as mcmc_save_chain does (mcmc.c:69-92)."""
    import math
    import subprocess
    import sys
    pkg = os.path.join(os.path.dirname(HERE), "seriation-in-paleontological-data-using-mcmc_amd")
    ds_path = os.path.join(DS, "g5s5.txt")
    r = subprocess.run([sys.executable, "-m", "seriation_amd", ds_path, "--chains", "3", "--burnin", "2", "--samples", "3",
                        "--seed-base", "21", "--root", str(tmp_path), "--manycd"], cwd=pkg, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    text = _text("g5s5.txt")
    ds = sa.Dataset.parse(text)
    M = ds.M
    for k in range(3):
        o = oracle_ref.run_chain(text, 21 + k, 2, 3, manycd=1)
        with open(os.path.join(str(tmp_path), "Chains", "chain_%02d" % k, "chain_data.csv")) as fh:
            lines = fh.read().splitlines()
        assert len(lines) == 3
        for t, ln in enumerate(lines):
            f = ln.split(",")
            assert f[3].split() == ["%.14f" % math.exp(v) for v in o["rec_cdv"][t][:M]]
            assert f[4].split() == ["%.14f" % math.exp(v) for v in o["rec_cdv"][t][M:]]
            assert f[5] == "%.14f" % o["rec_dbl"][t][2]
