"""End-to-end GPU checks (BASELINE.json configs 2 and the golden fixtures).

* every committed golden fixture (tests/golden/chains.json) reproduced by the HIP path;
* config 2: g10s10, 100 chains (seeds 1..100), 1000 burn-in + 1000 saved mcmc_sample
  calls -- every saved sample bit-identical to the oracle, exp_data identical;
* the statistical known answers of the reference (Docs/Report.pdf Table 1: g10s10 with 8
  selected chains: E[c] 0.0119, E[d] 0.5127, CORRMN 0.940; g5s5 and g10s2 with 2 each)
  within the acceptance band proposed in SURVEY.md §8c (+-0.002, +-0.03, +-0.02);
* the script.py launcher writes the same Chains/ tree as the oracle CLI.
"""
import hashlib
import json
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle_ref
import seriation_amd as sa
from golden.make_golden import record_digest
from seriation_amd import analysis, launcher

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
DS = os.path.join(HERE, "golden", "datasets")
with open(os.path.join(HERE, "golden", "chains.json")) as fh:
    CASES = json.load(fh)["cases"]


def _text(name):
    with open(os.path.join(DS, name), "rb") as fh:
        return fh.read()


@pytest.mark.parametrize("case", CASES, ids=lambda c: "%s-seed%d" % (c["dataset"], c["seed"]))
def test_golden_fixture(case):
    ds = sa.Dataset.parse(_text(case["dataset"]))
    summ, (ri, rd) = sa.run_chains(ds, [case["seed"]], burnin_calls=0, sample_calls=case["calls"],
                                   keep_records=True)
    assert [record_digest(r) for r in ri[0]] == case["sha256"]
    assert [[float(v).hex() for v in r] for r in rd[0]] == case["cdl_hex"]
    got = [summ[0]["exp_loglik"], summ[0]["exp_c"], summ[0]["exp_d"]]
    assert [float(v).hex() for v in got] == case["exp_hex"]


def _digest_all(rec_int):
    return hashlib.sha256(np.ascontiguousarray(rec_int, dtype="<i4").tobytes()).hexdigest()


@pytest.fixture(scope="module")
def config2():
    text = _text("g10s10.txt")
    ds = sa.Dataset.parse(text)
    seeds = list(range(1, 101))
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=1000, sample_calls=1000, keep_records=True)
    workers = min(16, os.cpu_count() or 1)

    def one(s):   # ctypes releases the GIL: the oracle chains run in parallel threads
        o = oracle_ref.run_chain(text, s, 1000, 1000)
        return o["rc"], _digest_all(o["rec_int"]), o["rec_dbl"].copy(), o["exp"].copy(), o["rec_int"][-1].copy()

    with ThreadPoolExecutor(workers) as ex:
        ref = list(ex.map(one, seeds))
    return ds, seeds, summ, ri, rd, ref


def test_config2_g10s10_100_chains_bitexact(config2):
    ds, seeds, summ, ri, rd, ref = config2
    bad = []
    for k, (rc, dig, rdbl, ex, last) in enumerate(ref):
        assert rc == 0
        if _digest_all(ri[k]) != dig:
            bad.append(k)
            continue
        assert np.array_equal(rd[k].view(np.uint64), rdbl.view(np.uint64)), k
        assert [summ[k]["exp_loglik"], summ[k]["exp_c"], summ[k]["exp_d"]] == list(ex), k
        assert summ[k]["consistent"] == 0
    assert not bad, "chains with integer mismatches: %s" % bad


def test_config2_statistical_known_answer(config2):
    ds, seeds, summ, ri, rd, ref = config2
    vals = {"chain_%02d" % k: s["exp_loglik"] for k, s in enumerate(summ)}
    chosen = launcher.choose_from_values(vals, 8)
    assert 1 <= len(chosen) <= 100
    ec, ed = analysis.exp_cd_from_records([rd[k] for k in chosen])
    corr = analysis.corr_mn_from_records([ri[k][:, 2 * ds.M:] for k in chosen])
    print("g10s10 selected %s: E[c]=%.4f E[d]=%.4f CORRMN=%.4f" % (chosen, ec, ed, corr))
    assert abs(ec - 0.0119) < 0.002
    assert abs(ed - 0.5127) < 0.03
    assert abs(corr - 0.940) < 0.02


def test_launcher_matches_oracle_cli(tmp_path):
    cli = os.path.join(os.path.dirname(HERE), "oracle", "build", "mcmc_oracle")
    seeds = [9, 10, 11]
    launcher.run_all_chains(os.path.join(DS, "g10s10.txt"), n_chains=3, seeds=seeds, devices=[0, 0],
                            burnin_calls=20, sample_calls=30, root=str(tmp_path / "gpu"), verbose=False)
    for k, s in enumerate(seeds):
        d = tmp_path / ("cpu%d" % k)
        (d / "Chains" / "chain_00").mkdir(parents=True)
        with open(os.path.join(DS, "g10s10.txt"), "rb") as fin:
            subprocess.check_call([cli, "0", "20", "30"], cwd=str(d), stdin=fin,
                                  env=dict(os.environ, GSL_RNG_SEED=str(s)), stderr=subprocess.DEVNULL)
        for f in ("chain_data.csv", "exp_data.csv", "taxa.csv", "sites.csv", "hard_sites.csv"):
            a = (d / "Chains" / "chain_00" / f).read_bytes()
            b = (tmp_path / "gpu" / "Chains" / ("chain_%02d" % k) / f).read_bytes()
            assert a == b, (k, f)


@pytest.mark.parametrize("name", ["g5s5", "g10s2"])
def test_table1_other_rows(name):
    """The other two rows of Report Table 1 (2 selected chains each).  With two selected chains
    the estimator's spread between seed sets exceeds the fixed band (the reference's seeds are
    random and unpublished), so the published row must lie within max(band, 3 sd) of the mean
    over 6 disjoint blocks of 100 chains (tools/table1.py run_row_spread)."""
    import table1
    r = table1.run_row_spread(name, blocks=6)
    for b in r["blocks"]:
        assert 1 <= len(b["selected"]) <= 100
    print(name, {k: r[k] for k in ("E_c", "E_d", "CORRMN")})
    assert all(r["within_spread"]), r


def test_batched_cli_matches_oracle_cli(tmp_path):
    """python -m seriation_amd (one session, many chains) writes the oracle CLI's files."""
    import sys
    pkg = os.path.join(os.path.dirname(HERE), "seriation-in-paleontological-data-using-mcmc_amd")
    rc = subprocess.call([sys.executable, "-m", "seriation_amd", os.path.join(DS, "g10s10.txt"), "--chains", "3",
                          "--burnin", "20", "--samples", "30", "--seed-base", "9", "--root", str(tmp_path / "gpu"),
                          "--select", "2"], cwd=pkg, stdout=subprocess.DEVNULL)
    assert rc == 0
    cli = os.path.join(os.path.dirname(HERE), "oracle", "build", "mcmc_oracle")
    for k in range(3):
        d = tmp_path / ("cpu%d" % k)
        (d / "Chains" / "chain_00").mkdir(parents=True)
        with open(os.path.join(DS, "g10s10.txt"), "rb") as fin:
            subprocess.check_call([cli, "0", "20", "30"], cwd=str(d), stdin=fin,
                                  env=dict(os.environ, GSL_RNG_SEED=str(9 + k)), stderr=subprocess.DEVNULL)
        for f in ("chain_data.csv", "exp_data.csv", "taxa.csv", "sites.csv", "hard_sites.csv"):
            assert (d / "Chains" / "chain_00" / f).read_bytes() == \
                (tmp_path / "gpu" / "Chains" / ("chain_%02d" % k) / f).read_bytes(), (k, f)


@pytest.mark.parametrize("sweeps", [1, 5, 23])
def test_thinning_bitexact(sweeps):
    """sweeps_per_call other than the reference's 10 (the --thin flag) against the oracle."""
    text = _text("g5s5.txt")
    ds = sa.Dataset.parse(text)
    seeds = [3, 4]
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=7, sample_calls=11, sweeps_per_call=sweeps,
                                   keep_records=True)
    for k, s in enumerate(seeds):
        o = oracle_ref.run_chain(text, s, 7, 11, sweeps=sweeps)
        assert o["rc"] == 0
        assert np.array_equal(ri[k], o["rec_int"]), (sweeps, s)
        assert np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64)), (sweeps, s)
        assert [summ[k]["exp_loglik"], summ[k]["exp_c"], summ[k]["exp_d"]] == list(o["exp"])
