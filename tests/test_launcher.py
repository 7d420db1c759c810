"""script.py-compatible launcher pieces that need no GPU (script.py:15-99)."""
import os

import numpy as np
import pytest

from seriation_amd import launcher


def reference_choose(vals_by_dir, k):
    """script.py:70-99 restated literally (list walk, np.std ddof=0, strict window)."""
    neg = list(vals_by_dir.values())
    lo = min(neg)
    sd = np.std(neg)
    y = sorted(x for x in neg if lo - sd < x < lo + sd)
    out = []
    for z in y[:k]:
        for d, x in vals_by_dir.items():
            if x == z:
                out.append(int(d.split("_")[1]))
    return sorted(out)


def test_choose_matches_reference_rule():
    rng = np.random.default_rng(4)
    for trial in range(50):
        n = int(rng.integers(2, 100))
        vals = {"chain_%02d" % i: float(np.round(rng.normal(1500, 30), int(rng.integers(0, 3))))
                for i in rng.permutation(n)}
        for k in (1, 2, 8):
            assert launcher.choose_from_values(vals, k) == reference_choose(vals, k)


def test_choose_quirks():
    # equal values map back to every chain holding them (may return more than k)
    vals = {"chain_00": 10.0, "chain_01": 10.0, "chain_02": 30.0, "chain_03": 11.0}
    assert launcher.choose_from_values(vals, 1) == [0, 1]
    assert launcher.choose_from_values(vals, 2) == [0, 0, 1, 1]
    # strict window: a value exactly one sigma away is excluded
    vals = {"chain_00": 0.0, "chain_01": 2.0}   # sigma = 1 -> window (-1, 1)
    assert launcher.choose_from_values(vals, 2) == [0]


def test_choose_chains_reads_exp_data(tmp_path):
    for i, v in enumerate([1500.5, 1490.25, 1600.0]):
        d = tmp_path / "Chains" / ("chain_%02d" % i)
        d.mkdir(parents=True)
        (d / "exp_data.csv").write_text("exp_loglik,exp_c,exp_d\n%.14f,0.01,0.5" % v)
    assert launcher.choose_chains(2, root=str(tmp_path)) == [0, 1]


def test_seed_generation_like_script_py():
    s = launcher.generate_random_seed()
    assert 0 <= int(s.strip()) <= 255
    old = []
    seeds = [launcher._unique_seed(old) for _ in range(20)]
    assert len(set(seeds)) == 20 and len(old) == 20
    assert all(0 <= x <= 255 for x in seeds)


def test_batched_cli_rejects_bad_flags(capsys):
    """Argument errors are reported before anything touches a GPU."""
    from seriation_amd.__main__ import main
    for argv in (["x.txt", "--chains", "0"], ["x.txt", "--thin", "0"], ["x.txt", "--chains", "300"]):
        with pytest.raises(SystemExit) as e:
            main(argv)
        assert e.value.code == 2


def test_choose_chains_equals_pandas_parsing(tmp_path):
    """script.py:76-96 reads each exp_data.csv with pd.read_csv (pandas' own float parser, here 2.x; the reference
    pinned 1.0.4, absent) and maps values back by float equality.  On a Chains/ tree the oracle CLI wrote (24 chains
    of g10s10, the reference's file format), launcher.choose_chains (Python float()) must select exactly the chains
    the reference's pandas code selects, and every exp_loglik must parse to the same double."""
    import subprocess
    pd = pytest.importorskip("pandas")
    here = os.path.dirname(os.path.abspath(__file__))
    cli = os.path.join(os.path.dirname(here), "oracle", "build", "mcmc_oracle")
    if not os.path.exists(cli):
        subprocess.check_call(["make", "-s", "-C", os.path.join(os.path.dirname(here), "oracle")])
    ds = os.path.join(here, "golden", "datasets", "g10s10.txt")
    for k in range(24):
        d = tmp_path / ("run%02d" % k)
        (d / "Chains" / "chain_00").mkdir(parents=True)
        with open(ds, "rb") as fin:
            subprocess.check_call([cli, "0", "2", "6"], cwd=str(d), stdin=fin, stderr=subprocess.DEVNULL,
                                  env=dict(os.environ, GSL_RNG_SEED=str(k + 1)))
        dst = tmp_path / "Chains" / ("chain_%02d" % k)
        dst.mkdir(parents=True)
        (dst / "exp_data.csv").write_bytes((d / "Chains" / "chain_00" / "exp_data.csv").read_bytes())

    def pandas_choose(k):   # script.py:70-99 with pd.read_csv, literally
        root = str(tmp_path / "Chains")
        neg = [pd.read_csv(os.path.join(root, cd, "exp_data.csv")).exp_loglik.to_list()[0] for cd in os.listdir(root)]
        lo, sd = min(neg), np.std(neg)
        y = sorted(x for x in neg if lo - sd < x < lo + sd)
        out = []
        for z in y[:k]:
            for cd in os.listdir(root):
                if pd.read_csv(os.path.join(root, cd, "exp_data.csv")).exp_loglik.to_list()[0] == z:
                    out.append(int(cd.split("_")[1]))
        return sorted(out)

    for cd in os.listdir(str(tmp_path / "Chains")):
        path = os.path.join(str(tmp_path / "Chains"), cd, "exp_data.csv")
        assert launcher._read_exp_loglik(path) == pd.read_csv(path).exp_loglik.to_list()[0], cd
    for k in (1, 2, 8):
        assert launcher.choose_chains(k, root=str(tmp_path)) == pandas_choose(k)
