"""The `mcmc` CLI contract (mcmc.c:102-210).

CPU: the oracle CLI's five output files have the reference's exact layout; the product
CLI fails loudly (exit 1) when no GPU is present -- there is no CPU fallback.
GPU: the product CLI's files are byte-identical to the oracle CLI's for the same seed.
"""
import os
import subprocess

import pytest

import oracle_ref
from seriation_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DS = os.path.join(ROOT, "tests", "golden", "datasets")
ORACLE_CLI = os.path.join(ROOT, "oracle", "build", "mcmc_oracle")
PRODUCT_CLI = os.path.join(os.path.dirname(L.LIB_PATH), "mcmc")
FILES = ["chain_data.csv", "exp_data.csv", "taxa.csv", "sites.csv", "hard_sites.csv"]


def run_cli(exe, cwd, dataset, args, seed, chain_dir):
    os.makedirs(os.path.join(cwd, "Chains", chain_dir), exist_ok=True)
    env = dict(os.environ, GSL_RNG_SEED=str(seed))
    with open(os.path.join(DS, dataset), "rb") as fin:
        p = subprocess.run([exe] + list(args), cwd=cwd, stdin=fin, env=env, capture_output=True, timeout=900)
    return p


def read_dir(cwd, chain_dir):
    out = {}
    for f in FILES:
        with open(os.path.join(cwd, "Chains", chain_dir, f), "rb") as fh:
            out[f] = fh.read()
    return out


def test_oracle_cli_format(tmp_path):
    oracle_ref.lib()
    if not os.path.exists(ORACLE_CLI):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    p = run_cli(ORACLE_CLI, str(tmp_path), "g10s10.txt", ["0", "2", "3"], 7, "chain_00")
    assert p.returncode == 0, p.stderr
    assert b"GSL_RNG_SEED=7" in p.stderr
    files = read_dir(str(tmp_path), "chain_00")
    N, M = 124, 139
    lines = files["chain_data.csv"].decode().splitlines()
    assert len(lines) == 3
    for ln in lines:
        f = ln.split(",")
        assert len(f) == 6
        assert len(f[0].split()) == M and len(f[1].split()) == M and len(f[2].split()) == N
        assert len(f[3].split()) == M and f[3].endswith(" ")
        assert sorted(map(int, f[2].split())) == list(range(N))
    ex = files["exp_data.csv"].decode()
    assert ex.startswith("exp_loglik,exp_c,exp_d\n") and not ex.endswith("\n")
    o = oracle_ref.run_chain(open(os.path.join(DS, "g10s10.txt"), "rb").read(), 7, 2, 3)
    assert ex.split("\n")[1] == "%.14f,%.14f,%.14f" % tuple(o["exp"])
    assert files["taxa.csv"].decode().splitlines()[0] == "a,b,c,d"
    assert len(files["taxa.csv"].decode().splitlines()) == M + 1
    assert files["sites.csv"].decode().splitlines()[1:] == [str(v) for v in o["rec_int"][-1][2 * M:]]
    hs = files["hard_sites.csv"].decode().splitlines()
    assert hs[0] == "i,pi_i" and len(hs) == 1 + 11


def test_product_cli_fails_loudly_without_gpu(tmp_path):
    if os.path.exists("/dev/kfd"):
        pytest.skip("GPU node: covered by the gpu tests")
    p = run_cli(PRODUCT_CLI, str(tmp_path), "g2s2.txt", ["3"], 1, "chain_03")
    assert p.returncode == 1
    assert p.stderr.strip()


def test_cli_usage_error(tmp_path):
    p = subprocess.run([PRODUCT_CLI, "1", "2"], cwd=str(tmp_path), capture_output=True, stdin=subprocess.DEVNULL)
    assert p.returncode == 1 and b"usage" in p.stderr


def _compare(tmp_path, dataset, args, seed, chain_dir):
    a, b = str(tmp_path / "oracle"), str(tmp_path / "product")
    pa = run_cli(ORACLE_CLI, a, dataset, args, seed, chain_dir)
    pb = run_cli(PRODUCT_CLI, b, dataset, args, seed, chain_dir)
    assert pa.returncode == 0, pa.stderr
    assert pb.returncode == 0, pb.stderr
    fa, fb = read_dir(a, chain_dir), read_dir(b, chain_dir)
    for f in FILES:
        assert fa[f] == fb[f], f
    assert os.path.exists(os.path.join(b, "mcmc_c.log"))
    # the reference's own stderr lines (GSL_RNG_SEED=..., mcmc_initab's zero-column notes, mcmc.c:457)
    # in the same order; the HIP runtime may add lines of its own
    assert ref_lines(pa.stderr) == ref_lines(pb.stderr)


def ref_lines(err):
    txt = err.decode() if isinstance(err, bytes) else err
    return [l for l in txt.splitlines() if l.startswith(("GSL_RNG_SEED=", "mcmc_"))]


def test_oracle_cli_zero_column_notes(tmp_path):
    """g2s2 has 3 all-zero columns: mcmc_readmodel's and mcmc_randomize's mcmc_initab
    (0 < nh < N) each print "mcmc_initab: zero column at %d, continuing." for them (mcmc.c:457)."""
    p = run_cli(ORACLE_CLI, str(tmp_path), "g2s2.txt", ["0", "1", "1"], 4, "chain_00")
    assert p.returncode == 0, p.stderr
    notes = [l for l in ref_lines(p.stderr) if l.startswith("mcmc_initab")]
    assert len(notes) == 6 and notes[:3] == notes[3:]
    assert all(l.startswith("mcmc_initab: zero column at ") and l.endswith(", continuing.") for l in notes)


@pytest.mark.gpu
@pytest.mark.parametrize("index,chain_dir", [("5", "chain_05"), ("42", "chain_42")])
def test_product_cli_byte_identical_g10s10(tmp_path, index, chain_dir):
    """chain-index form: defaults 1000 + 1000 calls, output dir named as mcmc.c:153-178."""
    _compare(tmp_path, "g10s10.txt", [index], int(index) + 100, chain_dir)


@pytest.mark.gpu
def test_product_cli_four_argument_form(tmp_path):
    _compare(tmp_path, "g10s10.txt", ["0", "20", "30"], 3, "chain_00")


@pytest.mark.gpu
def test_product_cli_g2s2_reference_defaults(tmp_path):
    """BASELINE config 1: g2s2, 1 chain, CLI defaults (1000 burn-in + 1000 saved calls)."""
    _compare(tmp_path, "g2s2.txt", ["7"], 1, "chain_07")


def test_product_cli_stderr_lines_on_fake_device(tmp_path):
    """The product CLI's initialisation runs on the host, so its reference stderr lines can be
    checked without a GPU: built against the host-memory fake device (tests/asan/srk_fake.c), it
    prints what the oracle CLI prints (GSL_RNG_SEED=..., the six zero-column notes of g2s2)."""
    pkg = os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd")
    r = subprocess.run(["make", "-s", "-C", pkg, "build/fake/mcmc"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    pa = run_cli(ORACLE_CLI, str(tmp_path / "o"), "g2s2.txt", ["0", "1", "1"], 3, "chain_00")
    pb = run_cli(os.path.join(pkg, "build", "fake", "mcmc"), str(tmp_path / "p"), "g2s2.txt", ["0", "1", "1"], 3,
                 "chain_00")
    assert pa.returncode == 0 and pb.returncode == 0, pb.stderr
    assert ref_lines(pa.stderr) == ref_lines(pb.stderr) and len(ref_lines(pb.stderr)) == 7


def test_oracle_cli_manycd_format(tmp_path):
    """`mcmc 1 Tburnin T` (manycd = 1, mcmc.c:118): every taxon carries its own c, d -- chain_data.csv's c and
    d fields (mcmc.c:86-90) and taxa.csv's columns differ between taxa, the oracle's records say the same."""
    oracle_ref.lib()
    p = run_cli(ORACLE_CLI, str(tmp_path), "g10s10.txt", ["1", "2", "3"], 7, "chain_00")
    assert p.returncode == 0, p.stderr
    files = read_dir(str(tmp_path), "chain_00")
    M = 139
    f = files["chain_data.csv"].decode().splitlines()[-1].split(",")
    assert len(set(f[3].split())) > 1 and len(set(f[4].split())) > 1
    o = oracle_ref.run_chain(open(os.path.join(DS, "g10s10.txt"), "rb").read(), 7, 2, 3, manycd=1)
    import math
    assert f[3].split() == ["%.14f" % math.exp(v) for v in o["rec_cdv"][-1][:M]]
    assert f[4].split() == ["%.14f" % math.exp(v) for v in o["rec_cdv"][-1][M:]]


def test_manycd_block_size_and_no_specialised_kernel():
    """manycd sessions run the generic 1024-thread kernels: any other block size is SR_EUNSUPPORTED before a
    device call, and no shape-specialised kernel exists for them (sr_specialize reports 0)."""
    import ctypes
    import seriation_amd as sa
    ds = sa.Dataset.load(os.path.join(DS, "g5s5.txt"))
    o = sa.core.make_opts(manycd=1, block_threads=512)
    h = ctypes.c_void_p()
    assert L.lib().sr_session_create(ctypes.byref(ds.c), sa.core.make_specs([1]), 1, ctypes.byref(o), ctypes.byref(h)) == \
        L.SR_EUNSUPPORTED
    o = sa.core.make_opts(manycd=1)
    assert L.lib().sr_specialize(ctypes.byref(ds.c), ctypes.byref(o)) == 0


@pytest.mark.gpu
def test_product_cli_manycd_byte_identical(tmp_path):
    """manycd = 1 through the drop-in CLI: the five files byte-identical to the oracle CLI's (per-taxon c, d in
    chain_data.csv and taxa.csv)."""
    _compare(tmp_path, "g10s10.txt", ["1", "5", "12"], 11, "chain_00")


# ---- GSL_RNG_TYPE (gsl_rng_env_setup, mcmc.c:591-592): mt19937 echoed and run, any other generator refused
RNG_TYPES = [(None, 0), ("mt19937", 0), ("ranlxd2", 1), ("no_such_rng", 1)]


def run_cli_env(exe, cwd, dataset, args, env_extra, chain_dir="chain_00"):
    os.makedirs(os.path.join(cwd, "Chains", chain_dir), exist_ok=True)
    env = {k: v for k, v in os.environ.items() if k != "GSL_RNG_TYPE"}
    env.update(env_extra)
    with open(os.path.join(DS, dataset), "rb") as fin:
        return subprocess.run([exe] + list(args), cwd=cwd, stdin=fin, env=env, capture_output=True, timeout=900)


def gsl_lines(err):
    """stderr lines of gsl_rng_env_setup and of the refusal (the HIP runtime may add lines of its own)"""
    txt = err.decode() if isinstance(err, bytes) else err
    keep = ("GSL_RNG_", "Valid generator types are:", " ")
    return [l for l in txt.splitlines() if l.startswith(keep) and not l.startswith("  HIP")]


def _fake_cli():
    pkg = os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd")
    r = subprocess.run(["make", "-s", "-C", pkg, "build/fake/mcmc"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return os.path.join(pkg, "build", "fake", "mcmc")


@pytest.mark.parametrize("rtype,code", RNG_TYPES)
def test_gsl_rng_type_oracle_and_fake_device(tmp_path, rtype, code):
    """unset / mt19937 run (mt19937 echoed as GSL_RNG_TYPE=mt19937 before the seed line); another GSL generator
    (ranlxd2) and an unknown name exit 1 before reading the dataset -- the oracle CLI and the product CLI (host
    layer on the fake device) print the same lines and return the same code."""
    if not os.path.exists(ORACLE_CLI):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    env = {"GSL_RNG_SEED": "5"}
    if rtype:
        env["GSL_RNG_TYPE"] = rtype
    pa = run_cli_env(ORACLE_CLI, str(tmp_path / "o"), "g2s2.txt", ["0", "1", "1"], env)
    pb = run_cli_env(_fake_cli(), str(tmp_path / "p"), "g2s2.txt", ["0", "1", "1"], env)
    assert pa.returncode == code and pb.returncode == code, (pa.stderr, pb.stderr)
    la, lb = gsl_lines(pa.stderr), gsl_lines(pb.stderr)
    assert la == lb
    if rtype == "mt19937":
        assert la[:2] == ["GSL_RNG_TYPE=mt19937", "GSL_RNG_SEED=5"]
    elif rtype is None:
        assert la[0] == "GSL_RNG_SEED=5"
    elif rtype == "ranlxd2":
        assert la == ["GSL_RNG_TYPE=ranlxd2: generator not available, only mt19937 (GSL's default) is implemented"]
    else:
        assert la[:2] == ["GSL_RNG_TYPE=no_such_rng not recognized", "Valid generator types are:"]
        assert "mt19937" in " ".join(la[2:]).split() and not any(l.startswith("GSL_RNG_SEED") for l in la)
    if code:
        assert not os.path.exists(os.path.join(str(tmp_path / "p"), "Chains", "chain_00", "chain_data.csv"))


def test_gsl_rng_type_library_refuses(monkeypatch):
    """the library entry points apply the same check: sr_rng_env_setup's codes, and sr_session_create refuses
    another generator before any device call (SR_EUNSUPPORTED / SR_EINVAL) for every session that samples
    MT19937's stream, whatever the device; Philox sessions (SR_F_RNG_PHILOX) are not refused."""
    import ctypes
    import seriation_amd as sa
    lib = L.lib()
    seed = ctypes.c_uint64(99)
    for rtype, want in [("mt19937", L.SR_OK), ("ranlxd2", L.SR_EUNSUPPORTED), ("bogus", L.SR_EINVAL)]:
        monkeypatch.setenv("GSL_RNG_TYPE", rtype)
        monkeypatch.setenv("GSL_RNG_SEED", "0x10")
        assert lib.sr_rng_env_setup(ctypes.byref(seed), 0) == want
        if want == L.SR_OK:
            assert seed.value == 16
        else:
            ds = sa.Dataset.load(os.path.join(DS, "g2s2.txt"))
            h = ctypes.c_void_p()
            o = sa.core.make_opts()
            assert lib.sr_session_create(ctypes.byref(ds.c), sa.core.make_specs([1]), 1, ctypes.byref(o),
                                         ctypes.byref(h)) == want
            # an opt-in Philox session samples no GSL stream: the variable does not refuse it (here it then
            # fails for want of a device, or runs on one)
            o = sa.core.make_opts(rng="philox")
            rc = lib.sr_session_create(ctypes.byref(ds.c), sa.core.make_specs([1]), 1, ctypes.byref(o), ctypes.byref(h))
            assert rc in (L.SR_OK, L.SR_EDEVICE), rc
            if rc == L.SR_OK:
                lib.sr_session_destroy(h)


@pytest.mark.gpu
@pytest.mark.parametrize("rtype,code", RNG_TYPES)
def test_gsl_rng_type_product_cli_gpu(tmp_path, rtype, code):
    """on the GPU: the same stderr lines and exit codes as the oracle CLI; the mt19937 run's files equal the
    unset run's (the same generator) and the oracle's."""
    env = {"GSL_RNG_SEED": "5"}
    if rtype:
        env["GSL_RNG_TYPE"] = rtype
    pa = run_cli_env(ORACLE_CLI, str(tmp_path / "o"), "g2s2.txt", ["0", "2", "3"], env)
    pb = run_cli_env(PRODUCT_CLI, str(tmp_path / "p"), "g2s2.txt", ["0", "2", "3"], env)
    assert pa.returncode == code and pb.returncode == code, (pa.stderr, pb.stderr)
    assert gsl_lines(pa.stderr) == gsl_lines(pb.stderr)
    if code == 0:
        fa, fb = read_dir(str(tmp_path / "o"), "chain_00"), read_dir(str(tmp_path / "p"), "chain_00")
        assert fa == fb
