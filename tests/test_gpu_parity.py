"""GPU parity: the HIP sampler (through the C ABI) against the CPU oracle, bit for bit.

Integers (a, b, pi every saved sample) must be identical; c, d and loglik must be
bitwise identical too (same deterministic libm, same expression order, -ffp-contract=off).
The north-star tolerance for the expected negative log-likelihood (1e-6 relative) is
therefore met with margin; tests assert exact equality.
"""
import os

import numpy as np
import pytest

import oracle_ref
import seriation_amd as sa

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
DS = os.path.join(HERE, "golden", "datasets")


def _text(name):
    with open(os.path.join(DS, name), "rb") as fh:
        return fh.read()


def test_device_math_bitexact():
    rng = np.random.default_rng(7)
    xs = np.concatenate([
        rng.uniform(-745.5, 710.0, 200000),
        rng.uniform(-33.0, 0.0, 200000),           # logtop arguments
        rng.uniform(-7.0, 0.0, 100000),            # c, d
        -0.5 * rng.normal(0, 3, 100000) ** 2,      # ziggurat exp(-x^2/2)
    ])
    ys = np.concatenate([
        rng.uniform(0.0, 1.0, 200000),
        rng.uniform(0.9, 1.0, 200000),             # log(1 - e^c)
        np.ldexp(rng.uniform(0.5, 1.0, 100000), rng.integers(-1070, 1000, 100000)),
        rng.uniform(0.0, 50.0, 100000),
    ])
    x = np.concatenate([xs, ys])
    e_ref, l_ref = oracle_ref.exp_log(x)
    import ctypes
    P = ctypes.POINTER(ctypes.c_double)
    e = np.zeros_like(x)
    l = np.zeros_like(x)
    rc = sa.lib().sr_device_selftest_math(0, x.ctypes.data_as(P), len(x), e.ctypes.data_as(P), l.ctypes.data_as(P))
    assert rc == 0
    ok_e = (e.view(np.uint64) == e_ref.view(np.uint64)) | (np.isnan(e) & np.isnan(e_ref))
    ok_l = (l.view(np.uint64) == l_ref.view(np.uint64)) | (np.isnan(l) & np.isnan(l_ref))
    assert ok_e.all(), x[~ok_e][:5]
    assert ok_l.all(), x[~ok_l][:5]


def _compare_chains(name, seeds, tb, ts, spc=10, cpl=0):
    text = _text(name)
    ds = sa.Dataset.parse(text)
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=tb, sample_calls=ts, sweeps_per_call=spc,
                                   keep_records=True, calls_per_launch=cpl)
    for k, s in enumerate(seeds):
        o = oracle_ref.run_chain(text, s, tb, ts, sweeps=spc)
        assert o["rc"] == 0
        for t in range(ts):
            if not np.array_equal(ri[k, t], o["rec_int"][t]):
                bad = np.nonzero(ri[k, t] != o["rec_int"][t])[0]
                raise AssertionError("chain %d (seed %d) sample %d: %d int mismatches, first at %s"
                                     % (k, s, t, len(bad), bad[:8]))
            assert np.array_equal(rd[k, t].view(np.uint64), o["rec_dbl"][t].view(np.uint64)), \
                ("chain %d sample %d cdl" % (k, t), rd[k, t], o["rec_dbl"][t])
        assert summ[k]["consistent"] == 0
        np.testing.assert_array_equal(np.array([summ[k]["exp_loglik"], summ[k]["exp_c"], summ[k]["exp_d"]]), o["exp"])
    return summ


def test_parity_g10s10_first_calls():
    _compare_chains("g10s10.txt", [1, 2, 3, 42], tb=0, ts=4)


def test_parity_g10s10_burnin():
    _compare_chains("g10s10.txt", [5, 255], tb=20, ts=10, cpl=7)


def test_parity_g2s2():
    _compare_chains("g2s2.txt", [1], tb=2, ts=3)


def test_parity_synth_256x512():
    _compare_chains("synth_256x512.txt", [1, 2], tb=1, ts=3)


_ORACLE = {}


def _oracle_runs(text, seeds, tb, ts):
    """The oracle's (rc, sha256 of the integer records, c/d/loglik records, exp_data) per seed, on 16 threads;
    kept for the second kernel build of the same case."""
    import hashlib
    from concurrent.futures import ThreadPoolExecutor
    key = (hashlib.sha256(text).hexdigest(), tuple(seeds), tb, ts)
    if key not in _ORACLE:
        def one(s):
            o = oracle_ref.run_chain(text, s, tb, ts, maxs=0)
            return (o["rc"], hashlib.sha256(np.ascontiguousarray(o["rec_int"], "<i4").tobytes()).hexdigest(),
                    o["rec_dbl"].copy(), np.asarray(o["exp"]).copy())

        with ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
            _ORACLE.clear()   # one case at a time: the 100-chain records are large
            _ORACLE[key] = list(ex.map(one, seeds))
    return _ORACLE[key]


def _run_build(ds, seeds, tb, ts, kernel):
    """sr_run_chains with the shape-specialised kernel (the default) or the generic one; asserts the build ran."""
    generic = kernel == "generic"
    with sa.Session(ds, seeds[:1], generic=generic) as s:
        assert s.specialized == (not generic), "%s leg: specialized=%s" % (kernel, s.specialized)
    return sa.run_chains(ds, seeds, burnin_calls=tb, sample_calls=ts, keep_records=True, generic=generic)


KERNELS = pytest.mark.parametrize("kernel", ["specialized", "generic"])


@KERNELS
def test_parity_config3_100_chains_200_calls(kernel):
    """BASELINE config 3's workload (synthetic 256x512, 100 chains) for 200 saved calls (2000
    sweeps) per chain: every saved sample of every chain against the oracle (run on 16 threads), on the
    default shape-specialised kernel (the benched one) and on the generic kernel."""
    import hashlib
    text = _text("synth_256x512.txt")
    ds = sa.Dataset.parse(text, maxs=0)
    seeds = list(range(1, 101))
    summ, (ri, rd) = _run_build(ds, seeds, 0, 200, kernel)
    ref = _oracle_runs(text, seeds, 0, 200)
    bad = []
    for k, (rc, dig, od, _) in enumerate(ref):
        assert rc == 0
        if hashlib.sha256(np.ascontiguousarray(ri[k], "<i4").tobytes()).hexdigest() != dig or \
                not np.array_equal(rd[k].view(np.uint64), od.view(np.uint64)):
            bad.append(k)
        assert summ[k]["consistent"] == 0
    assert not bad, "chains differing from the oracle: %s" % bad


@KERNELS
def test_parity_config3_reference_protocol(kernel):
    """The reference CLI's own protocol (tb = 1000 burn-in calls, then ts = 1000 saved calls, mcmc.c:
    140-185) at BASELINE config 3's size (synthetic 256x512): 16 chains, i.e. 20 000 sweeps each, well
    into the converged regime; every one of the 1000 saved samples of every chain and its exp_data
    summary against the oracle, bit for bit (oracle on 16 threads, ~30 s), on both kernel builds."""
    import hashlib
    text = _text("synth_256x512.txt")
    ds = sa.Dataset.parse(text, maxs=0)
    seeds = list(range(201, 217))
    summ, (ri, rd) = _run_build(ds, seeds, 1000, 1000, kernel)
    ref = _oracle_runs(text, seeds, 1000, 1000)
    bad = []
    for k, (rc, dig, od, oexp) in enumerate(ref):
        assert rc == 0
        if hashlib.sha256(np.ascontiguousarray(ri[k], "<i4").tobytes()).hexdigest() != dig or \
                not np.array_equal(rd[k].view(np.uint64), od.view(np.uint64)) or \
                not np.array_equal(np.array([summ[k]["exp_loglik"], summ[k]["exp_c"], summ[k]["exp_d"]]), oexp):
            bad.append(k)
        assert summ[k]["consistent"] == 0
    assert not bad, "chains differing from the oracle: %s" % bad
