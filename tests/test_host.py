"""Host-side pieces of the product against the oracle (CPU only, no device calls).

* exp/log (csrc/sr_math.h, the device's algorithm): glibc's own exp/log restated; bitwise
  equal to the oracle's om_libm.h, which is bitwise equal to this machine's glibc (which the
  reference links) on >= 10^7 inputs;
* sr_run_add / sr_run_sub (closed-form runs of equal sequential roundings used by the
  device for the clamped tails of mcmc_logtop / mcmc_randompick, mcmc.c:731-737,
  909-913) against the naive loops they replace;
* chain initialisation (mcmc_readmodel + mcmc_randomize + mcmc_init, mcmc.c:339-593,
  including its ran_choose / ran_shuffle RNG consumption) against the oracle.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle_ref
import seriation_amd as sa

HERE = os.path.dirname(os.path.abspath(__file__))
DS = os.path.join(HERE, "golden", "datasets")
PD = ctypes.POINTER(ctypes.c_double)
PI = ctypes.POINTER(ctypes.c_int32)


def host_exp_log(x):
    x = np.ascontiguousarray(x, np.float64)
    e, l = np.zeros_like(x), np.zeros_like(x)
    sa.lib().sr_host_exp_log(x.ctypes.data_as(PD), len(x), e.ctypes.data_as(PD), l.ctypes.data_as(PD))
    return e, l


def _inputs():
    rng = np.random.default_rng(5)
    return np.concatenate([
        rng.uniform(-745.5, 710.0, 100000), rng.uniform(-33.0, 0.0, 100000),
        rng.uniform(-7.0, 0.0, 50000), -0.5 * rng.normal(0, 3, 50000) ** 2,
        rng.uniform(0.0, 1.0, 100000), rng.uniform(0.9, 1.0, 100000),
        np.ldexp(rng.uniform(0.5, 1.0, 50000), rng.integers(-1070, 1000, 50000)),
        [0.0, -0.0, 1.0, np.inf, -np.inf, np.nan, 5e-324, 709.78, -745.13, 1e-300],
    ])


def _bits_equal(a, b):
    return (a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))


def test_exp_log_bitwise_equal_to_oracle():
    x = _inputs()
    e, l = host_exp_log(x)
    e0, l0 = oracle_ref.exp_log(x)
    assert _bits_equal(e, e0).all()
    assert _bits_equal(l, l0).all()


def _sampler_range_inputs(n_each, seed):
    """The argument ranges the sampler feeds exp/log (mcmc.c:644, 734, 757-760, 847-848, 1214,
    1261, 1441, 1636 and GSL's gamma/ziggurat)."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(np.log(.001), np.log(.8), n_each)
    return np.concatenate([
        rng.uniform(-33.0, 0.0, n_each),                       # logtop: max(LOGEPSILON, q - z)
        c,                                                      # exp(c), exp(d)
        1.0 - np.exp(c),                                        # log(1 - e^c)
        (rng.integers(1, 2 ** 32, n_each) / 2.0 ** 32),         # log(uniform_pos)
        -0.5 * rng.uniform(0.0, 10.0, n_each) ** 2,             # ziggurat exp(-x^2/2)
        rng.uniform(0.0, 1.0, n_each),                          # log of a beta draw
        rng.uniform(0.5, 40.0, n_each),                         # log(v) of gamma
    ])


def test_exp_log_equal_glibc_in_sampler_ranges():
    """om_exp/om_log (oracle) == glibc exp/log bit for bit on 10.5 M inputs from the sampler's
    argument ranges (the product's host copy is bitwise equal to the oracle above, the device
    copy in tests/test_gpu_parity.py)."""
    x = _sampler_range_inputs(1_500_000, 11)
    assert len(x) >= 10_000_000
    be, bl = ctypes.c_long(), ctypes.c_long()
    oracle_ref.lib().oracle_libm_mismatch(x.ctypes.data_as(PD), len(x), ctypes.byref(be), ctypes.byref(bl))
    assert (be.value, bl.value) == (0, 0)


def test_exp_log_equal_glibc_everywhere():
    """... and over the whole double range (normal and subnormal results, |x| >= 512 special
    cases, the near-1 log path, special values)."""
    rng = np.random.default_rng(12)
    x = np.concatenate([
        rng.uniform(-745.5, 710.0, 500000), rng.uniform(-1100, 1100, 100000),
        np.ldexp(rng.uniform(0.5, 1.0, 500000), rng.integers(-1074, 1024, 500000)),
        rng.uniform(0.93, 1.07, 500000), rng.uniform(-1e-3, 1e-3, 100000), _inputs(),
    ])
    be, bl = ctypes.c_long(), ctypes.c_long()
    oracle_ref.lib().oracle_libm_mismatch(x.ctypes.data_as(PD), len(x), ctypes.byref(be), ctypes.byref(bl))
    assert (be.value, bl.value) == (0, 0)


def test_run_add_matches_loop():
    rng = np.random.default_rng(9)
    lib = sa.lib()
    for _ in range(300):
        x = float(rng.uniform(0, 2) * 2.0 ** rng.integers(-40, 3))
        e = float(np.exp(-32.236191301916641) * rng.choice([1.0, rng.uniform(0.5, 3)]))
        L = int(rng.integers(1, 3000))
        ref = x
        for _k in range(L):
            ref = ref + e
        assert lib.sr_host_run_add(x, e, L) == ref


def test_run_sub_matches_loop():
    rng = np.random.default_rng(10)
    lib = sa.lib()
    for _ in range(300):
        r0 = float(rng.uniform(0, 1) * 2.0 ** rng.integers(-30, 1))
        p = float(rng.uniform(0.2, 4) * 2.0 ** rng.integers(-50, -20))
        L = int(rng.integers(1, 5000))
        ref, steps = r0, 0
        while steps < L:
            ref = ref - p
            steps += 1
            if ref <= 0.0:
                break
        r = ctypes.c_double(r0)
        got = lib.sr_host_run_sub(ctypes.byref(r), p, L)
        assert (got, r.value) == (steps, ref)


@pytest.mark.parametrize("name", ["g2s2.txt", "g10s10.txt", "g5s5.txt", "g10s2.txt", "synth_256x512.txt"])
def test_init_chain_matches_oracle(name):
    with open(os.path.join(DS, name), "rb") as fh:
        text = fh.read()
    ds = sa.Dataset.parse(text)
    for seed in (0, 1, 2, 77, 4357):
        a = np.zeros(ds.M, np.int32)
        b = np.zeros(ds.M, np.int32)
        pi = np.zeros(ds.N, np.int32)
        cdl = np.zeros(3)
        pos = ctypes.c_uint64()
        rc = sa.lib().sr_host_init_chain(ctypes.byref(ds.c), seed, a.ctypes.data_as(PI), b.ctypes.data_as(PI),
                                         pi.ctypes.data_as(PI), cdl.ctypes.data_as(PD), ctypes.byref(pos))
        assert rc == 0
        o = oracle_ref.run_chain(text, seed, 0, 0)
        M = ds.M
        np.testing.assert_array_equal(a, o["init"][:M])
        np.testing.assert_array_equal(b, o["init"][M:2 * M])
        np.testing.assert_array_equal(pi, o["init"][2 * M:])
        assert cdl.view(np.uint64).tolist() == o["init_cdl"].view(np.uint64).tolist()
        # hard sites keep their relative order under mcmc_randomize (mcmc.c:496-593)
        hp = pi[ds.hard.astype(bool)]
        assert (np.diff(hp) > 0).all()


@pytest.mark.parametrize("N,nh", [(40, 39), (41, 39), (12, 11), (30, 0), (30, 30)])
def test_init_chain_hard_sites_near_n(N, nh):
    """mcmc_randomize with nh close to N: the reference's scan of the chosen hard positions reads
    q[nh] one past the end once all nh are matched (mcmc.c:530, UB); host and oracle both stop at nh.
    nh = 0 only shuffles (no initab, mcmc.c:486-494); nh = N keeps the identity order.  The host
    initialisation equals the oracle's for several seeds, hard sites in their original order."""
    rng = np.random.default_rng(N * 100 + nh)
    M = 9
    X = (rng.random((N, M)) < 0.3).astype(int)
    X[:, 3] = 0   # a zero column
    hard = np.zeros(N, bool)
    hard[rng.choice(N, nh, replace=False)] = True
    text = ("%d %d\n" % (N, M) + "".join(" ".join(map(str, X[i])) + (" *" if hard[i] else "") + "\n"
                                        for i in range(N))).encode()
    ds = sa.Dataset.parse(text)
    assert ds.nh == nh
    for seed in (1, 5, 99):
        a = np.zeros(M, np.int32)
        b = np.zeros(M, np.int32)
        pi = np.zeros(N, np.int32)
        cdl = np.zeros(3)
        pos = ctypes.c_uint64()
        assert sa.lib().sr_host_init_chain(ctypes.byref(ds.c), seed, a.ctypes.data_as(PI), b.ctypes.data_as(PI),
                                           pi.ctypes.data_as(PI), cdl.ctypes.data_as(PD), ctypes.byref(pos)) == 0
        o = oracle_ref.run_chain(text, seed, 0, 0)
        np.testing.assert_array_equal(np.concatenate([a, b, pi]), o["init"])
        assert cdl.view(np.uint64).tolist() == o["init_cdl"].view(np.uint64).tolist()
        assert sorted(pi.tolist()) == list(range(N))
        assert (np.diff(pi[hard]) > 0).all()


def test_parallel_chain_init_equals_serial(tmp_path, monkeypatch):
    """session_new initialises the chains on several host threads (init_chains: each chain its own RNG and state
    slice); the state must be the serial loop's byte for byte.  sr_host_initial_checkpoint writes that state
    (mcmc.c:339-437, 592-708 restated) without a device: 1 thread against 7, 37 chains of g5s5 and of a synthetic
    700 x 300 matrix."""
    import ctypes
    import os
    import seriation_amd as sa
    from seriation_amd import _lib as L
    here = os.path.dirname(os.path.abspath(__file__))
    import gen_synthetic
    X, hard = gen_synthetic.make(700, 300, 5)
    for ds in (sa.Dataset.load(os.path.join(here, "golden", "datasets", "g5s5.txt")), sa.Dataset(X, hard)):
        specs = sa.core.make_specs(list(range(11, 48)))
        out = []
        for nt in ("1", "7"):
            monkeypatch.setenv("SR_INIT_THREADS", nt)
            p = tmp_path / ("init%s.srck" % nt)
            assert L.lib().sr_host_initial_checkpoint(ctypes.byref(ds.c), specs, 37, os.fsencode(str(p))) == 0
            out.append(p.read_bytes())
        assert out[0] == out[1]
