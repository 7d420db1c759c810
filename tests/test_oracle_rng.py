"""Pins for the oracle's GSL 2.6 restatement (oracle/om_gsl.h) -- CPU only.

GSL is a third-party dependency of the reference (mcmc.c:41-43 includes gsl_rng.h /
gsl_randist.h; the shipped binary links libgsl.so.25 = GSL 2.6) and is absent here, so
each piece is pinned against an independent source:
  * gsl_rng_mt19937: numpy.random.RandomState(seed) uses the same init_genrand seeding
    (GSL maps seed 0 to 4357) -> raw words must be identical;
  * uniform / uniform_pos / uniform_int / ran_shuffle / ran_choose: restated here in
    Python from GSL's published definitions and driven by the same raw stream;
  * gaussian_ziggurat / gamma / beta: distribution moments and a KS test (the exact
    GSL stream for these is "parity unpinned", see DESIGN.md "Oracle").
"""
import ctypes
import json
import os

import numpy as np
import pytest
from scipy import stats

import oracle_ref

HERE = os.path.dirname(os.path.abspath(__file__))


def raw(seed, n):
    w, words = oracle_ref.rng_stream(seed, 0, n)
    assert words == n
    return w.astype(np.uint64)


def numpy_mt(seed, n):
    rs = np.random.RandomState(4357 if seed == 0 else seed)
    return rs.randint(0, 2 ** 32, size=n, dtype=np.uint64)


@pytest.mark.parametrize("seed", [0, 1, 2, 42, 255, 4357, 2 ** 31 + 7])
def test_mt19937_matches_numpy(seed):
    np.testing.assert_array_equal(raw(seed, 3000), numpy_mt(seed, 3000))


def test_mt19937_known_answer():
    # MT19937 reference value: 10000th output for the default seed 5489 is 4123659995
    assert int(raw(5489, 10000)[-1]) == 4123659995


def test_mt19937_golden_fixture():
    with open(os.path.join(HERE, "golden", "mt19937.json")) as fh:
        g = json.load(fh)["words"]
    for s, words in g.items():
        np.testing.assert_array_equal(raw(int(s), len(words)), np.array(words, np.uint64))


def test_uniform_and_uniform_pos():
    w = raw(7, 5000)
    u, _ = oracle_ref.rng_stream(7, 1, 5000)
    np.testing.assert_array_equal(u, w / 4294967296.0)
    up, words = oracle_ref.rng_stream(7, 2, 4000)
    nz = w[w != 0][:4000] / 4294967296.0
    np.testing.assert_array_equal(up, nz)


def gsl_uniform_int(stream, n):
    """gsl_rng_uniform_int (GSL 2.6 rng.h): scale = range/n, reject k >= n."""
    scale = 0xFFFFFFFF // n
    while True:
        k = int(next(stream)) // scale
        if k < n:
            return k


@pytest.mark.parametrize("n", [1, 2, 3, 123, 1000, 2 ** 31 + 5, 0xFFFFFFFF])
def test_uniform_int(n):
    count = 2000
    got, words = oracle_ref.rng_stream(11, 3, count, float(n))
    stream = iter(raw(11, words))
    exp = [gsl_uniform_int(stream, n) for _ in range(count)]
    np.testing.assert_array_equal(got.astype(np.int64), np.array(exp, np.int64))


def test_shuffle():
    for n in (1, 2, 5, 124, 501):
        base = np.arange(n, dtype=np.int32)
        oracle_ref.lib().oracle_shuffle(3, base.ctypes.data_as(oracle_ref.P(oracle_ref.ctypes.c_int32)), n)
        stream = iter(raw(3, 10 * n + 10))
        ref = list(range(n))
        for i in range(n - 1, 0, -1):          # gsl_ran_shuffle (randist/shuffle.c)
            j = gsl_uniform_int(stream, i + 1)
            ref[i], ref[j] = ref[j], ref[i]
        assert base.tolist() == ref


def test_choose():
    import ctypes
    for n, k in ((10, 3), (124, 113), (526, 511), (7, 7)):
        src = np.arange(100, 100 + n, dtype=np.int32)
        dest = np.zeros(k, np.int32)
        P = oracle_ref.P(ctypes.c_int32)
        oracle_ref.lib().oracle_choose(5, dest.ctypes.data_as(P), k, src.ctypes.data_as(P), n)
        stream = iter(raw(5, n + 1))
        ref, j = [], 0
        for i in range(n):                     # gsl_ran_choose (randist/shuffle.c)
            if j >= k:
                break
            if (n - i) * (int(next(stream)) / 4294967296.0) < k - j:
                ref.append(int(src[i]))
                j += 1
        assert dest.tolist() == ref


def test_gaussian_ziggurat_distribution():
    z, _ = oracle_ref.rng_stream(17, 4, 200000)
    assert abs(z.mean()) < 0.01 and abs(z.var() - 1) < 0.015
    assert stats.kstest(z, "norm").pvalue > 1e-3


@pytest.mark.parametrize("a", [1.0, 1.5, 3.0, 17.0, 250.0])
def test_gamma_moments(a):
    g, _ = oracle_ref.rng_stream(23, 5, 100000, a)
    assert (g > 0).all()
    assert abs(g.mean() - a) < 0.02 * a + 0.02
    assert abs(g.var() - a) < 0.06 * a + 0.06


@pytest.mark.parametrize("a,b", [(1.0, 1.0), (2.0, 120.0), (60.0, 40.0), (300.0, 8.0)])
def test_beta_moments(a, b):
    x, _ = oracle_ref.rng_stream(29, 6, 100000, a, b)
    mean = a / (a + b)
    var = a * b / ((a + b) ** 2 * (a + b + 1))
    assert ((x >= 0) & (x <= 1)).all()
    assert abs(x.mean() - mean) < 5 * np.sqrt(var / len(x)) + 1e-12
    assert stats.kstest(x, "beta", args=(a, b)).pvalue > 1e-3


def test_beta_johnk_branch_exact():
    """gsl_ran_beta takes Johnk's method when both shapes are <= 1 (GSL 2.6 randist/beta.c); the
    sampler reaches it with shapes (1, 1) (both counts 0).  Then pow(U, 1) = U, so the draw is
    U / (U + V) for the first uniform_pos pair with U + V <= 1 -- restated here over the raw stream."""
    count = 3000
    x, words = oracle_ref.rng_stream(31, 6, count, 1.0, 1.0)
    stream = iter(raw(31, words + 4))

    def upos():
        while True:
            w = int(next(stream))
            if w:
                return w / 4294967296.0
    exp = []
    for _ in range(count):
        while True:
            u, v = upos(), upos()
            if u + v <= 1.0:
                exp.append(u / (u + v))
                break
    np.testing.assert_array_equal(x, np.array(exp))


# ---- the opt-in Philox stream (SR_F_RNG_PHILOX) ----------------------------------------------
# Philox4x32-10 known answers (Random123's published kat_vectors for philox4x32_10)
PHILOX_KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


def _u32(v):
    return (ctypes.c_uint32 * len(v))(*v)


def test_philox_known_answers_oracle_and_product():
    import seriation_amd as sa
    for ctr, key, want in PHILOX_KAT:
        o1, o2 = (ctypes.c_uint32 * 4)(), (ctypes.c_uint32 * 4)()
        oracle_ref.lib().oracle_philox(_u32(ctr), _u32(key), o1)
        sa.lib().sr_host_philox(_u32(ctr), _u32(key), o2)
        assert tuple(o1) == want and tuple(o2) == want


def test_mt_untemper_inverts_tempering():
    """The Philox mode stores untempered words in the MT ring (every read site tempers)."""
    import seriation_amd as sa
    x = np.random.default_rng(5).integers(0, 2 ** 32, 200000, dtype=np.uint64).astype(np.uint32)
    x = np.concatenate([x, np.array([0, 1, 0xffffffff, 0x80000000], np.uint32)])
    un, rt = np.zeros_like(x), np.zeros_like(x)
    P = ctypes.POINTER(ctypes.c_uint32)
    sa.lib().sr_host_mt_untemper(x.ctypes.data_as(P), len(x), un.ctypes.data_as(P), rt.ctypes.data_as(P))
    assert np.array_equal(rt, x)
    assert not np.array_equal(un, x)


def test_oracle_philox_chain_runs_consistent_and_differs():
    text = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "datasets", "g5s5.txt"), "rb").read()
    a = oracle_ref.run_chain(text, 3, 5, 5, check=1, rng="philox")
    b = oracle_ref.run_chain(text, 3, 5, 5, check=1)
    assert a["rc"] == 0 and b["rc"] == 0
    assert np.array_equal(a["init"], b["init"])          # initialisation stays MT19937
    assert not np.array_equal(a["rec_int"], b["rec_int"])
    c = oracle_ref.run_chain(text, 3, 5, 5, rng="philox")
    assert np.array_equal(a["rec_int"], c["rec_int"])    # deterministic per seed
