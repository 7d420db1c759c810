"""A third, independent reading of the reference's chain initialisation -- CPU only.

The product's host init (csrc/sr_host.c) and the oracle's (oracle/om_mcmc.c) both restate mcmc.c:339-593;
a misreading shared by the two would pass tests/test_host.py.  This file restates the same lines once more,
in plain Python straight from the reference text, on an RNG stream taken from numpy's MT19937
(RandomState: the same init_genrand seeding as gsl_rng_mt19937, seed 0 -> 4357) instead of either C
restatement of GSL:
  mcmc_readmodel  mcmc.c:339-437  header "N M", then per row the first M characters '0'/'1' (others
                                  skipped), a '*' after them marks a hard site; pi = identity
  mcmc_initab     mcmc.c:440-474  a = first occurrence in position order, b = last + 1; zero column -> 0, N
  mcmc_randomize  mcmc.c:477-578  nh = 0: gsl_ran_shuffle of pi only (no initab); 0 < nh < N:
                                  gsl_ran_choose of nh positions, the rest shuffled, hard sites take the
                                  chosen ones in order, then initab; nh = N: unchanged
  mcmc_count01    mcmc.c:651-708  t0, f0, t1, f1 per taxon; mcmc_logl mcmc.c:625-648 in m order
and requires a, b, pi and the initial loglik (bit for bit: Python's math.log / math.exp are glibc's) to
equal the product's sr_host_init_chain.
"""
import ctypes
import math
import os

import numpy as np
import pytest

import seriation_amd as sa

DS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "datasets")
PI = ctypes.POINTER(ctypes.c_int32)
PD = ctypes.POINTER(ctypes.c_double)


class MT:
    """gsl_rng_mt19937 words from numpy's MT19937 (seed 0 is GSL's 4357)."""

    def __init__(self, seed):
        self.rs = np.random.RandomState(4357 if seed == 0 else seed)

    def get(self):
        return int(self.rs.randint(0, 2 ** 32, dtype=np.uint64))

    def uniform(self):
        return self.get() / 4294967296.0

    def uniform_int(self, n):   # gsl_rng_uniform_int: scale = 0xffffffff / n, reject k >= n
        scale = 0xFFFFFFFF // n
        while True:
            k = self.get() // scale
            if k < n:
                return k


def readmodel(text):
    lines = text.decode().split("\n")
    N, M = map(int, lines[0].split()[:2])
    X = np.zeros((N, M), np.int64)
    hard = np.zeros(N, bool)
    for i in range(N):
        row = lines[1 + i]
        k, m = 0, 0
        while m < M:           # characters other than 0/1 are skipped
            ch = row[k]
            if ch in "01":
                X[i, m] = ch == "1"
                m += 1
            k += 1
        hard[i] = "*" in row[k:]
    return X, hard


def initab(X, rpi):
    N, M = X.shape
    a, b = np.zeros(M, np.int64), np.zeros(M, np.int64)
    for m in range(M):
        col = X[rpi, m]
        nz = np.nonzero(col)[0]
        if len(nz) == 0:
            a[m], b[m] = 0, N
        else:
            a[m], b[m] = nz[0], nz[-1] + 1
    return a, b


def shuffle(r, arr):        # gsl_ran_shuffle
    for i in range(len(arr) - 1, 0, -1):
        j = r.uniform_int(i + 1)
        arr[i], arr[j] = arr[j], arr[i]


def choose(r, k, src):      # gsl_ran_choose: selection sampling, order kept
    out, n = [], len(src)
    for i in range(n):
        if len(out) >= k:
            break
        if (n - i) * r.uniform() < k - len(out):
            out.append(src[i])
    return out


def init(text, seed):
    X, hard = readmodel(text)
    N, M = X.shape
    nh = int(hard.sum())
    pi = list(range(N))
    a, b = initab(X, np.arange(N))
    r = MT(seed)
    if nh == 0:
        shuffle(r, pi)            # a, b stay those of the identity order (mcmc.c:486-494)
    elif nh < N:
        q = choose(r, nh, list(range(N)))
        qs = set(q)
        p = [i for i in range(N) if i not in qs]
        shuffle(r, p)
        it_q, it_p = iter(q), iter(p)
        pi = [next(it_q) if hard[i] else next(it_p) for i in range(N)]
        rpi = np.argsort(pi)
        a, b = initab(X, rpi)
    pi = np.array(pi)
    c, d = math.log(.01), math.log(.3)
    loglik = 0.0
    for m in range(M):
        alive = (a[m] <= pi) & (pi < b[m])
        t1 = int((alive & (X[:, m] == 1)).sum())
        f0 = int((alive & (X[:, m] == 0)).sum())
        f1 = int((~alive & (X[:, m] == 1)).sum())
        t0 = int((~alive & (X[:, m] == 0)).sum())
        loglik += t0 * math.log(1. - math.exp(c)) + f0 * d + t1 * math.log(1. - math.exp(d)) + f1 * c
    return a, b, pi, loglik


@pytest.mark.parametrize("name", ["g2s2.txt", "g10s10.txt", "g5s5.txt", "g10s2.txt", "synth_256x512.txt"])
def test_host_init_equals_independent_restatement(name):
    with open(os.path.join(DS, name), "rb") as fh:
        text = fh.read()
    ds = sa.Dataset.parse(text, maxs=0)
    for seed in (0, 3, 4357):
        a = np.zeros(ds.M, np.int32)
        b = np.zeros(ds.M, np.int32)
        pi = np.zeros(ds.N, np.int32)
        cdl = np.zeros(3)
        pos = ctypes.c_uint64()
        assert sa.lib().sr_host_init_chain(ctypes.byref(ds.c), seed, a.ctypes.data_as(PI), b.ctypes.data_as(PI),
                                           pi.ctypes.data_as(PI), cdl.ctypes.data_as(PD), ctypes.byref(pos)) == 0
        ra, rb, rpi_, rl = init(text, seed)
        np.testing.assert_array_equal(a, ra, err_msg="%s seed %d: a" % (name, seed))
        np.testing.assert_array_equal(b, rb, err_msg="%s seed %d: b" % (name, seed))
        np.testing.assert_array_equal(pi, rpi_, err_msg="%s seed %d: pi" % (name, seed))
        assert cdl[2] == rl, (name, seed, cdl[2], rl)
