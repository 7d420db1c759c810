"""ctypes access to the CPU oracle (oracle/build/liboracle.so) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "build", "liboracle.so")
_L = None
P = ctypes.POINTER


def lib():
    global _L
    if _L is None:
        _L = load(LIB)
    return _L


def use_variant(name):
    """Switch this process to another build of the oracle: "O0" = oracle/build/O0/liboracle.so
    (the reference-like -O0 CPU baseline of bench.py)."""
    global _L
    _L = load(os.path.join(ORACLE_DIR, "build", name, "liboracle.so"))


def load(path):
    if not os.path.exists(path):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    L = ctypes.CDLL(path)
    L.oracle_parse.restype = ctypes.c_int
    L.oracle_parse.argtypes = [ctypes.c_char_p, ctypes.c_long, ctypes.c_int, P(ctypes.c_int), P(ctypes.c_int),
                               P(ctypes.c_int), P(ctypes.c_int32), P(ctypes.c_int32)]
    L.oracle_run_chain.restype = ctypes.c_int
    L.oracle_run_chain.argtypes = [ctypes.c_char_p, ctypes.c_long, ctypes.c_int, ctypes.c_ulong, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   P(ctypes.c_int32), P(ctypes.c_double), P(ctypes.c_int32), P(ctypes.c_double),
                                   P(ctypes.c_double), P(ctypes.c_longlong), P(ctypes.c_ulonglong)]
    L.oracle_run_chain_v.restype = ctypes.c_int
    L.oracle_run_chain_v.argtypes = [ctypes.c_char_p, ctypes.c_long, ctypes.c_int, ctypes.c_ulong, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     P(ctypes.c_int32), P(ctypes.c_double), P(ctypes.c_int32), P(ctypes.c_double),
                                     P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_longlong), P(ctypes.c_ulonglong)]
    L.oracle_auxa_pick.restype = ctypes.c_int
    L.oracle_auxa_pick.argtypes = [P(ctypes.c_int32), ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                   ctypes.c_double, P(ctypes.c_double)]
    L.oracle_auxa_boundary.restype = ctypes.c_double
    L.oracle_auxa_boundary.argtypes = [P(ctypes.c_int32), ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_int]
    L.oracle_delta_terms.restype = ctypes.c_double
    L.oracle_delta_terms.argtypes = [P(ctypes.c_int32), P(ctypes.c_int32), ctypes.c_long, ctypes.c_double, ctypes.c_double]
    L.oracle_mh_outcome.restype = ctypes.c_int
    L.oracle_mh_outcome.argtypes = [ctypes.c_double, ctypes.c_double]
    L.oracle_phase_seconds.restype = None
    L.oracle_phase_seconds.argtypes = [P(ctypes.c_double)]
    L.oracle_rng_stream.restype = None
    L.oracle_rng_stream.argtypes = [ctypes.c_ulong, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_long,
                                    P(ctypes.c_double), P(ctypes.c_ulonglong)]
    L.oracle_shuffle.argtypes = [ctypes.c_ulong, P(ctypes.c_int32), ctypes.c_long]
    L.oracle_choose.argtypes = [ctypes.c_ulong, P(ctypes.c_int32), ctypes.c_long, P(ctypes.c_int32), ctypes.c_long]
    L.oracle_exp_log.argtypes = [P(ctypes.c_double), ctypes.c_long, P(ctypes.c_double), P(ctypes.c_double)]
    L.oracle_set_rng.restype = None
    L.oracle_set_rng.argtypes = [ctypes.c_int]
    L.oracle_philox.restype = None
    L.oracle_philox.argtypes = [P(ctypes.c_uint32), P(ctypes.c_uint32), P(ctypes.c_uint32)]
    L.oracle_libm_mismatch.restype = None
    L.oracle_libm_mismatch.argtypes = [P(ctypes.c_double), ctypes.c_long, P(ctypes.c_long), P(ctypes.c_long)]
    return L


def _p(a, t):
    return a.ctypes.data_as(P(t)) if a is not None else None


def parse(text, maxs=2000):
    if isinstance(text, str):
        text = text.encode()
    N, M, nh = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    rc = lib().oracle_parse(text, len(text), maxs, ctypes.byref(N), ctypes.byref(M), ctypes.byref(nh), None, None)
    if rc:
        return rc, None, None
    X = np.zeros(N.value * M.value, np.int32)
    h = np.zeros(N.value, np.int32)
    lib().oracle_parse(text, len(text), maxs, ctypes.byref(N), ctypes.byref(M), ctypes.byref(nh),
                       _p(X, ctypes.c_int32), _p(h, ctypes.c_int32))
    return 0, X.reshape(N.value, M.value), h


def run_chain(text, seed, tb, ts, sweeps=10, check=0, maxs=2000, want_init=False, rng="mt", manycd=0):
    """Returns dict(rc, init (a,b,pi), init_cdl, rec_int [ts, 2M+N], rec_dbl [ts, 3], exp, acc, words, burnin_s,
    sample_s (wall seconds of the tb burn-in and the ts saved calls, timed inside the oracle)) and, for
    manycd=1 (per-taxon c, d: mcmc.c:777-786, 807-816), rec_cdv [ts, 2M] (every taxon's c then d per sample).
    rng="philox": the sampling phase on the Philox stream (the product's SR_F_RNG_PHILOX)."""
    if isinstance(text, str):
        text = text.encode()
    lib().oracle_set_rng(1 if rng == "philox" else 0)
    rc, X, h = parse(text, maxs)
    assert rc == 0, rc
    N, M = X.shape
    W = 2 * M + N
    init = np.zeros(W, np.int32)
    initd = np.zeros(3)
    ri = np.zeros(max(ts, 1) * W, np.int32)
    rd = np.zeros(max(ts, 1) * 3)
    ex = np.zeros(3)
    acc = np.zeros(7, np.int64)
    words = ctypes.c_ulonglong()
    cv = np.zeros(max(ts, 1) * 2 * M) if manycd else None
    rc = lib().oracle_run_chain_v(text, len(text), maxs, seed, 1 if manycd else 0, tb, ts, sweeps, check,
                                  _p(init, ctypes.c_int32), _p(initd, ctypes.c_double),
                                  _p(ri, ctypes.c_int32), _p(rd, ctypes.c_double), _p(cv, ctypes.c_double),
                                  _p(ex, ctypes.c_double), _p(acc, ctypes.c_longlong), ctypes.byref(words))
    ph = np.zeros(2)
    lib().oracle_phase_seconds(_p(ph, ctypes.c_double))
    out = dict(rc=rc, N=N, M=M, init=init, init_cdl=initd, rec_int=ri[:ts * W].reshape(ts, W),
               rec_dbl=rd[:ts * 3].reshape(ts, 3), exp=ex, acc=acc, words=words.value,
               burnin_s=float(ph[0]), sample_s=float(ph[1]))
    if manycd:
        out["rec_cdv"] = cv[:ts * 2 * M].reshape(ts, 2 * M)
    return out


def rng_stream(seed, kind, count, a=0.0, b=0.0):
    out = np.zeros(count)
    w = ctypes.c_ulonglong()
    lib().oracle_rng_stream(seed, kind, a, b, count, _p(out, ctypes.c_double), ctypes.byref(w))
    return out, w.value


def exp_log(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    e = np.zeros_like(x)
    l = np.zeros_like(x)
    lib().oracle_exp_log(_p(x, ctypes.c_double), len(x), _p(e, ctypes.c_double), _p(l, ctypes.c_double))
    return e, l


def auxa_pick(x, o, c, d, u, want_p=False):
    """mcmc_auxa + logtop + randompick over walk-order bits x (length L = the walk end) from limit o with the
    uniform u given: the pick (and the probabilities randompick subtracts)."""
    x = np.ascontiguousarray(x, np.int32)
    p = np.zeros(len(x) + 1) if want_p else None
    r = lib().oracle_auxa_pick(_p(x, ctypes.c_int32), len(x), int(o), float(c), float(d), float(u), _p(p, ctypes.c_double))
    return (r, p) if want_p else r


def auxa_boundary(x, o, c, d, i):
    """The smallest u in [0, 1] whose pick exceeds entry i (2.0: none)."""
    x = np.ascontiguousarray(x, np.int32)
    return lib().oracle_auxa_boundary(_p(x, ctypes.c_int32), len(x), int(o), float(c), float(d), int(i))


def delta_terms(dt0, dt1, c, d):
    """A proposal's delta summed as the reference does (per-taxon terms in taxon order)."""
    dt0 = np.ascontiguousarray(dt0, np.int32)
    dt1 = np.ascontiguousarray(dt1, np.int32)
    return lib().oracle_delta_terms(_p(dt0, ctypes.c_int32), _p(dt1, ctypes.c_int32), len(dt0), float(c), float(d))


def mh_outcome(delta, u):
    """1 accepted without drawing u (delta >= 0), 2 accepted with u drawn, 0 rejected (mcmc.c:492)."""
    return lib().oracle_mh_outcome(float(delta), float(u))
