"""Runs the certification self-tests (sr_device_selftest_gibbs / sr_device_selftest_decide) of whichever library
SERIATION_LIB names over the adversarial cases of tests/cert_cases.py -- TEST INFRASTRUCTURE.

    SERIATION_LIB=<pkg>/build/cert8/libseriation.so python tests/cert_run.py    # prints one JSON summary

tests/test_gpu_cert.py runs it in-process on the product library (every answer must equal the oracle's) and as a
child process on the negative-control build (margins / 2^8: some certified answer must be wrong)."""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
for _p in (HERE, os.path.join(os.path.dirname(HERE), "seriation-in-paleontological-data-using-mcmc_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import cert_cases  # noqa: E402

P = ctypes.POINTER
# (mode, N, column kinds, columns per kind): mode 0 / 1 = draw_fast_s<9> / <17> (register walks), 2 = draw_fast
# (LDS columns beyond N = 543), 3 = draw_fast with the HBM columns' byte tables and grouped checkpoints
GIBBS_SHAPES = [(0, 256, ("random", "tail", "steep"), 3), (0, 100, ("random", "tail"), 2),
                (1, 543, ("random", "tail", "steep"), 2), (1, 400, ("random", "tail"), 2),
                (2, 1024, ("random", "tail", "steep"), 2), (3, 1024, ("random", "tail", "steep"), 2),
                (3, 3000, ("random", "tail", "rise"), 1)]


def _ptr(a, t):
    return a.ctypes.data_as(P(t))


def run_gibbs(lib, mode, cs):
    n = cs["n"]
    out = np.zeros(5 * n, np.int32)
    fb = np.zeros(n, np.uint64)
    f = lib.sr_device_selftest_gibbs
    f.restype = ctypes.c_int
    rc = f(0, mode, cs["N"], n, _ptr(cs["P"], ctypes.c_uint32), _ptr(cs["pre"], ctypes.c_uint16),
           _ptr(cs["cd"], ctypes.c_double), _ptr(cs["o"], ctypes.c_int32), _ptr(cs["L"], ctypes.c_int32),
           _ptr(cs["rev"], ctypes.c_int32), _ptr(cs["u"], ctypes.c_double), _ptr(out, ctypes.c_int32),
           _ptr(fb, ctypes.c_uint64))
    if rc:
        raise RuntimeError("sr_device_selftest_gibbs returned %d" % rc)
    return out.reshape(n, 5), fb


def run_decide(lib, cs):
    out = np.zeros(cs["n"], np.int32)
    f = lib.sr_device_selftest_decide
    f.restype = ctypes.c_int
    rc = f(0, cs["n"], _ptr(cs["sums"], ctypes.c_int32), _ptr(cs["cd"], ctypes.c_double),
           _ptr(cs["uw"], ctypes.c_uint32), _ptr(out, ctypes.c_int32))
    if rc:
        raise RuntimeError("sr_device_selftest_decide returned %d" % rc)
    return out


def gibbs_summary(lib, mode, N, kinds, per_kind, seed=1):
    cs = cert_cases.gibbs_cases(N, kinds, seed + N + 7 * mode, per_kind)
    out, fb = run_gibbs(lib, mode, cs)
    pick = out[:, 0]
    wrong = np.nonzero(pick != cs["expected"])[0]
    cert = fb == 0
    bad_counts = 0
    for k in range(cs["n"]):
        col = cs["cols"][cs["cidx"][k]]
        want = cert_cases.pick_counts(col, N, bool(cs["rev"][k]), int(cs["o"][k]), int(pick[k]))
        bad_counts += tuple(int(v) for v in out[k, 1:]) != want
    return {"mode": mode, "N": N, "cases": int(cs["n"]), "certified": int(cert.sum()),
            "wrong": int(len(wrong)), "wrong_certified": int((~(pick == cs["expected"]) & cert).sum()),
            "wrong_counts": int(bad_counts),
            "first_wrong": [dict(u=float(cs["u"][k]).hex(), got=int(pick[k]), want=int(cs["expected"][k]),
                                 certified=bool(cert[k])) for k in wrong[:3]]}


def decide_summary(lib, seed=3):
    cs = cert_cases.decide_cases(seed)
    got = run_decide(lib, cs)
    decided = got != 3
    wrong = decided & (got != cs["expected"])
    return {"cases": int(cs["n"]), "decided": int(decided.sum()), "wrong": int(wrong.sum()),
            "first_wrong": [dict(got=int(got[k]), want=int(cs["expected"][k]), sums=cs["sums"][k].tolist(),
                                 c=float(cs["cd"][k, 0]).hex(), d=float(cs["cd"][k, 1]).hex(), uw=int(cs["uw"][k]))
                            for k in np.nonzero(wrong)[0][:3]]}


def run_all(lib):
    return {"gibbs": [gibbs_summary(lib, *s) for s in GIBBS_SHAPES], "decide": decide_summary(lib)}


if __name__ == "__main__":
    import seriation_amd as sa
    if len(sys.argv) > 1:   # more seeds (a soak beyond the test suite's fixed cases): cert_run.py SEED ...
        out = {}
        for sd in sys.argv[1:]:
            k = int(sd)
            out[sd] = {"gibbs": [gibbs_summary(sa.lib(), *g, seed=k) for g in GIBBS_SHAPES],
                       "decide": decide_summary(sa.lib(), seed=k + 100)}
        print(json.dumps(out))
    else:
        print(json.dumps(run_all(sa.lib())))
