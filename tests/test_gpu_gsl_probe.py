"""Probe the GPU box for a real GNU Scientific Library and, if one is there, pin the oracle's GSL 2.6
restatement (oracle/om_gsl.h) against it word for word (VERDICT r03 Next #6).

The reference links libgsl.so.25 (GSL 2.6) and draws c and d through gsl_ran_beta -> gsl_ran_gamma ->
gsl_ran_gaussian_ziggurat on gsl_rng_mt19937 (mcmc.c:751-765).  Neither this container nor the
reference holds GSL, so that stream is "parity unpinned" unless the box has the library.  Nothing is
installed: the test looks the library up with ctypes.util.find_library and the usual sonames, skips
with the probe's result when it is absent, and otherwise compares raw words, uniforms, uniform_int,
gaussian_ziggurat, gamma and beta draws for seeds 1..4 (and the shapes the sampler uses: 1 + counts).
The probe result is written to gpurun_out/gsl_probe.json when that directory exists.
"""
import ctypes
import ctypes.util
import json
import os

import numpy as np
import pytest

import oracle_ref

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SONAMES = ["libgsl.so.25", "libgsl.so.27", "libgsl.so.23", "libgsl.so"]


def _probe():
    found = {"find_library": ctypes.util.find_library("gsl"), "cblas": ctypes.util.find_library("gslcblas")}
    cands = ([found["find_library"]] if found["find_library"] else []) + SONAMES
    for name in cands:
        try:
            if found["cblas"]:
                ctypes.CDLL(found["cblas"], mode=ctypes.RTLD_GLOBAL)
            else:
                for cb in ("libgslcblas.so.0", "libgslcblas.so"):
                    try:
                        ctypes.CDLL(cb, mode=ctypes.RTLD_GLOBAL)
                        break
                    except OSError:
                        pass
            lib = ctypes.CDLL(name)
            found["loaded"] = name
            return lib, found
        except OSError as e:
            found.setdefault("errors", []).append("%s: %s" % (name, e))
    return None, found


def _record(found):
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "gsl_probe.json"), "w") as fh:
            json.dump(found, fh, indent=1)


def test_gsl_stream_pinned_or_absence_recorded():
    lib, found = _probe()
    if lib is None:
        found["result"] = "absent: no libgsl on this box; the GSL gamma/ziggurat stream stays parity unpinned"
        _record(found)
        pytest.skip(found["result"])
    lib.gsl_rng_alloc.restype = ctypes.c_void_p
    lib.gsl_rng_alloc.argtypes = [ctypes.c_void_p]
    lib.gsl_rng_set.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
    lib.gsl_rng_free.argtypes = [ctypes.c_void_p]
    lib.gsl_rng_get.restype = ctypes.c_ulong
    lib.gsl_rng_get.argtypes = [ctypes.c_void_p]
    for fn in ("gsl_rng_uniform", "gsl_rng_uniform_pos"):
        getattr(lib, fn).restype = ctypes.c_double
        getattr(lib, fn).argtypes = [ctypes.c_void_p]
    lib.gsl_rng_uniform_int.restype = ctypes.c_ulong
    lib.gsl_rng_uniform_int.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
    lib.gsl_ran_gaussian_ziggurat.restype = ctypes.c_double
    lib.gsl_ran_gaussian_ziggurat.argtypes = [ctypes.c_void_p, ctypes.c_double]
    lib.gsl_ran_gamma.restype = ctypes.c_double
    lib.gsl_ran_gamma.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double]
    lib.gsl_ran_beta.restype = ctypes.c_double
    lib.gsl_ran_beta.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double]
    mt = ctypes.c_void_p.in_dll(lib, "gsl_rng_mt19937")
    kinds = [(0, 0, 0, lambda r: float(lib.gsl_rng_get(r))), (1, 0, 0, lib.gsl_rng_uniform),
             (2, 0, 0, lib.gsl_rng_uniform_pos), (3, 97, 0, lambda r: float(lib.gsl_rng_uniform_int(r, 97))),
             (4, 0, 0, lambda r: lib.gsl_ran_gaussian_ziggurat(r, 1.0)),
             (5, 1.0, 0, lambda r: lib.gsl_ran_gamma(r, 1.0, 1.0)), (5, 37.0, 0, lambda r: lib.gsl_ran_gamma(r, 37.0, 1.0)),
             (6, 1.0, 1.0, lambda r: lib.gsl_ran_beta(r, 1.0, 1.0)),   # Johnk's branch (both shapes <= 1)
             (6, 3.0, 260.0, lambda r: lib.gsl_ran_beta(r, 3.0, 260.0)),
             (6, 5200.0, 900.0, lambda r: lib.gsl_ran_beta(r, 5200.0, 900.0))]
    n = 4000
    report = []
    for seed in (1, 2, 3, 4):
        for kind, a, b, draw in kinds:
            r = lib.gsl_rng_alloc(mt)
            lib.gsl_rng_set(r, seed)
            got = np.array([draw(r) for _ in range(n)])
            lib.gsl_rng_free(r)
            ref, _ = oracle_ref.rng_stream(seed, kind, n, a, b)
            same = bool(np.array_equal(got.view(np.uint64), ref.view(np.uint64)))
            report.append({"seed": seed, "kind": kind, "a": a, "b": b, "equal": same})
    found["result"] = "present: %d of %d streams bit-equal" % (sum(r["equal"] for r in report), len(report))
    found["streams"] = report
    _record(found)
    bad = [r for r in report if not r["equal"]]
    assert not bad, bad
