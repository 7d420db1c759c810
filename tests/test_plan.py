"""Every shape the C ABI accepts has a sweep kernel (CPU test: srk_plan, the library's own kernel choice, needs no
GPU).  Round 5 found sessions of more than ~1250 sites and more than 512 taxa without one: the HBM-column kernels
at 1024 threads kept 16 per-wave copies of the hard-site tables (64 N bytes of LDS); they share one copy now.
The only refusals are the documented ones: N > 4095, hard sites > N, and manycd below 1024 threads."""
import ctypes

import pytest

from seriation_amd import _lib as L

SITES = (2, 64, 256, 287, 288, 543, 600, 1024, 1250, 1300, 1700, 2000, 2500, 3000, 4000, 4095)
TAXA = (1, 100, 256, 512, 513, 1024, 1025, 1100, 2048, 2049, 5000, 40000)


def _plan():
    f = L.lib().srk_plan
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int] * 6 + [ctypes.c_void_p]
    return f


@pytest.mark.parametrize("manycd", [0, 1])
def test_every_shape_has_a_kernel(manycd):
    f = _plan()
    buf = ctypes.create_string_buffer(512)
    missing = []
    for N in SITES:
        for M in TAXA:
            for nh in (0, 12, 64, 65, 200):
                if nh > N:
                    continue
                for tb in ((0, 1024) if manycd else (0, 256, 512, 1024)):
                    if f(N, M, nh, tb, -1, manycd, buf) < 0:
                        missing.append((N, M, nh, tb))
    assert not missing, missing[:10]


def test_documented_refusals():
    f = _plan()
    buf = ctypes.create_string_buffer(512)
    assert f(4096, 512, 0, 0, -1, 0, buf) == L.SR_EUNSUPPORTED
    assert f(100, 512, 101, 0, -1, 0, buf) == L.SR_EUNSUPPORTED
    assert f(256, 512, 12, 512, -1, 1, buf) == L.SR_EUNSUPPORTED   # manycd: 1024 threads only
