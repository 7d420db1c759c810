"""The fast paths' fallbacks, exercised: the forced-fallback build (-DSR_FORCE_EXACT, built by
`make` as <pkg>/build/force/libseriation.so) routes every Gibbs draw, proposal decision and c/d
draw through the exact computation the fast paths certify against; its records must equal the
oracle's bit for bit (tests/fallback_parity.py, run in a child process so it loads that
library).  The product build's own fallback counters are checked here too."""
import os
import subprocess
import sys

import numpy as np
import pytest

import seriation_amd as sa

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
FORCE = os.path.join(os.path.dirname(HERE), "seriation-in-paleontological-data-using-mcmc_amd", "build", "force",
                     "libseriation.so")


def test_forced_fallback_build_bitexact():
    assert os.path.exists(FORCE), "forced-fallback library not built (make in the package directory)"
    env = dict(os.environ, SERIATION_LIB=FORCE)
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "fallback_parity.py")], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=600)
    print(r.stdout.decode())
    assert r.returncode == 0, r.stdout.decode()[-3000:]


def test_product_fallback_counters():
    """The product build certifies nearly every draw: fallbacks are rare but counted."""
    ds = sa.Dataset.load(os.path.join(HERE, "golden", "datasets", "g10s10.txt"))
    with sa.Session(ds, [1, 2, 3, 4], calls_per_launch=50) as s:
        s.run(50)
        fb = np.array([s.fallback_counts(k) for k in range(4)])
        acc = np.array([s.accept_counts(k) for k in range(4)])
    sweeps = 500
    assert (fb >= 0).all()
    assert (fb[:, 1] < 2 * ds.M * sweeps // 100).all(), fb      # < 1 % of the Gibbs draws
    assert (fb[:, 2] < sweeps // 4).all(), fb                    # small counts: ziggurat/gamma retries
    assert (acc[:, 0] == sweeps).all() and (acc[:, 1] == sweeps).all()
