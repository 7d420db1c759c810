"""The certification margins, tested where chain sampling cannot reach them (round-5 review item 2).

Every fast path of the sampler is exact because an analytic error bound holds: the Gibbs picks' REL / ABS
(mcmc.c:828-915 against draw_fast_s / draw_fast) and phase C's Eb (mcmc.c:492 / 569 / 637 against pc_classify /
pc_resolve).  tests/cert_cases.py places the inputs on those bounds -- u on the reference's own CDF boundaries and at
a ladder of distances up to twice the margin, including walks whose tails the reference clamps at e^LOGEPS, steep
walks, long walks the window trims (SR_QSPAN); proposals whose reference delta crosses 0 or log u, with term lists
whose sequential rounding is large -- and the device functions run on them through the library's self-test hooks.

* product build: every Gibbs pick (certified or through the exact fallback) and every decided proposal equals the
  oracle; the certified fraction is reported and must be substantial (the tests exercise the fast path, not only the
  fallback);
* negative control: the same library built with every margin divided by 2^8 (SR_CERT_SHIFT=8,
  <pkg>/build/cert8/libseriation.so, run in a child process) must answer some case wrongly -- proof that the cases
  can see an understated bound."""
import json
import os
import subprocess
import sys

import pytest

import cert_run
import seriation_amd as sa

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
CERT8 = os.path.join(os.path.dirname(HERE), "seriation-in-paleontological-data-using-mcmc_amd", "build", "cert8",
                     "libseriation.so")


@pytest.mark.parametrize("shape", cert_run.GIBBS_SHAPES, ids=lambda s: "mode%d-n%d" % (s[0], s[1]))
def test_gibbs_picks_on_the_boundaries(shape):
    r = cert_run.gibbs_summary(sa.lib(), *shape)
    print(json.dumps(r))
    assert r["wrong"] == 0, r
    assert r["wrong_counts"] == 0, r
    assert r["certified"] >= r["cases"] // 7, r   # the rungs beyond the margin are certified (the fast path's picks)


def test_phase_c_decisions_on_the_thresholds():
    r = cert_run.decide_summary(sa.lib())
    print(json.dumps(r))
    assert r["cases"] >= 500 and r["wrong"] == 0, r
    assert r["decided"] >= r["cases"] // 5, r


def test_shrunken_margins_are_caught():
    assert os.path.exists(CERT8), "negative-control library not built (make in the package directory)"
    env = dict(os.environ, SERIATION_LIB=CERT8)
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "cert_run.py")], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, timeout=600)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    r = json.loads(p.stdout.decode().strip().splitlines()[-1])
    print(json.dumps({"gibbs_wrong": [g["wrong_certified"] for g in r["gibbs"]], "decide_wrong": r["decide"]["wrong"]}))
    assert sum(g["wrong_certified"] for g in r["gibbs"]) > 0, r["gibbs"]
    assert r["decide"]["wrong"] > 0, r["decide"]
