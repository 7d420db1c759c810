"""Shape-specialised sweep kernels (SR_JIT=1; srk_jit_load in csrc/sr_device.hip): the kernel compiled
at session creation with the dataset's sites, taxa and hard-site count fixed at compile time gives the
same bits as the generic kernel and as the CPU oracle, on every kernel family it replaces (register
walks of 9 and 17 words, the LDS walk, many hard sites) and on the bench's own shape.  The HBM-column
kernels keep the generic build (specialising the split kernel measured 4.4 % slower,
profiles/r03z6_ab_jit.json).
"""
import os

import numpy as np
import pytest

import oracle_ref
import seriation_amd as sa
from test_gpu_edge import make_text

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
SYNTH = os.path.join(HERE, "golden", "datasets", "synth_256x512.txt")

# name, dataset text (None: the bench's synthetic 256 x 512), session keywords, extra environment
CASES = [
    ("bench-256x512", None, {}, {}),
    ("walk9-tb256", (96, 200, 5), {}, {}),
    ("walk17", (300, 130, 9), {}, {}),
    ("lds-walk", (600, 80, 7), {}, {}),
    ("nh40", (120, 70, 40), {}, {}),
    ("tb1024", (64, 700, 4), {}, {}),
]


def _text(spec):
    if spec is None:
        with open(SYNTH, "rb") as fh:
            return fh.read()
    N, M, nh = spec
    return make_text(N, M, nh, seed=N * 1000 + M)


def _records(monkeypatch, ds, seeds, jit, kw):
    monkeypatch.setenv("SR_JIT", "1" if jit else "0")
    with sa.Session(ds, seeds, **kw) as s:
        assert s.specialized == jit, "SR_JIT=%d but specialized=%s" % (jit, s.specialized)
        kernel = s.kernel
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=2, sample_calls=4, keep_records=True, **kw)
    return kernel, summ, ri, rd


@pytest.mark.parametrize("name,spec,kw,env", CASES, ids=[c[0] for c in CASES])
def test_specialized_equals_generic_and_oracle(monkeypatch, name, spec, kw, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    text = _text(spec)
    ds = sa.Dataset.parse(text, maxs=0)
    seeds = [3, 17]
    kg, sg, rig, rdg = _records(monkeypatch, ds, seeds, False, kw)
    kj, sj, rij, rdj = _records(monkeypatch, ds, seeds, True, kw)
    assert kg == kj
    for k, s in enumerate(seeds):
        np.testing.assert_array_equal(rij[k], rig[k], err_msg="%s seed %d" % (name, s))
        assert np.array_equal(rdj[k].view(np.uint64), rdg[k].view(np.uint64)), (name, s)
        o = oracle_ref.run_chain(text, s, 2, 4, maxs=0)
        assert o["rc"] == 0
        np.testing.assert_array_equal(rij[k], o["rec_int"], err_msg="%s seed %d vs oracle" % (name, s))
        assert np.array_equal(rdj[k].view(np.uint64), o["rec_dbl"].view(np.uint64)), (name, s)
        assert sj[k]["consistent"] == 0


def test_specialized_long_run_bench_shape(monkeypatch):
    """The bench's shape over 8 chains x 60 calls (600 sweeps): every saved sample of the specialised
    kernel equals the generic kernel's, and the acceptance and fallback counters agree."""
    with open(SYNTH, "rb") as fh:
        ds = sa.Dataset.parse(fh.read(), maxs=0)
    seeds = list(range(1, 9))
    out = {}
    for jit in (False, True):
        monkeypatch.setenv("SR_JIT", "1" if jit else "0")
        with sa.Session(ds, seeds, calls_per_launch=60) as s:
            assert s.specialized == jit
            s.run(60, save=True)
            ri, rd = s.fetch_records()
            cnt = [np.concatenate([s.accept_counts(k), s.fallback_counts(k)]) for k in range(len(seeds))]
        out[jit] = (ri, rd, np.array(cnt))
    np.testing.assert_array_equal(out[True][0], out[False][0])
    assert np.array_equal(out[True][1].view(np.uint64), out[False][1].view(np.uint64))
    np.testing.assert_array_equal(out[True][2], out[False][2])


@pytest.mark.parametrize("kw,env", [({"columns": "hbm"}, {}), ({"block_threads": 1024, "columns": "hbm"}, {"SR_SPLIT": "1"})],
                         ids=["hbm", "split"])
def test_hbm_columns_stay_generic(monkeypatch, kw, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("SR_JIT", "1")
    ds = sa.Dataset.parse(make_text(64, 1100, 6, seed=64 * 1000 + 1100), maxs=0)
    with sa.Session(ds, [1, 2], **kw) as s:
        assert s.variant == "hbm" and not s.specialized


def test_specialized_shards_compile_together(monkeypatch):
    """Two shards on one device (sr_run_chains_multi: one host thread and session each) create their
    sessions together and both compile the same new shape: same records as the generic single session."""
    text = make_text(70, 90, 3, seed=70 * 1000 + 90 + 1)   # a shape no other test compiles
    ds = sa.Dataset.parse(text, maxs=0)
    seeds = [2, 5, 8, 11]
    monkeypatch.setenv("SR_JIT", "0")
    _, (rig, rdg) = sa.run_chains(ds, seeds, burnin_calls=2, sample_calls=4, keep_records=True)
    monkeypatch.setenv("SR_JIT", "1")
    _, (rij, rdj) = sa.run_chains(ds, seeds, burnin_calls=2, sample_calls=4, keep_records=True, devices=[0, 0])
    np.testing.assert_array_equal(rij, rig)
    assert np.array_equal(rdj.view(np.uint64), rdg.view(np.uint64))
    with sa.Session(ds, seeds) as s:
        assert s.specialized
