"""Shape-specialised sweep kernels (the default for LDS-column sessions; csrc/sr_spec.c, srk_spec_load in
csrc/sr_device.hip): the kernel compiled for the dataset's sites, taxa and hard-site count gives the same
bits as the generic kernel and as the CPU oracle, on every kernel family it replaces (register walks of 9
and 17 words, the LDS walk, many hard sites) and on the bench's own shape.  The HBM-column kernels keep
the generic build (specialising the split kernel measured 4.4 % slower, profiles/r03z6_ab_jit.json).
A code object that does not load, or whose ABI record differs, leaves the generic kernel in place with a
message; shard threads compiling the same new shape together publish one object and all use it.
"""
import ctypes
import json
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import oracle_ref
import seriation_amd as sa
from test_gpu_edge import make_text

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd")
SYNTH = os.path.join(HERE, "golden", "datasets", "synth_256x512.txt")

# name, dataset text (None: the bench's synthetic 256 x 512), session keywords
CASES = [
    ("bench-256x512", None, {}),
    ("walk9-tb256", (96, 200, 5), {}),
    ("walk17", (300, 130, 9), {}),
    ("lds-walk", (600, 80, 7), {}),
    ("nh40", (120, 70, 40), {}),
    ("tb1024", (64, 700, 4), {}),
]


def _text(spec):
    if spec is None:
        with open(SYNTH, "rb") as fh:
            return fh.read()
    N, M, nh = spec
    return make_text(N, M, nh, seed=N * 1000 + M)


def _records(ds, seeds, generic, kw):
    with sa.Session(ds, seeds, generic=generic, **kw) as s:
        assert s.specialized == (not generic), "generic=%s but specialized=%s" % (generic, s.specialized)
        kernel = s.kernel
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=2, sample_calls=4, keep_records=True, generic=generic, **kw)
    return kernel, summ, ri, rd


@pytest.mark.parametrize("name,spec,kw", CASES, ids=[c[0] for c in CASES])
def test_specialized_equals_generic_and_oracle(name, spec, kw):
    text = _text(spec)
    ds = sa.Dataset.parse(text, maxs=0)
    seeds = [3, 17]
    kg, sg, rig, rdg = _records(ds, seeds, True, kw)
    kj, sj, rij, rdj = _records(ds, seeds, False, kw)
    assert kg == kj
    for k, s in enumerate(seeds):
        np.testing.assert_array_equal(rij[k], rig[k], err_msg="%s seed %d" % (name, s))
        assert np.array_equal(rdj[k].view(np.uint64), rdg[k].view(np.uint64)), (name, s)
        o = oracle_ref.run_chain(text, s, 2, 4, maxs=0)
        assert o["rc"] == 0
        np.testing.assert_array_equal(rij[k], o["rec_int"], err_msg="%s seed %d vs oracle" % (name, s))
        assert np.array_equal(rdj[k].view(np.uint64), o["rec_dbl"].view(np.uint64)), (name, s)
        assert sj[k]["consistent"] == 0


def test_environment_opt_out(monkeypatch):
    """SR_JIT=0 in the environment selects the generic kernel like SR_F_GENERIC_KERNEL."""
    ds = sa.Dataset.load(SYNTH, maxs=0)
    monkeypatch.setenv("SR_JIT", "0")
    with sa.Session(ds, [1]) as s:
        assert not s.specialized
    monkeypatch.delenv("SR_JIT")
    with sa.Session(ds, [1]) as s:
        assert s.specialized


def test_specialized_long_run_bench_shape():
    """The bench's shape over 8 chains x 60 calls (600 sweeps): every saved sample of the specialised
    kernel equals the generic kernel's, and the acceptance and fallback counters agree."""
    with open(SYNTH, "rb") as fh:
        ds = sa.Dataset.parse(fh.read(), maxs=0)
    seeds = list(range(1, 9))
    out = {}
    for generic in (True, False):
        with sa.Session(ds, seeds, calls_per_launch=60, generic=generic) as s:
            assert s.specialized == (not generic)
            s.run(60, save=True)
            ri, rd = s.fetch_records()
            cnt = [np.concatenate([s.accept_counts(k), s.fallback_counts(k)]) for k in range(len(seeds))]
        out[generic] = (ri, rd, np.array(cnt))
    np.testing.assert_array_equal(out[True][0], out[False][0])
    assert np.array_equal(out[True][1].view(np.uint64), out[False][1].view(np.uint64))
    np.testing.assert_array_equal(out[True][2], out[False][2])


@pytest.mark.parametrize("kw,env", [({"columns": "hbm"}, {}), ({"block_threads": 1024, "columns": "hbm"}, {"SR_SPLIT": "1"})],
                         ids=["hbm", "split"])
def test_hbm_columns_stay_generic(monkeypatch, kw, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ds = sa.Dataset.parse(make_text(64, 1100, 6, seed=64 * 1000 + 1100), maxs=0)
    with sa.Session(ds, [1, 2], **kw) as s:
        assert s.variant == "hbm" and not s.specialized


# child processes: each resolves its snapshot, cache and one-line notes afresh
SHARDS = textwrap.dedent("""
    import json, sys
    sys.path.insert(0, %r); sys.path.insert(0, %r)
    import numpy as np
    import seriation_amd as sa
    from test_gpu_edge import make_text
    ds = sa.Dataset.parse(make_text(70, 90, 3, seed=70 * 1000 + 90 + 1), maxs=0)
    seeds = [2, 5, 8, 11]
    _, (rig, rdg) = sa.run_chains(ds, seeds, burnin_calls=2, sample_calls=4, keep_records=True, generic=True)
    _, (rij, rdj) = sa.run_chains(ds, seeds, burnin_calls=2, sample_calls=4, keep_records=True, devices=[0, 0])
    same = bool(np.array_equal(rij, rig) and np.array_equal(rdj.view(np.uint64), rdg.view(np.uint64)))
    with sa.Session(ds, seeds) as s:
        spec = s.specialized
    print(json.dumps({"same": same, "specialized": spec}))
""" % (PKG, HERE))

PLANTED = textwrap.dedent("""
    import ctypes, json, sys
    sys.path.insert(0, %r)
    import seriation_amd as sa
    ds = sa.Dataset.load(sys.argv[1], maxs=0)
    buf = ctypes.create_string_buffer(4096)
    assert sa.lib().sr_spec_cache_path(ds.N, ds.M, ds.nh, 0, buf, 4096) == 0
    import os
    os.makedirs(os.path.dirname(buf.value), exist_ok=True)
    with open(buf.value, "wb") as fh:
        fh.write(sys.argv[2].encode())
    with sa.Session(ds, [1, 2]) as s:
        spec = s.specialized
    _, (ri, rd) = sa.run_chains(ds, [1, 2], burnin_calls=1, sample_calls=2, keep_records=True)
    print(json.dumps({"specialized": spec, "rec": ri.tolist()}))
""" % PKG)


def _child(code, env, *argv):
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, "-c", code] + list(argv), env=e, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1]), r.stderr


def test_specialized_shards_compile_together(tmp_path):
    """Two shards on one device (sr_run_chains_multi: one host thread and session each) create their sessions
    together and both compile the same new shape into an empty cache: one published code object, no
    leftovers, no fallback note, and the same records as the generic single session."""
    out, err = _child(SHARDS, {"SR_JIT_CACHE": str(tmp_path)})
    assert out["same"] and out["specialized"]
    files = os.listdir(tmp_path)
    assert len([f for f in files if f.endswith(".co")]) == 1, files
    assert not [f for f in files if f.endswith(".tmp")], files
    assert "unavailable" not in err, err


def test_bad_code_object_falls_back_to_generic(tmp_path):
    """A corrupt object under the session's own key: hipModuleLoad fails, one stderr line names it, and
    the session runs the generic kernel (same records as the oracle).  (A shape the library does not embed:
    the embedded ones never consult the cache.)"""
    text = make_text(120, 130, 9, seed=120130)
    path = tmp_path / "subject.txt"
    path.write_bytes(text)
    out, err = _child(PLANTED, {"SR_JIT_CACHE": str(tmp_path / "cache")}, str(path), "not a code object")
    assert out["specialized"] is False
    assert "did not load" in err and "hipModuleLoad" in err, err
    for k, s in enumerate([1, 2]):
        o = oracle_ref.run_chain(text, s, 1, 2)
        np.testing.assert_array_equal(np.array(out["rec"][k]), o["rec_int"])


EMBEDDED_RUN = textwrap.dedent("""
    import json, sys
    sys.path.insert(0, %r)
    import numpy as np
    import seriation_amd as sa
    ds = sa.Dataset.load(sys.argv[1], maxs=0)
    with sa.Session(ds, [4, 9]) as s:
        spec, emb = s.specialized, int(sa.lib().sr_session_spec_embedded(s.h))
    _, (ri, rd) = sa.run_chains(ds, [4, 9], burnin_calls=1, sample_calls=3, keep_records=True)
    print(json.dumps({"specialized": spec, "embedded": emb, "rec": ri.tolist(), "dbl": rd.view(np.uint64).tolist()}))
""" % PKG)


@pytest.mark.parametrize("name", ["synth_256x512.txt", "g10s10.txt"])
def test_embedded_kernel_needs_no_compiler_or_cache(tmp_path, name):
    """The bench matrix and the reference's datasets run the specialised kernel linked into libseriation.so:
    with no compiler (SR_HIPCC=/nonexistent) and an empty cache the session still reports specialized, its
    code object is the embedded one, nothing is written to the cache, no fallback note, and the records equal
    the oracle's."""
    path = os.path.join(HERE, "golden", "datasets", name)
    out, err = _child(EMBEDDED_RUN, {"SR_JIT_CACHE": str(tmp_path / "cache"), "SR_HIPCC": "/nonexistent/bin/hipcc"},
                      path)
    assert out["specialized"] is True and out["embedded"] == 1, err
    assert not (tmp_path / "cache").exists()
    assert "unavailable" not in err and "compiling" not in err, err
    with open(path, "rb") as fh:
        text = fh.read()
    for k, s in enumerate([4, 9]):
        o = oracle_ref.run_chain(text, s, 1, 3, maxs=0)
        np.testing.assert_array_equal(np.array(out["rec"][k]), o["rec_int"])
        np.testing.assert_array_equal(np.array(out["dbl"][k], dtype=np.uint64), o["rec_dbl"].view(np.uint64))
