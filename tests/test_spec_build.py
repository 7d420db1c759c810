"""Shape-specialised sweep kernels at the boundary (csrc/sr_spec.c, sr_specialize; CPU only, no GPU):
the code object is compiled from the source snapshot taken with the library (build/spec/), cached under a
key that covers the snapshot, the definitions, the flags, the target and the compiler's ROCm version, and
never compiled from a snapshot that differs from the one the library was built from or while a profiler
tool library is preloaded.  Each scenario runs in a fresh interpreter (the library resolves its snapshot
and compiler version once per process).  On the GPU, tests/test_gpu_jit.py loads and runs these objects."""
import json
import os
import shutil
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd")
LIBDIR = os.path.join(PKG, "build")
SYNTH = os.path.join(ROOT, "tests", "golden", "datasets", "synth_256x512.txt")


def _subject():
    """a 250 x 500 dataset (12 hard sites): the bench kernel's block and walk (TB 512, 9 words) but a shape the
    library does not embed, so its kernel goes through the cache / compiler machinery tested here"""
    import tempfile
    from test_gpu_edge import make_text
    path = os.path.join(tempfile.gettempdir(), "sr_spec_subject_250x500.txt")
    if not os.path.exists(path):
        with open(path, "wb") as fh:
            fh.write(make_text(250, 500, 12, seed=250500))
    return path


SUBJECT = _subject()
HIPCC = "/opt/rocm/bin/hipcc"
BENCH_KERNEL = b"_Z15sr_sweep_kernelILi512ELi9ELb0ELb0ELb0ELb0ELb0EEv5KArgs"

needs_hipcc = pytest.mark.skipif(not os.access(HIPCC, os.X_OK), reason="no hipcc")

# runs in a child: prints one JSON line {"rc": sr_specialize's result, "path": the cache path (or reason)}
CHILD = textwrap.dedent("""
    import ctypes, json, sys
    sys.path.insert(0, %r)
    import seriation_amd as sa
    from seriation_amd import _lib as L
    ds = sa.Dataset.load(sys.argv[1], maxs=0)
    buf = ctypes.create_string_buffer(4096)
    prc = sa.lib().sr_spec_cache_path(ds.N, ds.M, ds.nh, int(sys.argv[2]), buf, 4096)
    o = sa.core.make_opts(block_threads=int(sys.argv[2]))
    rc = sa.lib().sr_specialize(ctypes.byref(ds.c), ctypes.byref(o))
    print(json.dumps({"rc": rc, "path_rc": prc, "path": buf.value.decode()}))
""" % PKG)


def child(env_extra, dataset=SUBJECT, block_threads=0, lib=None):
    env = dict(os.environ)
    env.pop("SR_JIT_CACHE", None)
    env.update(env_extra)
    if lib:
        env["SERIATION_LIB"] = lib
    r = subprocess.run([sys.executable, "-c", CHILD, dataset, str(block_threads)], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1]), r.stderr


def test_snapshot_matches_sources_and_library_hash():
    """build/spec/ holds exactly the kernel sources, and the hash tool's value is the one compiled in."""
    for name, src in [("sr_device.hip", "csrc"), ("sr_math.h", "csrc"), ("sr_rng.h", "csrc"), ("sr_tables.h", "csrc"),
                      ("sr_internal.h", "csrc"), ("seriation.h", os.path.join("..", "include"))]:
        with open(os.path.join(PKG, src, name), "rb") as a, open(os.path.join(LIBDIR, "spec", name), "rb") as b:
            assert a.read() == b.read(), "%s: snapshot differs from the sources (run make)" % name
    h = subprocess.check_output([os.path.join(LIBDIR, "srhash"), os.path.join(LIBDIR, "spec")], text=True).strip()
    with open(os.path.join(LIBDIR, "spec.hash")) as fh:
        assert fh.read().strip() == h


@needs_hipcc
def test_specialize_compiles_once_into_the_cache(tmp_path):
    out, err = child({"SR_JIT_CACHE": str(tmp_path)})
    assert out["rc"] == 1 and out["path_rc"] == 0, (out, err)
    assert os.path.dirname(out["path"]) == str(tmp_path)
    blob = open(out["path"], "rb").read()
    assert BENCH_KERNEL in blob and b"sr_spec_abi" in blob
    # one kernel only: the specialised build excludes the session layer and every other instantiation
    assert blob.count(b"_Z15sr_sweep_kernelILi") == blob.count(BENCH_KERNEL)
    mtime = os.stat(out["path"]).st_mtime_ns
    out2, _ = child({"SR_JIT_CACHE": str(tmp_path)})
    assert out2 == out and os.stat(out["path"]).st_mtime_ns == mtime   # a cache hit, not a recompile
    assert not [f for f in os.listdir(tmp_path) if f.endswith(".tmp")]


def test_key_covers_shape_block_and_compiler_version(tmp_path, datasets_dir):
    base, _ = child({"SR_JIT_CACHE": str(tmp_path), "SR_HIPCC": "/nonexistent/bin/hipcc"})
    g10, _ = child({"SR_JIT_CACHE": str(tmp_path), "SR_HIPCC": "/nonexistent/bin/hipcc"},
                   dataset=os.path.join(datasets_dir, "g10s10.txt"))
    tb256, _ = child({"SR_JIT_CACHE": str(tmp_path), "SR_HIPCC": "/nonexistent/bin/hipcc"}, block_threads=256)
    # a compiler of another ROCm release: <hipcc>/../.info/version
    fake = tmp_path / "rocm"
    (fake / "bin").mkdir(parents=True)
    (fake / ".info").mkdir()
    (fake / ".info" / "version").write_text("9.9.9-test\n")
    cc = fake / "bin" / "hipcc"
    cc.write_text("#!/bin/sh\nexit 3\n")
    cc.chmod(0o755)
    other, err = child({"SR_JIT_CACHE": str(tmp_path), "SR_HIPCC": str(cc)})
    assert all(o["path_rc"] == 0 for o in (base, g10, tb256, other))
    paths = {base["path"], g10["path"], tb256["path"], other["path"]}
    assert len(paths) == 4, paths
    # no compiler: nothing cached -> SR_EIO and one line on stderr; a failing compiler likewise (g10s10's kernel
    # is embedded in the library: ready without either)
    assert base["rc"] == -7 and other["rc"] == -7 and g10["rc"] == 1
    assert "compile failed" in err and ".log" in err
    assert not os.path.exists(other["path"])


@needs_hipcc
def test_entry_under_another_key_is_not_used(tmp_path, datasets_dir):
    """A code object cached under another shape's key is never picked up: the subject shape compiles its own."""
    other, _ = child({"SR_JIT_CACHE": str(tmp_path)}, block_threads=256)
    assert other["rc"] == 1
    junk = open(other["path"], "rb").read()
    out, _ = child({"SR_JIT_CACHE": str(tmp_path)})
    assert out["rc"] == 1 and out["path"] != other["path"]
    blob = open(out["path"], "rb").read()
    assert blob != junk and BENCH_KERNEL in blob


def test_profiler_preload_never_compiles(tmp_path):
    # (rocprofv3 exports ROCPROF_* settings for its tool library; the variable alone loads nothing)
    out, err = child({"SR_JIT_CACHE": str(tmp_path), "ROCPROF_OUTPUT_PATH": str(tmp_path / "prof")})
    assert out["rc"] == -7 and "profiler" in err
    assert os.listdir(tmp_path) == [] or not [f for f in os.listdir(tmp_path) if f.endswith(".co")]


def test_stale_snapshot_is_refused(tmp_path):
    """A library whose snapshot was edited after the build (sources changed without a rebuild) compiles
    nothing: the kernel it would compile would not match its KArgs / LDS layout."""
    lib = tmp_path / "libseriation.so"
    shutil.copy(os.path.join(LIBDIR, "libseriation.so"), lib)
    shutil.copytree(os.path.join(LIBDIR, "spec"), tmp_path / "spec")
    with open(tmp_path / "spec" / "sr_internal.h", "a") as fh:
        fh.write("\n/* edited after the build */\n")
    out, err = child({"SR_JIT_CACHE": str(tmp_path / "cache")}, lib=str(lib))
    assert out["path_rc"] == -2 and out["rc"] == -7
    assert "differs from the sources the library was built from" in err
    assert not (tmp_path / "cache").exists()


def test_hbm_sessions_have_no_specialised_kernel(tmp_path):
    import seriation_amd as sa
    from test_gpu_edge import make_text
    ds = sa.Dataset.parse(make_text(64, 1100, 6, seed=64 * 1000 + 1100), maxs=0)
    assert sa.specialize(ds, columns="hbm") is False


def test_unwritable_cache_is_reported(tmp_path):
    """A cache directory that cannot be created (under a regular file): SR_EIO and a line naming the cache."""
    blocker = tmp_path / "file"
    blocker.write_text("x")
    out, err = child({"SR_JIT_CACHE": str(blocker / "cache")})
    assert out["rc"] == -7 and "cache directory" in err


EMBEDDED = [("g10s10.txt", 124, 139, 11), ("g10s2.txt", 501, 139, 14), ("g2s2.txt", 526, 296, 15),
            ("g5s5.txt", 273, 202, 14), ("synth_256x512.txt", 256, 512, 12)]


@pytest.mark.parametrize("name,N,M,nh", EMBEDDED, ids=[e[0] for e in EMBEDDED])
def test_reference_shapes_are_embedded_without_compiler_or_cache(tmp_path, datasets_dir, name, N, M, nh):
    """The reference's datasets and the bench matrix run code objects linked into libseriation.so at build time
    (csrc/sr_embed_shapes.txt): with no compiler (SR_HIPCC=/nonexistent) and an empty cache, sr_specialize
    reports the kernel ready (1) and writes nothing; the GPU side (tests/test_gpu_jit.py) loads them."""
    import seriation_amd as sa
    assert sa.lib().sr_spec_is_embedded(N, M, nh, 0) == 1
    out, err = child({"SR_JIT_CACHE": str(tmp_path / "cache"), "SR_HIPCC": "/nonexistent/bin/hipcc"},
                     dataset=os.path.join(datasets_dir, name))
    assert out["rc"] == 1, (out, err)
    assert not (tmp_path / "cache").exists()
    assert "unavailable" not in err


def test_embedded_objects_are_in_the_library():
    """one code object per embedded shape inside the library file, each with the bench kernel family's symbol
    and its ABI record; shapes outside the list (other block sizes, the test-only subject) are not embedded"""
    import seriation_amd as sa
    blob = open(os.path.join(LIBDIR, "libseriation.so"), "rb").read()
    assert blob.count(b"sr_spec_abi") >= len(EMBEDDED)
    assert BENCH_KERNEL in blob
    assert sa.lib().sr_spec_is_embedded(250, 500, 12, 0) == 0
    assert sa.lib().sr_spec_is_embedded(256, 512, 12, 1024) == 0


SESSION_CHILD = textwrap.dedent("""
    import sys
    sys.path.insert(0, %r)
    import seriation_amd as sa
    ds = sa.Dataset.load(sys.argv[1], maxs=0)
    try:
        sa.Session(ds, [1])
        print("created")
    except sa.SrError as e:
        print("refused %%d" %% e.code)
""" % PKG)


def test_cache_only_mode_never_spawns_the_compiler(tmp_path):
    """SR_JIT=cache: a session whose shape is neither embedded nor cached gets the generic kernel and one line saying
    why -- no compiler is spawned, nothing is written to the cache (the session's own shape resolution runs before
    any HIP call, so this holds without a GPU too); sr_specialize still fills the cache ahead of time."""
    env = dict(os.environ, SR_JIT="cache", SR_JIT_CACHE=str(tmp_path))
    r = subprocess.run([sys.executable, "-c", SESSION_CHILD, SUBJECT], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "SR_JIT=cache forbids compiling at run time" in r.stderr
    assert "compiling the sweep kernel" not in r.stderr
    assert not [f for f in os.listdir(tmp_path) if f.endswith(".co")]
