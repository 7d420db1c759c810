"""The C-ABI library loads and exports exactly what include/seriation.h declares (CPU only).

No compute calls: without a GPU the only device-facing calls made are the ones that must
fail loudly (session creation reports SR_EDEVICE -- there is no CPU fallback).
"""
import ctypes
import os
import re
import subprocess

import pytest

import seriation_amd as sa
from seriation_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "seriation.h")


def header_functions():
    with open(HEADER) as fh:
        text = fh.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sr_[a-z0-9_]+)\s*\(", text)) - {"sr_sample_sink_fn"})


def exported(path):
    out = subprocess.check_output(["nm", "-D", "--defined-only", path], text=True)
    return {ln.split()[-1] for ln in out.splitlines() if " T " in ln}


def test_header_matches_public_symbols():
    assert header_functions() == sorted(L.PUBLIC_SYMBOLS)


def test_library_exports_every_declared_symbol():
    syms = exported(L.LIB_PATH)
    missing = [s for s in header_functions() if s not in syms]
    assert not missing, missing
    sa.lib()  # loads and binds every prototype


def test_cli_binary_built():
    cli = os.path.join(os.path.dirname(L.LIB_PATH), "mcmc")
    assert os.access(cli, os.X_OK)


def test_version_and_errors():
    lib = sa.lib()
    assert lib.sr_version().decode().startswith("seriation")
    msgs = {c: lib.sr_strerror(c).decode() for c in range(-8, 1)}
    assert len(set(msgs.values())) == len(msgs)
    assert all(msgs.values())
    assert lib.sr_strerror(-999)


def test_default_opts_match_reference_cli():
    o = L.sr_run_opts()
    sa.lib().sr_default_opts(ctypes.byref(o))
    # mcmc.c:105-106 (tb = ts = 1000), mcmc.c:225 (10 sweeps per mcmc_sample), manycd 0
    assert (o.burnin_calls, o.sample_calls, o.sweeps_per_call, o.manycd) == (1000, 1000, 10, 0)


def test_invalid_arguments_rejected():
    lib = sa.lib()
    assert lib.sr_parse_dataset(None, 0, 2000, None) == L.SR_EINVAL
    h = ctypes.c_void_p()
    assert lib.sr_session_create(None, None, 0, None, ctypes.byref(h)) == L.SR_EINVAL
    assert lib.sr_session_run(None, 1, 0) == L.SR_EINVAL
    assert lib.sr_session_records(None) == 0


def _gpu_present():
    return os.path.exists("/dev/kfd") and sa.lib().sr_device_count() > 0


def test_no_cpu_fallback_without_device():
    if _gpu_present():
        pytest.skip("GPU present; the GPU suite covers sessions")
    ds = sa.Dataset.parse(b"3 2\n1 0\n1 1\n0 1\n")
    with pytest.raises(sa.SrError) as e:
        sa.Session(ds, [1])
    assert e.value.code == L.SR_EDEVICE


def test_restore_rejects_bad_checkpoints(tmp_path):
    """sr_session_restore validates the file before touching a device: missing file, bad magic,
    another dataset's checkpoint."""
    import struct
    ds = sa.Dataset.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "datasets", "g10s10.txt"))
    h = ctypes.c_void_p()
    opts = L.sr_run_opts()
    L.lib().sr_default_opts(ctypes.byref(opts))

    def restore(p):
        return L.lib().sr_session_restore(ctypes.byref(ds.c), os.fsencode(str(p)), ctypes.byref(opts), ctypes.byref(h))

    assert restore(tmp_path / "missing.srck") == -7                       # SR_EIO
    bad = tmp_path / "bad.srck"
    bad.write_bytes(b"XXXX" + bytes(40))
    assert restore(bad) == -2                                              # SR_EPARSE
    other = tmp_path / "other.srck"
    other.write_bytes(b"SRCK" + struct.pack("<I4iQ", 3, ds.N + 1, ds.M, 0, 2, 0))
    assert restore(other) == -1                                            # SR_EINVAL: other dataset
    samedims = tmp_path / "hash.srck"
    samedims.write_bytes(b"SRCK" + struct.pack("<I4iQ", 3, ds.N, ds.M, ds.nh, 2, 12345))
    assert restore(samedims) == -1                                         # SR_EINVAL: dataset hash differs


def test_restore_validates_chain_state(tmp_path):
    """A checkpoint whose chain state is damaged (the file length still right) is refused with
    SR_EPARSE before any upload: limits, permutation, counts, P == X, hard positions and the RNG
    cursor are checked.  The undamaged file passes validation (SR_EDEVICE without a GPU)."""
    import numpy as np
    ds = sa.Dataset.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "datasets", "g10s10.txt"))
    C = 2
    specs = (L.sr_chain_spec * C)()
    for k in range(C):
        specs[k].seed = k + 1
        specs[k].chain_id = k
    good = tmp_path / "good.srck"
    assert L.lib().sr_host_initial_checkpoint(ctypes.byref(ds.c), specs, C, os.fsencode(str(good))) == 0
    opts = L.sr_run_opts()
    L.lib().sr_default_opts(ctypes.byref(opts))

    def restore(p):
        h = ctypes.c_void_p()
        rc = L.lib().sr_session_restore(ctypes.byref(ds.c), os.fsencode(str(p)), ctypes.byref(opts), ctypes.byref(h))
        if rc == 0:
            L.lib().sr_session_destroy(h)
        return rc

    assert restore(good) in (0, L.SR_EDEVICE)
    raw7 = good.read_bytes()
    # version 7: the record count and the session's record capacity, then (after the state) the records
    assert raw7[:4] == b"SRCK" and np.frombuffer(raw7, "<u4", 1, 4)[0] == 7
    assert np.frombuffer(raw7, "<i4", 2, 32).tolist() == [0, 0]                # (none in an initial checkpoint)
    # a version-5 file (round 5: record count, no capacity) and a version-3 file (before round 5: no record count,
    # no records) still restore
    v5 = tmp_path / "v5.srck"
    v5.write_bytes(raw7[:4] + np.array([5], "<u4").tobytes() + raw7[8:36] + raw7[40:])
    assert restore(v5) in (0, L.SR_EDEVICE)
    v3 = tmp_path / "v3.srck"
    v3.write_bytes(raw7[:4] + np.array([3], "<u4").tobytes() + raw7[8:32] + raw7[40:])
    assert restore(v3) in (0, L.SR_EDEVICE)
    badcap = bytearray(raw7)   # a capacity below the record count is refused
    badcap[32:40] = np.array([5, 4], "<i4").tobytes()
    (tmp_path / "badcap.srck").write_bytes(bytes(badcap))
    assert restore(tmp_path / "badcap.srck") == -2
    trunc = tmp_path / "trunc.srck"
    trunc.write_bytes(raw7[:-8])
    assert restore(trunc) == -2
    N, M, nh, NW = ds.N, ds.M, ds.nh, (ds.N + 31) // 32
    off = 40 + C * ctypes.sizeof(L.sr_chain_spec)
    sizes = [("P", C * NW * M * 4), ("rpi", C * N * 4), ("hp", C * 64 * 4), ("ab", C * 2 * M * 4),
             ("cnt", C * 4 * M * 4), ("cdl", C * 4 * 8), ("mt", C * 8 * 624 * 4), ("rng", C * 2 * 8), ("acc", C * 10 * 8)]
    base = {}
    for name, n in sizes:
        base[name] = off
        off += n
    raw = good.read_bytes()
    assert len(raw) == off

    def damaged(name, word, value, dtype="<i4"):
        b = bytearray(raw)
        itemsize = np.dtype(dtype).itemsize
        b[base[name] + word * itemsize: base[name] + (word + 1) * itemsize] = np.array([value], dtype=dtype).tobytes()
        p = tmp_path / ("bad_%s_%d.srck" % (name, word))
        p.write_bytes(bytes(b))
        return p

    P0 = int(np.frombuffer(raw, "<u4", 1, base["P"])[0])
    assert restore(damaged("P", 0, P0 ^ 1, "<u4")) == -2                   # a column bit differs from X
    assert restore(damaged("rpi", 1, 0)) == -2                             # not a permutation
    assert restore(damaged("ab", 0, N + 5)) == -2                          # a limit outside [0, N]
    assert restore(damaged("cnt", 0, 10 ** 6)) == -2                       # counts disagree with X
    cdl = np.frombuffer(raw, "<f8", 4, base["cdl"]).copy()
    assert restore(damaged("cdl", 2, cdl[2] + 1.0, "<f8")) == -2           # loglik disagrees
    assert restore(damaged("rng", 1, 0, "<u8")) == -2                      # no generated block
    pos = int(np.frombuffer(raw, "<u8", 1, base["rng"])[0])
    assert restore(damaged("rng", 0, pos + 624 * 20, "<u8")) == -2         # cursor beyond the ring
    if nh:
        assert restore(damaged("hp", 0, N + 3)) == -2                      # hard position out of range


def test_hard_site_limit_boundary():
    """Up to SR_NHMAX = 64 hard sites take the mask paths (a 64-bit mask per taxon, one hard site per lane),
    more take the bitmap paths: 65 are accepted (40, 64, 65, 200 and N - 1 = 129 run bit-exact in
    tests/test_gpu_edge.py).  Sites are limited to N <= 4095 (12-bit positions in the packed proposal
    records): 4096 are refused with SR_EUNSUPPORTED before any device call.  Taxa are not limited by the
    records (they hold positions): M = 40000 is accepted."""
    def text(nh, N=90, M=6):
        rows = ["%d %d" % (N, M)]
        for i in range(N):
            rows.append(" ".join("1" if (i + m) % 3 == 0 else "0" for m in range(M)) + (" *" if i < nh else ""))
        return ("\n".join(rows) + "\n").encode()
    ds65 = sa.Dataset.parse(text(65))
    assert ds65.nh == 65
    big = sa.Dataset.parse(text(3, N=4096, M=2), maxs=0)
    with pytest.raises(sa.SrError) as e:
        sa.Session(big, [1])
    assert e.value.code == L.SR_EUNSUPPORTED
    if not _gpu_present():   # (taxa beyond int16: M = 40000 runs, tests/test_gpu_edge.py::test_taxa_beyond_int16)
        for ok in (sa.Dataset.parse(text(64)), ds65, sa.Dataset.parse(text(3, N=4095, M=2), maxs=0),
                   sa.Dataset.parse(text(3, N=8, M=40000), maxs=0)):
            with pytest.raises(sa.SrError) as e:
                sa.Session(ok, [1])
            assert e.value.code == L.SR_EDEVICE   # accepted by the limit check, then no device


def test_multi_device_arguments_rejected():
    lib = sa.lib()
    ds = sa.Dataset.parse(b"3 2\n1 0\n1 1\n0 1\n")
    out = (L.sr_chain_summary * 2)()
    devs = (ctypes.c_int32 * 3)(0, 0, 0)
    none = ctypes.cast(None, L.SINK_FN)
    # more shards than chains, no device list, no shards
    assert lib.sr_run_chains_multi(ctypes.byref(ds.c), sa.core.make_specs([1, 2]), 2, None, devs, 3, none, None, out) == L.SR_EINVAL
    assert lib.sr_run_chains_multi(ctypes.byref(ds.c), sa.core.make_specs([1, 2]), 2, None, None, 1, none, None, out) == L.SR_EINVAL
    assert lib.sr_run_to_dirs_multi(ctypes.byref(ds.c), sa.core.make_specs([1, 2]), 2, None, devs, 0, b"/tmp", out) == L.SR_EINVAL


def test_checkpoint_many_hard_sites(tmp_path):
    """More than 64 hard sites: the state keeps nh hard positions per chain rounded up to whole waves (128 for
    nh = 100); such a checkpoint validates (SR_EDEVICE without a GPU), a damaged hard position beyond the
    first 64 is refused."""
    import numpy as np
    N, M, nh, C = 150, 8, 100, 2
    rows = ["%d %d" % (N, M)] + [" ".join("1" if (i * 7 + m) % 5 == 0 else "0" for m in range(M)) + (" *" if i % 3 else "")
                                 for i in range(N)]
    ds = sa.Dataset.parse(("\n".join(rows) + "\n").encode())
    assert ds.nh == nh
    specs = sa.core.make_specs([3, 4])
    good = tmp_path / "nh100.srck"
    assert L.lib().sr_host_initial_checkpoint(ctypes.byref(ds.c), specs, C, os.fsencode(str(good))) == 0
    opts = L.sr_run_opts()
    L.lib().sr_default_opts(ctypes.byref(opts))
    h = ctypes.c_void_p()
    rc = L.lib().sr_session_restore(ctypes.byref(ds.c), os.fsencode(str(good)), ctypes.byref(opts), ctypes.byref(h))
    if rc == 0:
        L.lib().sr_session_destroy(h)
    assert rc in (0, L.SR_EDEVICE)
    NW = (N + 31) // 32
    off = 40 + C * ctypes.sizeof(L.sr_chain_spec) + C * NW * M * 4 + C * N * 4
    raw = bytearray(good.read_bytes())
    assert len(raw) == off + C * 128 * 4 + C * 2 * M * 4 + C * 4 * M * 4 + C * 4 * 8 + C * 8 * 624 * 4 + C * 2 * 8 + C * 10 * 8
    hp = np.frombuffer(bytes(raw), "<i4", C * 128, off).reshape(C, 128)
    assert (np.diff(hp[0, :nh]) > 0).all() and (hp[:, nh:] == 0).all()
    raw[off + 4 * 80: off + 4 * 81] = np.array([N + 9], "<i4").tobytes()
    bad = tmp_path / "bad.srck"
    bad.write_bytes(bytes(raw))
    assert L.lib().sr_session_restore(ctypes.byref(ds.c), os.fsencode(str(bad)), ctypes.byref(opts), ctypes.byref(h)) == -2
