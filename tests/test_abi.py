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
    other.write_bytes(b"SRCK" + struct.pack("<I4iQ", 1, ds.N + 1, ds.M, 0, 2, 0))
    assert restore(other) == -1                                            # SR_EINVAL: other dataset
    samedims = tmp_path / "hash.srck"
    samedims.write_bytes(b"SRCK" + struct.pack("<I4iQ", 1, ds.N, ds.M, ds.nh, 2, 12345))
    assert restore(samedims) == -1                                         # SR_EINVAL: dataset hash differs
