"""CPU sanitizer builds (SURVEY §5 race/sanitizer tooling): the C host layer (csrc/sr_host.c, device
layer stubbed: tests/asan/) and the oracle CLI under AddressSanitizer + UndefinedBehaviorSanitizer.
Any sanitizer report aborts the program (-fno-sanitize-recover), so exit 0 means a clean run."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd")
DATA = os.path.join(ROOT, "tests", "golden", "datasets")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")


def _make(d, target):
    r = subprocess.run(["make", "-s", "-C", d, target], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail("sanitizer build failed:\n" + r.stdout + r.stderr)
    return os.path.join(d, target)


@pytest.mark.parametrize("name", ["g10s10", "g5s5", "g2s2"])
def test_host_layer_under_asan_ubsan(tmp_path, name):
    exe = _make(PKG, "build/asan/host_asan")
    r = subprocess.run([exe, os.path.join(DATA, name + ".txt"), str(tmp_path)], capture_output=True, text=True,
                       env=ENV, timeout=300)
    assert r.returncode == 0 and "host_asan: ok" in r.stdout, r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr


def test_oracle_cli_under_asan_ubsan(tmp_path):
    exe = _make(os.path.join(ROOT, "oracle"), "build/asan/mcmc_oracle")
    os.makedirs(tmp_path / "Chains" / "chain_00")
    with open(os.path.join(DATA, "g5s5.txt"), "rb") as fh:
        r = subprocess.run([exe, "0", "10", "20"], stdin=fh, cwd=str(tmp_path), capture_output=True,
                           env=dict(ENV, GSL_RNG_SEED="3"), timeout=300)
    err = r.stderr.decode()
    assert r.returncode == 0, err
    assert "runtime error" not in err and "AddressSanitizer" not in err, err
    lines = (tmp_path / "Chains" / "chain_00" / "chain_data.csv").read_text().splitlines()
    assert len(lines) == 20
