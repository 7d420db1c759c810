"""The shape-specialised kernel build (srk_jit_load, csrc/sr_device.hip) compiles on the CPU: the same
hipcc --genco command the library spawns at session creation, for the bench shape, yields a code object
holding exactly the kernel the loader looks up.  (On the GPU, tests/test_gpu_jit.py runs it.)"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd")
HIPCC = os.environ.get("SR_HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.access(HIPCC, os.X_OK), reason="no hipcc")
@pytest.mark.parametrize("tb,nwm,n,m,nh", [(512, 9, 256, 512, 12), (1024, 0, 600, 700, 7)], ids=["bench-shape", "lds-walk"])
def test_specialised_kernel_compiles(tmp_path, tb, nwm, n, m, nh):
    out = tmp_path / "k.co"
    cmd = [HIPCC, "--genco", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
           "-DSR_JIT", "-DSR_JIT_TB=%d" % tb, "-DSR_JIT_NWM=%d" % nwm, "-DSR_FN=%d" % n, "-DSR_FM=%d" % m,
           "-DSR_FH=%d" % nh, "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc"),
           "-o", str(out), os.path.join(PKG, "csrc", "sr_device.hip")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    blob = out.read_bytes()
    name = b"_Z15sr_sweep_kernelILi%dELi%dELb0ELb0ELb0EEv5KArgs" % (tb, nwm)
    assert name in blob
    # one kernel only: the JIT build excludes the session layer and every other instantiation
    assert blob.count(b"_Z15sr_sweep_kernelILi") == blob.count(name)
