"""bench.py's host-side pieces on the CPU: the device count taken without HIP (the parent of `--gpus N` must not
initialise the GPU before it starts the ranks), and the like-for-like CPU baseline (burn-in window untimed, the
GPU's timed window timed inside the oracle, mcmc.c:140-185)."""
import os

import bench

HERE = os.path.dirname(os.path.abspath(__file__))


def _node(root, name, simds):
    d = root / name
    d.mkdir()
    (d / "properties").write_text("cpu_cores_count 0\nsimd_count %d\nmem_banks_count 1\n" % simds)


def test_visible_gpu_count_from_kfd_topology(tmp_path, monkeypatch):
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    _node(tmp_path, "0", 0)        # the CPU agent
    for k in range(1, 9):
        _node(tmp_path, str(k), 1024)
    assert bench.visible_gpu_count(str(tmp_path)) == 8
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "2,5")
    assert bench.visible_gpu_count(str(tmp_path)) == 2
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "3")
    assert bench.visible_gpu_count(str(tmp_path)) == 1
    assert bench.visible_gpu_count(str(tmp_path / "missing")) is None


def test_cpu_baseline_times_the_window_after_burnin():
    ds = os.path.join(HERE, "golden", "datasets", "g5s5.txt")
    r = bench.cpu_baseline(ds, 4, 6, 2)
    assert r["value"] > 0 and r["cores"] == 2 and r["kind"] == "port"
    assert "4 untimed" in r["sample"] and "6 timed" in r["sample"]
    assert r["from_birth"]["value"] > 0
    r0 = bench.cpu_baseline(ds, 0, 3, 1)
    assert "from_birth" not in r0
