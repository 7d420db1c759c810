"""The multi-GPU path's collectives on real hardware (RCCL = torch.distributed "nccl" on ROCm).

The box has one GPU, so the RCCL world is 1: the all-gathers still run through RCCL on cuda
tensors, and bench.py under torch.distributed.run (--nproc-per-node 1) must give
the single-process result bit for bit: the same selected chains, the same E[c] / E[d] / CORRMN and
the same gathered records (script.py:55-99).  Each run is a fresh child process."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--gpus", "1", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--chains-per-gpu", "24",
        "--calls-per-step", "20"]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    e = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        e.pop(k, None)
    return e


def _bench_line(cmd):
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{") and '"metric"' in l]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_rccl_collectives_world1():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_child.py")], capture_output=True, text=True,
                       timeout=240, env=_env())
    assert r.returncode == 0 and "rccl ok" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def test_bench_under_launcher_equals_single_process():
    single = _bench_line([sys.executable, "bench.py"] + ARGS)
    port = _port()
    launched = _bench_line([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                            "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py"] + ARGS)
    assert single["n_gpus"] == launched["n_gpus"] == 1
    a, b = single["selection"], launched["selection"]
    assert a["chains_selected"] == b["chains_selected"] and len(a["chains_selected"]) >= 1
    assert a["records_sha256"] == b["records_sha256"]
    for k in ("exp_c", "exp_d", "corr_mn"):
        assert a[k] == b[k], k
    assert a["samples_per_chain"] == b["samples_per_chain"] == 40


def test_bench_two_ranks_on_one_gpu_equals_single_process():
    """bench.py's N>1 path end to end on the one-GPU box: `--gpus 2` launches two ranks itself
    (torch.distributed.run children), both on device 0 (--device-of-rank 0,0) with gloo collectives (RCCL
    cannot host two ranks on one GPU); rank 1 owns chains 24..47, the summary all-gather, the one-sigma
    selection on every rank, the record gather from non-zero owners and the max-over-ranks timing all run.
    The selection, the gathered records and E[c] / E[d] / CORRMN must equal a single process running all
    48 chains (script.py:55-99), and both lines' parity legs must match the oracle."""
    common = ["--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--calls-per-step", "20"]
    single = _bench_line([sys.executable, "bench.py", "--gpus", "1", "--chains-per-gpu", "48"] + common)
    two = _bench_line([sys.executable, "bench.py", "--gpus", "2", "--chains-per-gpu", "24", "--device-of-rank", "0,0",
                       "--dist-backend", "gloo"] + common)
    assert two["n_gpus"] == 2 and two["config"]["chains"] == 48 and "gloo" in two["config"]["parallelism"]
    a, b = single["selection"], two["selection"]
    assert a["chains_selected"] == b["chains_selected"] and len(a["chains_selected"]) >= 1
    assert a["records_sha256"] == b["records_sha256"]
    for k in ("exp_c", "exp_d", "corr_mn"):
        assert a[k] == b[k], k
    assert single["parity"]["match"] and two["parity"]["match"]
    # the parity legs check every selected chain and two the selection rejected (rank 0's first and last)
    for line in (single, two):
        p = line["parity"]
        assert p["selected_checked"] == line["selection"]["chains_selected"]
        assert len(p["rejected_checked"]) == 2 and not set(p["rejected_checked"]) & set(p["selected_checked"])
        assert p["chains"] == p["selected_checked"] + p["rejected_checked"]
    assert two["parity"]["rejected_checked"][-1] < 24   # rank 0's shard


def test_bench_total_chains_ragged_three_ranks_equals_single_process():
    """The metric's own form (BASELINE.json: 100 chains at 1/2/4/8 GPUs; script.py:55-62 runs a fixed 100): with
    --total-chains 100 the chains are sharded contiguously and raggedly (dist.shard: 33/33/34 over three ranks,
    13/13/13/13/12/12/12/12 over eight).  Three gloo ranks on the one GPU must give the single-process 100-chain
    line bit for bit -- selection, gathered records, E[c], E[d], CORRMN -- and both lines say strong scaling."""
    common = ["--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--calls-per-step", "20", "--total-chains", "100"]
    single = _bench_line([sys.executable, "bench.py", "--gpus", "1"] + common)
    three = _bench_line([sys.executable, "bench.py", "--gpus", "3", "--device-of-rank", "0,0,0", "--dist-backend",
                         "gloo"] + common)
    assert single["config"]["chains"] == three["config"]["chains"] == 100
    assert single["config"]["chains_per_rank"] == [100] and three["config"]["chains_per_rank"] == [33, 33, 34]
    assert single["scaling"] == three["scaling"] == "strong" and three["n_gpus"] == 3
    a, b = single["selection"], three["selection"]
    assert a["chains_selected"] == b["chains_selected"] and len(a["chains_selected"]) >= 1
    assert a["records_sha256"] == b["records_sha256"]
    for k in ("exp_c", "exp_d", "corr_mn"):
        assert a[k] == b[k], k
    assert single["parity"]["match"] and three["parity"]["match"]
    assert three["parity"]["rejected_checked"][-1] < 33   # rank 0's shard
    assert "config2" not in single and "config5" not in single   # --no-cpu-baseline: no extra legs
