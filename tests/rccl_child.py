"""Child process of tests/test_gpu_rccl.py: the two collectives of seriation_amd.dist (summary
all-gather, selected-records all-gather) on cuda tensors over the "nccl" (RCCL) backend at world 1,
checked against their inputs.  Prints "rccl ok" on success.  Env: MASTER_ADDR/PORT set by the test."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "seriation-in-paleontological-data-using-mcmc_amd"))
from seriation_amd import dist as sd  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    rng = np.random.default_rng(5)
    n, T, W = 12, 7, 2 * 9 + 5
    rows = np.column_stack([np.arange(n), rng.uniform(100, 200, n), rng.uniform(0.001, 0.1, n),
                            rng.uniform(0.2, 0.8, n)])
    got = sd.gather_summaries(rows, n, device="cuda")
    assert np.array_equal(got.view(np.uint64), rows.view(np.uint64)), "summary all-gather changed bits"
    sel = sd.select_chains(got, 4)
    ab = rng.integers(-30000, 30000, (n, T, W)).astype(np.int16)
    cdl = rng.standard_normal((n, T, 3))
    gab, gcd = sd.gather_selected_records(sel, n, list(range(n)), ab, cdl, device="cuda")
    assert np.array_equal(gab, ab[sel]) and np.array_equal(gcd.view(np.uint64), cdl[sel].view(np.uint64))
    t = torch.tensor([1.5], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert float(t.item()) == 1.5
    dist.barrier()
    dist.destroy_process_group()
    print("rccl ok", sel)


if __name__ == "__main__":
    main()
