"""A fixed-seed subset of the random-shape parity fuzz (tools/fuzz_shapes.py) in the GPU suite.

Twenty shapes chosen to cover the planner's every kernel family: register walks of 9 and 17 words and their
boundaries (N = 287 / 288, 543 / 544), LDS-column walks beyond, HBM columns on one workgroup, split chains (two
workgroups per chain, 1025-2048 taxa, LDS and HBM Gibbs checkpoints), taxa beyond the block (several per thread),
manycd (per-taxon c, d), 256 / 512 / 1024-thread blocks, and hard-site counts around the mask / bitmap switches
(31, 32, 33, 64, 65, 70).  Each runs 2 chains x (2 burn-in + 3 saved calls) against the CPU oracle bit for bit
(a, b, pi, c, d, loglik; manycd: every taxon's c, d) -- mcmc.c:140-185."""
import numpy as np
import pytest

import oracle_ref
import seriation_amd as sa
from test_gpu_edge import make_text

pytestmark = pytest.mark.gpu

# name, N, M, hard sites, block_threads (0 = planner), columns, manycd
SHAPES = [
    ("reg9-small", 37, 300, 3, 0, "auto", 0),
    ("reg9-m700", 250, 700, 12, 0, "auto", 0),
    ("reg9-nh31", 287, 512, 31, 0, "auto", 0),
    ("reg17-n288-nh32", 288, 256, 32, 0, "auto", 0),
    ("reg17-nh33", 500, 900, 33, 0, "auto", 0),
    ("reg9-nh64", 200, 1024, 64, 0, "auto", 0),
    ("reg9-nh65", 190, 333, 65, 0, "auto", 0),
    ("reg17-n543", 543, 1024, 12, 0, "auto", 0),
    ("lds-n544", 544, 300, 12, 0, "auto", 0),
    ("lds-n600", 600, 400, 12, 0, "auto", 0),
    ("mid-341x890", 341, 890, 12, 0, "auto", 0),
    ("tb256", 60, 40, 0, 256, "auto", 0),
    ("tb512-two-per-thread", 288, 513, 12, 512, "auto", 0),
    ("hbm-single", 1000, 600, 12, 0, "hbm", 0),
    ("split-1024x1500-nh40", 1024, 1500, 40, 0, "auto", 0),
    ("split-n1300", 1300, 1100, 12, 0, "auto", 0),
    ("split-nh70", 800, 2048, 70, 0, "auto", 0),
    ("hbm-m2600", 1500, 2600, 12, 0, "auto", 0),
    ("manycd-lds", 150, 200, 5, 0, "auto", 1),
    ("manycd-hbm", 700, 1500, 12, 1024, "auto", 1),
]


def lds_shapes():
    """(N, M, nh, block_threads) of the LDS-column shapes here (__graft_entry__.prewarm compiles their specialised
    kernels ahead; tests/spec_shapes.py)."""
    return [(N, M, nh, tb) for _, N, M, nh, tb, cols, mcd in SHAPES if cols == "auto" and not mcd and N <= 600 and M <= 1024]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: s[0])
def test_fuzz_shape_equals_oracle(shape):
    name, N, M, nh, tb, cols, mcd = shape
    seed = 1000 + sum(map(ord, name))
    text = make_text(N, M, nh, seed=seed)
    ds = sa.Dataset.parse(text, maxs=0)
    seeds = [seed % 997 + 1, seed % 991 + 2]
    with sa.Session(ds, seeds, block_threads=tb, columns=cols, manycd=mcd) as s:
        desc = (s.variant, s.kernel, s.block_threads)
    print(name, desc)
    summ, recs = sa.run_chains(ds, seeds, burnin_calls=2, sample_calls=3, keep_records=True, block_threads=tb,
                               columns=cols, manycd=mcd)
    for k, sd in enumerate(seeds):
        o = oracle_ref.run_chain(text, sd, 2, 3, maxs=0, manycd=mcd)
        assert o["rc"] == 0
        assert np.array_equal(recs[0][k], o["rec_int"]), (name, sd, desc)
        assert np.array_equal(recs[1][k].view(np.uint64), o["rec_dbl"].view(np.uint64)), (name, sd, desc)
        if mcd:
            assert np.array_equal(recs[2][k].view(np.uint64), o["rec_cdv"].view(np.uint64)), (name, sd, desc)
        assert summ[k]["consistent"] == 0
