"""N>1 path on the CPU: world_size-2 gloo processes shard chains, all-gather the summary
records (the one collective) and select identical chains on every rank.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from seriation_amd import dist as sd


def test_shard_covers_all_chains_contiguously():
    for n in (0, 1, 7, 100, 800, 101):
        for world in (1, 2, 3, 4, 8):
            got = [list(sd.shard(n, world, r)) for r in range(world)]
            flat = [i for g in got for i in g]
            assert flat == list(range(n))
            assert max(map(len, got)) - min(map(len, got)) <= 1
    assert list(sd.shard(800, 8, 3)) == list(range(300, 400))
    with pytest.raises(ValueError):
        sd.shard(10, 2, 2)


def test_summaries_from_records_matches_exp_data_rule():
    rng = np.random.default_rng(0)
    cdl = np.stack([np.log(rng.uniform(0.001, 0.1, (2, 5))), np.log(rng.uniform(0.2, 0.8, (2, 5))),
                    -rng.uniform(100, 200, (2, 5))], axis=-1)
    rows = sd.summaries_from_records([4, 9], cdl)
    assert rows[:, 0].tolist() == [4, 9]
    np.testing.assert_allclose(rows[1, 1], -cdl[1, :, 2].sum() / 1000)
    np.testing.assert_allclose(rows[0, 2], np.exp(cdl[0, :, 0]).sum() / 1000)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_total, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids = list(sd.shard(n_total, world, rank))
        # deterministic fake per-chain summaries (value depends only on chain id)
        rows = np.array([[i, 1000.0 + ((i * 37) % 23) * 0.5, 0.01, 0.5] for i in ids]).reshape(-1, 4)
        allrows = sd.gather_summaries(rows, n_total)
        out[rank] = (allrows.tobytes(), sd.select_chains(allrows, 8))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [100, 7])
def test_gloo_world2_gather_and_select(n_total):
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    (b0, s0), (b1, s1) = out[0], out[1]
    assert b0 == b1 and s0 == s1
    allrows = np.frombuffer(b0).reshape(-1, 4)
    assert allrows[:, 0].tolist() == list(range(n_total))
    expect = np.array([1000.0 + ((i * 37) % 23) * 0.5 for i in range(n_total)])
    np.testing.assert_array_equal(allrows[:, 1], expect)
    ref = sd.choose_from_values({"chain_%02d" % i: v for i, v in enumerate(expect)}, 8)
    assert s0 == ref


def test_summaries_match_exp_data_bits():
    """summaries_from_records (the all-gather payload) equals compute_exp_data / print_exp_data
    (mcmc.c:53-67) bit for bit: the oracle's exp_data over the same saved samples."""
    import oracle_ref
    from seriation_amd import dist as sd
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "datasets", "g10s10.txt"), "rb") as fh:
        text = fh.read()
    for seed in (1, 2, 3):
        o = oracle_ref.run_chain(text, seed, 5, 40)
        row = sd.summaries_from_records([7], o["rec_dbl"][None])[0]
        assert row[0] == 7
        assert [float(v).hex() for v in row[1:]] == [float(v).hex() for v in o["exp"]], seed
