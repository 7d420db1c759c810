"""N>1 path on the CPU: world_size-2 gloo processes shard chains (run by the CPU oracle),
all-gather the summary records, select identical chains on every rank and gather the selected
chains' records (the two collectives), matching a single-process run exactly.
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


DS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "datasets", "g10s10.txt")
TB, TS, K = 2, 6, 3   # burn-in calls, saved calls, chains selected


def _oracle_shard(ids):
    """The chains of one shard (seed = chain id + 1), run by the CPU oracle: records as the
    GPU session returns them (a|b|pi int16 rows, c/d/loglik)."""
    import oracle_ref
    with open(DS, "rb") as fh:
        text = fh.read()
    runs = [oracle_ref.run_chain(text, i + 1, TB, TS) for i in ids]
    ab = np.array([r["rec_int"] for r in runs], np.int16).reshape(len(ids), TS, -1)
    cdl = np.array([r["rec_dbl"] for r in runs]).reshape(len(ids), TS, 3)
    return ab, cdl


def _single_process(n_total):
    ids = list(range(n_total))
    ab, cdl = _oracle_shard(ids)
    rows = sd.summaries_from_records(ids, cdl)
    sel = sd.select_chains(rows, K)
    sab, scd = ab[sel], cdl[sel]
    return rows, sel, sab, scd, sd.selection_statistics(sab, scd, 124, 139, K)


def _worker(rank, world, port, n_total, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids = list(sd.shard(n_total, world, rank))
        ab, cdl = _oracle_shard(ids)
        rows = sd.summaries_from_records(ids, cdl)
        allrows = sd.gather_summaries(rows, n_total)           # collective 1
        sel = sd.select_chains(allrows, K)
        sab, scd = sd.gather_selected_records(sel, n_total, ids, ab, cdl)   # collective 2
        stats = sd.selection_statistics(sab, scd, 124, 139, K)
        # collective 2 in bench.py's form (gather_selected_records_device): the rank's selected records copied
        # by pointer into one slab buffer (sr_session_copy_chain_records there; a memmove from the shard's
        # records here, CPU tensors under gloo), one all-gather per array
        import ctypes

        def copy_chain(j, pa, pc):
            ctypes.memmove(pa, np.ascontiguousarray(ab[j]).ctypes.data, ab[j].nbytes)
            ctypes.memmove(pc, np.ascontiguousarray(cdl[j]).ctypes.data, cdl[j].nbytes)

        dab, dcd = sd.gather_selected_records_device(sel, n_total, ids, copy_chain, TS, ab.shape[2], device="cpu")
        dev_same = dab.numpy().tobytes() == sab.tobytes() and dcd.numpy().tobytes() == scd.tobytes()
        ws = sd.selected_records_workspace(K, TS, ab.shape[2], "cpu")   # bench.py's preallocated form
        wab, wcd = sd.gather_selected_records_device(sel, n_total, ids, copy_chain, TS, ab.shape[2], device="cpu", ws=ws)
        dev_same = dev_same and wab.numpy().tobytes() == sab.tobytes() and wcd.numpy().tobytes() == scd.tobytes()
        out[rank] = (allrows.tobytes(), sel, sab.tobytes(), scd.tobytes(), stats, dev_same)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [8, 5])
def test_gloo_world2_matches_single_process(n_total):
    """Two gloo ranks shard real (oracle-run) chains, all-gather the summaries, select, gather the
    selected chains' records and compute E[c] / E[d] / CORRMN: every rank gets exactly what one
    process running all chains gets."""
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    rows, sel, sab, scd, stats = _single_process(n_total)
    assert 0 < len(sel) <= K
    for r in range(2):
        b, s_, ab_b, cd_b, st, dev_same = out[r]
        assert dev_same
        assert b == rows.tobytes()
        assert s_ == sel
        assert ab_b == sab.tobytes() and cd_b == scd.tobytes()
        assert st == stats


def test_owner_matches_shard():
    for n, world in ((800, 8), (7, 3), (5, 2)):
        for c in range(n):
            assert c in sd.shard(n, world, sd.owner(c, n, world))


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


def test_gloo_world8_ragged_100_chains():
    """The metric's own N = 8 form on the CPU: 100 chains over 8 gloo ranks in ragged contiguous shards (12 or 13
    chains each, bench.py --gpus 8 --total-chains 100), both collectives and the statistics equal to one process
    holding all 100 chains (script.py:55-99)."""
    world, n_total = 8, 100
    assert sorted({len(sd.shard(n_total, world, r)) for r in range(world)}) == [12, 13]
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    rows, sel, sab, scd, stats = _single_process(n_total)
    assert 0 < len(sel) <= K
    for r in range(world):
        b, s_, ab_b, cd_b, st, dev_same = out[r]
        assert dev_same
        assert b == rows.tobytes() and s_ == sel
        assert ab_b == sab.tobytes() and cd_b == scd.tobytes()
        assert st == stats
