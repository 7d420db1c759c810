"""Multi-GPU chain sharding and the one collective.

Chains are independent given their seed, so ranks never talk while sampling.  One
process per GPU owns a contiguous block of chains.  At the end:
  1. every rank contributes a fixed-size summary record per chain (chain_id, exp_loglik,
     exp_c, exp_d -- the exp_data.csv payload, mcmc.c:53-67) to ONE all-gather (RCCL over
     xGMI with the "nccl" backend, gloo in the CPU tests), after which every rank runs the
     one-sigma chain selection of script.py:70-99 locally and identically;
  2. the selected chains' saved samples (a, b, pi rows + c, d, loglik) -- the input of
     script.py:102-189 (E[c], E[d], CORRMN, pair-order matrix) -- are all-gathered from the
     ranks that own them (one collective of k_max selected chains per rank, k_max = the
     largest number of selected chains any one rank owns), so any rank can compute the
     posterior statistics exactly as a single-GPU run does.
"""
import math

import numpy as np

from .launcher import choose_from_values

SUMMARY_FIELDS = ("chain_id", "exp_loglik", "exp_c", "exp_d")


def shard(n_chains, world, rank):
    """Contiguous block of chain indices owned by `rank`: [r*C/G, (r+1)*C/G)."""
    if world <= 0 or not 0 <= rank < world or n_chains < 0:
        raise ValueError("bad shard arguments")
    return range(rank * n_chains // world, (rank + 1) * n_chains // world)


def summaries_from_records(chain_ids, cdl):
    """Per-chain summary rows from saved-sample records cdl[chain, sample, (c, d, loglik)]
    exactly as compute_exp_data / print_exp_data (mcmc.c:53-67): sums over the saved
    samples in order, divided by 1000 (the reference hard-codes the divisor)."""
    rows = np.asarray(cdl, np.float64).tolist()
    out = np.zeros((len(chain_ids), 4))
    for k, cid in enumerate(chain_ids):
        ls = cs = ds = 0.0
        for c, d, ll in rows[k]:   # math.exp is the C library's exp, as in mcmc.c
            ls += -ll
            cs += math.exp(c)
            ds += math.exp(d)
        out[k] = (cid, ls / 1000, cs / 1000, ds / 1000)
    return out


def gather_summaries(rows, n_total, device="cpu", group=None):
    """All-gather every rank's summary rows [n_local, 4] (float64) into [n_total, 4],
    ordered by chain_id.  Shards may be ragged: each rank pads to the largest shard
    with chain_id = -1 rows, so the collective is a single fixed-size all_gather."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    width = max(len(shard(n_total, world, r)) for r in range(world))
    buf = torch.full((width, 4), -1.0, dtype=torch.float64, device=device)
    if len(rows):
        buf[:len(rows)] = torch.as_tensor(np.asarray(rows, np.float64), device=device)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    allrows = torch.cat(parts).cpu().numpy()
    allrows = allrows[allrows[:, 0] >= 0]
    allrows = allrows[np.argsort(allrows[:, 0], kind="stable")]
    if len(allrows) != n_total or not np.array_equal(allrows[:, 0], np.arange(n_total)):
        raise RuntimeError("gathered summaries do not cover chains 0..%d" % (n_total - 1))
    return allrows


def select_chains(all_rows, chains_selected):
    """script.py choose_chains on gathered rows (chain dirs named as the reference does)."""
    vals = {"chain_%02d" % int(r[0]): float(r[1]) for r in all_rows}
    return choose_from_values(vals, chains_selected)


def owner(chain_id, n_total, world):
    """Rank whose contiguous shard holds chain_id."""
    for r in range(world):
        sh = shard(n_total, world, r)
        if sh.start <= chain_id < sh.stop:
            return r
    raise ValueError("chain %d outside 0..%d" % (chain_id, n_total - 1))


def gather_selected_records(selected, n_total, local_ids, ab_pi, cdl, device="cpu", group=None):
    """Step 2 of the collective: the saved samples of the `selected` chain ids, in selection
    order, on every rank.  local_ids: this rank's chain ids (its shard); ab_pi [n_local, T, W]
    int16 and cdl [n_local, T, 3] float64 are its records (T saved calls, W = 2M + N).
    One all_gather per array of [k_max, T, ...] slabs (int16 rows travel as bytes: RCCL has no
    16-bit integer type).  Returns (ab_pi [k, T, W] int16, cdl [k, T, 3] float64)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    ab_pi = np.ascontiguousarray(ab_pi, np.int16)
    cdl = np.ascontiguousarray(cdl, np.float64)
    T, W = ab_pi.shape[1], ab_pi.shape[2]
    owners = [owner(int(c), n_total, world) for c in selected]
    k_max = max([owners.count(r) for r in range(world)] + [1])
    pos = {int(c): k for k, c in enumerate(local_ids)}
    mine = [int(c) for c, o in zip(selected, owners) if o == rank]
    sab = np.zeros((k_max, T, W), np.int16)
    scd = np.zeros((k_max, T, 3), np.float64)
    for j, c in enumerate(mine):
        sab[j] = ab_pi[pos[c]]
        scd[j] = cdl[pos[c]]
    tab = torch.as_tensor(sab.view(np.uint8), device=device)
    tcd = torch.as_tensor(scd, device=device)
    pab = [torch.empty_like(tab) for _ in range(world)]
    pcd = [torch.empty_like(tcd) for _ in range(world)]
    dist.all_gather(pab, tab, group=group)
    dist.all_gather(pcd, tcd, group=group)
    gab = [p.cpu().numpy().view(np.int16).reshape(k_max, T, W) for p in pab]
    gcd = [p.cpu().numpy() for p in pcd]
    out_ab = np.zeros((len(selected), T, W), np.int16)
    out_cd = np.zeros((len(selected), T, 3), np.float64)
    slot = [0] * world
    for k, o in enumerate(owners):
        out_ab[k] = gab[o][slot[o]]
        out_cd[k] = gcd[o][slot[o]]
        slot[o] += 1
    return out_ab, out_cd


def selected_records_workspace(k_cap, T, W, device, group=None):
    """Device buffers for gather_selected_records_device, allocated ahead of a timed region (up to k_cap
    selected chains per rank): the slab, the per-rank receive buffers and the output."""
    import torch
    import torch.distributed as dist
    on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if on else 1
    gloo = on and dist.get_backend(group) == "gloo"
    rdev = "cpu" if gloo else device
    ws = {"k_cap": k_cap,
          "sab": torch.zeros((k_cap, T, W), dtype=torch.int16, device=device),
          "scd": torch.zeros((k_cap, T, 3), dtype=torch.float64, device=device)}
    if world > 1:
        ws["pab"] = [torch.empty((k_cap, T, 2 * W), dtype=torch.uint8, device=rdev) for _ in range(world)]
        ws["pcd"] = [torch.empty((k_cap, T, 3), dtype=torch.float64, device=rdev) for _ in range(world)]
        ws["out_ab"] = torch.empty((k_cap, T, 2 * W), dtype=torch.uint8, device=rdev)
        ws["out_cd"] = torch.empty((k_cap, T, 3), dtype=torch.float64, device=rdev)
    return ws


def gather_selected_records_device(selected, n_total, local_ids, copy_chain, T, W, device, group=None, ws=None):
    """Step 2 on the device: the saved samples of the `selected` chain ids, in selection order, without a host
    round trip.  Each rank queues device-to-device copies of the selected chains it owns (copy_chain(local_index,
    ab_ptr, cdl_ptr): sr_session_copy_chain_records on the stream the collective runs on) into its slab of a
    [k_max, T, W] int16 / [k_max, T, 3] float64 buffer on `device`, then ONE all-gather per array moves the slabs
    (int16 rows as bytes: RCCL has no 16-bit integer type).  At world 1 (no process group) the copies alone.
    Returns device tensors (ab_pi [k, T, W] int16, cdl [k, T, 3] float64).  With a gloo group (the one-GPU
    rehearsal) the slabs cross through host tensors, as gloo requires."""
    import torch
    import torch.distributed as dist
    on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if on else 1
    rank = dist.get_rank(group) if on else 0
    owners = [owner(int(c), n_total, world) for c in selected]
    k_max = max([owners.count(r) for r in range(world)] + [1])
    pos = {int(c): k for k, c in enumerate(local_ids)}
    mine = [int(c) for c, o in zip(selected, owners) if o == rank]
    if ws is not None and ws["k_cap"] >= k_max and ws["k_cap"] >= len(selected):
        sab, scd = ws["sab"][:k_max], ws["scd"][:k_max]
    else:
        ws = None
        sab = torch.zeros((k_max, T, W), dtype=torch.int16, device=device)
        scd = torch.zeros((k_max, T, 3), dtype=torch.float64, device=device)
    for j, c in enumerate(mine):
        copy_chain(pos[c], sab[j].data_ptr(), scd[j].data_ptr())
    if world == 1:
        return sab[:len(selected)], scd[:len(selected)]
    gloo = dist.get_backend(group) == "gloo"
    tab = sab.view(torch.uint8).cpu() if gloo else sab.view(torch.uint8)
    tcd = scd.cpu() if gloo else scd
    if ws is not None:
        pab, pcd = [t[:k_max] for t in ws["pab"]], [t[:k_max] for t in ws["pcd"]]
    else:
        pab = [torch.empty_like(tab) for _ in range(world)]
        pcd = [torch.empty_like(tcd) for _ in range(world)]
    dist.all_gather(pab, tab, group=group)
    dist.all_gather(pcd, tcd, group=group)
    slot = [0] * world
    idx = []
    for o in owners:
        idx.append((o, slot[o]))
        slot[o] += 1
    k = len(selected)
    if ws is not None:
        out_ab = torch.stack([pab[o][j] for o, j in idx], out=ws["out_ab"][:k])
        out_cd = torch.stack([pcd[o][j] for o, j in idx], out=ws["out_cd"][:k])
    else:
        out_ab = torch.stack([pab[o][j] for o, j in idx])
        out_cd = torch.stack([pcd[o][j] for o, j in idx])
    return out_ab.to(device).view(torch.int16), out_cd.to(device)


def selection_statistics(ab_pi, cdl, N, M, chains_selected):
    """E[c], E[d], CORRMN of script.py:102-152 on the selected chains' records (record form of
    analysis.compute_exp_cd / compute_exp_ages)."""
    from . import analysis
    ec, ed = analysis.exp_cd_from_records(list(cdl), chains_selected)
    corr = analysis.corr_mn_from_records([np.asarray(r)[:, 2 * M:2 * M + N] for r in ab_pi], chains_selected)
    return ec, ed, corr
