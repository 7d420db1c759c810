"""GPU parity on edge-case datasets (every integer and f64 bit against the oracle).

Covers: tiny matrices, no hard sites, many hard sites (<= 64), N - nh < 2 (pi3 always vetoed), N > 2048,
M not a multiple of 64, all-zero columns, N on a word boundary, the register-resident Gibbs
kernels (walks of <= 9 and <= 17 words) and the LDS-walk kernel (longer walks), block sizes
256 / 512 / 1024 and several taxa per thread.
"""
import numpy as np
import pytest

import oracle_ref
import seriation_amd as sa
from seriation_amd import _lib as L

pytestmark = pytest.mark.gpu


def make_text(N, M, nh, seed, zero_cols=2, density=0.15, noise=0.02):
    rng = np.random.default_rng(seed)
    X = np.zeros((N, M), np.uint8)
    for m in range(M):
        a = rng.integers(0, N)
        L = rng.integers(1, max(2, N // 2) + 1)
        col = (rng.random(N) < noise).astype(np.uint8)
        col[a:min(N, a + L)] = (rng.random(min(N, a + L) - a) < density * 3).astype(np.uint8)
        X[:, m] = col
    X[:, rng.choice(M, size=min(zero_cols, M), replace=False)] = 0
    hard = np.zeros(N, bool)
    hard[rng.choice(N, size=nh, replace=False)] = True
    lines = ["%d %d" % (N, M)]
    for i in range(N):
        lines.append(" ".join(str(v) for v in X[i]) + (" *" if hard[i] else ""))
    return ("\n".join(lines) + "\n").encode()


CASES = [
    # name, N, M, nh, block_threads
    ("tiny", 3, 5, 0, 0),
    ("pi3-veto", 3, 6, 2, 0),
    ("two-sites", 2, 4, 0, 0),
    ("no-hard", 40, 70, 0, 0),
    ("many-hard", 60, 100, 30, 0),
    ("nh32", 90, 64, 32, 0),
    ("nh40", 120, 70, 40, 0),
    ("nh64", 150, 64, 64, 0),
    # more than 64 hard sites: the bitmap paths (hard ones of a column from the wave's hard bitmap, hard
    # positions in several waves of lanes)
    ("nh65", 160, 70, 65, 0),
    ("nh200", 300, 90, 200, 0),
    ("nh-n-1-big", 130, 40, 129, 0),
    ("n2500", 2500, 24, 10, 0),
    # nh = N - 1 / N - 2: mcmc_randomize's hard-position scan reads q[nh] past the end there
    # (mcmc.c:530, UB); host and oracle both stop at nh (the intended reading)
    ("nh-n-1", 40, 30, 39, 0),
    ("nh-n-2", 41, 30, 39, 0),
    ("word-boundary-256", 256, 64, 12, 0),
    ("walk17", 300, 130, 9, 0),
    ("lds-walk", 600, 80, 7, 0),
    ("tb256-2-per-thread", 96, 512, 5, 256),
    ("tb1024", 64, 700, 4, 0),
    ("3-per-thread", 64, 1100, 6, 0),
]


@pytest.mark.parametrize("name,N,M,nh,tb", CASES, ids=[c[0] for c in CASES])
def test_edge_parity(name, N, M, nh, tb):
    text = make_text(N, M, nh, seed=N * 1000 + M)
    ds = sa.Dataset.parse(text, maxs=0)
    seeds = [1, 7]
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=2, sample_calls=3, keep_records=True, block_threads=tb)
    for k, s in enumerate(seeds):
        o = oracle_ref.run_chain(text, s, 2, 3, maxs=0)
        assert o["rc"] == 0
        np.testing.assert_array_equal(ri[k], o["rec_int"], err_msg="%s seed %d" % (name, s))
        assert np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64)), (name, s)
        assert summ[k]["consistent"] == 0


# The HBM-column variant (columns, prefix tables, a/b, counts in HBM; chosen automatically when
# the LDS layout exceeds 160 KB) forced on small cases: same bits as the oracle.
HBM_CASES = [c for c in CASES if c[0] in ("tiny", "many-hard", "nh64", "nh200", "n2500", "walk17", "lds-walk",
                                          "tb256-2-per-thread", "3-per-thread")]


@pytest.mark.parametrize("name,N,M,nh,tb", HBM_CASES, ids=["hbm-" + c[0] for c in HBM_CASES])
def test_edge_parity_hbm_columns(name, N, M, nh, tb):
    text = make_text(N, M, nh, seed=N * 1000 + M)
    ds = sa.Dataset.parse(text, maxs=0)
    seeds = [3, 11]
    with sa.Session(ds, seeds, block_threads=tb, columns="hbm") as s:
        assert s.variant == "hbm"
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=2, sample_calls=3, keep_records=True, block_threads=tb,
                                   columns="hbm")
    for k, s in enumerate(seeds):
        o = oracle_ref.run_chain(text, s, 2, 3, maxs=0)
        assert o["rc"] == 0
        np.testing.assert_array_equal(ri[k], o["rec_int"], err_msg="%s seed %d" % (name, s))
        assert np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64)), (name, s)
        assert summ[k]["consistent"] == 0


@pytest.mark.parametrize("N,M,noise,seeds,burnin", [(256, 300, 0.003, [4], 60), (400, 150, 0.02, [4, 19], 45)],
                         ids=["walk9", "walk17"])
def test_steep_walks(N, M, noise, seeds, burnin):
    """Ranges filled with ones (little noise outside): once the order settles d ends near its bound 0.2
    and |vA| = |log2(d / (1 - c))| near its largest value, the regime where Gibbs walks sink deepest
    between window words (draw_fast_s: the 9-word walks rely on the bound -40 - 32 nk |vA| > -710
    and take no test; the 17-word walks test for window word starts below 2^-700).  Same bits as
    the oracle."""
    text = make_text(N, M, 5, seed=N * 7 + M, density=0.34, noise=noise)
    ds = sa.Dataset.parse(text, maxs=0)
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=burnin, sample_calls=10, keep_records=True)
    for k, s in enumerate(seeds):
        o = oracle_ref.run_chain(text, s, burnin, 10, maxs=0)
        assert o["rc"] == 0
        np.testing.assert_array_equal(ri[k], o["rec_int"], err_msg="seed %d" % s)
        assert np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64)), s
        assert summ[k]["consistent"] == 0
        # the steep regime on the last call: 32 nk |vA| > 650 with its c, d (log values in the records)
        c, d = np.exp(rd[k][-1, 0]), np.exp(rd[k][-1, 1])
        assert 32 * ((N >> 5) + 1) * abs(np.log2(d / (1 - c))) > 650, (c, d)


# Split chains (two workgroups per chain exchanging sums through HBM flags), forced on small HBM-column
# cases at 1024 threads (SR_SPLIT=1; by default only chains of 1025..2048 taxa split).
SPLIT_CASES = [("m700", 64, 700, 4), ("m1100", 64, 1100, 6), ("nh64", 150, 1200, 64), ("lds-walk", 600, 1300, 7),
               ("many-hard", 60, 1500, 30), ("n1300", 1300, 1100, 8)]   # n1300: 11 LDS checkpoint slots per thread,
# the largest split layout of round 5 (the per-wave hard tables of round 4's layout did not fit 160 KB there)


@pytest.mark.parametrize("name,N,M,nh", SPLIT_CASES, ids=["split-" + c[0] for c in SPLIT_CASES])
def test_split_chain_parity(monkeypatch, name, N, M, nh):
    monkeypatch.setenv("SR_SPLIT", "1")
    text = make_text(N, M, nh, seed=N * 1000 + M)
    ds = sa.Dataset.parse(text, maxs=0)
    seeds = [5, 13, 21]
    with sa.Session(ds, seeds, block_threads=1024, columns="hbm") as s:
        assert s.variant == "hbm" and s.kernel == "split"
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=2, sample_calls=3, keep_records=True, block_threads=1024,
                                   columns="hbm")
    for k, s in enumerate(seeds):
        o = oracle_ref.run_chain(text, s, 2, 3, maxs=0)
        assert o["rc"] == 0
        np.testing.assert_array_equal(ri[k], o["rec_int"], err_msg="%s seed %d" % (name, s))
        assert np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64)), (name, s)
        assert summ[k]["consistent"] == 0
    # the per-half counters (a / b changes, exact-walk fallbacks) add up to the one-workgroup kernel's
    counts = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("SR_SPLIT", mode)
        with sa.Session(ds, seeds, block_threads=1024, columns="hbm") as s:
            assert s.kernel == ("split" if mode == "1" else "single")
            s.run(5)
            counts[mode] = [np.concatenate([s.accept_counts(k), s.fallback_counts(k)]) for k in range(len(seeds))]
    np.testing.assert_array_equal(np.array(counts["1"]), np.array(counts["0"]))


@pytest.mark.parametrize("N,M,nh", [(3000, 1100, 9), (1700, 1500, 70), (1024, 3000, 200)],
                         ids=["n3000", "n1700-nh70", "n1024-nh200"])
def test_hbm_columns_1024_threads_long_columns(monkeypatch, N, M, nh):
    """HBM columns at 1024 threads with long columns (round 5: one block-shared copy of the hard-site and 4-step
    tables; the per-wave copies of 16 waves passed 160 KB of LDS at N ~ 1250, so these shapes had no kernel).
    One-workgroup kernel (SR_SPLIT=0) and, where its layout fits, the split kernel, both against the oracle."""
    text = make_text(N, M, nh, seed=N * 7 + M)
    ds = sa.Dataset.parse(text, maxs=0)
    seeds = [3, 11]
    orc = [oracle_ref.run_chain(text, s, 2, 3, maxs=0) for s in seeds]
    for mode in ("0", "1"):
        monkeypatch.setenv("SR_SPLIT", mode)
        with sa.Session(ds, seeds, block_threads=1024, columns="hbm") as s:
            assert s.variant == "hbm"
            kern = s.kernel
        if mode == "1" and kern != "split":
            continue   # (the split layout, LDS checkpoints included, does not fit at this N)
        summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=2, sample_calls=3, keep_records=True,
                                       block_threads=1024, columns="hbm")
        for k, o in enumerate(orc):
            assert o["rc"] == 0
            np.testing.assert_array_equal(ri[k], o["rec_int"], err_msg="N %d mode %s seed %d" % (N, mode, seeds[k]))
            assert np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64)), (N, mode, seeds[k])
            assert summ[k]["consistent"] == 0


@pytest.mark.parametrize("name,N,M,nh", [("m1100", 64, 1100, 6), ("many-hard", 60, 1500, 30)], ids=["split512-m1100",
                                                                                                  "split512-many-hard"])
def test_split_512_thread_halves_parity(monkeypatch, name, N, M, nh):
    """The opt-in 512-thread split (SR_SPLIT=2: halves of up to 1024 taxa, several taxa per thread, 256 VGPRs)
    equals the oracle, ragged halves and the Gibbs step's rounds of 512 taxa included."""
    monkeypatch.setenv("SR_SPLIT", "2")
    text = make_text(N, M, nh, seed=N * 1000 + M)
    ds = sa.Dataset.parse(text, maxs=0)
    seeds = [5, 13, 21]
    with sa.Session(ds, seeds, block_threads=512, columns="hbm") as s:
        assert s.variant == "hbm" and s.kernel == "split" and s.block_threads == 512
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=2, sample_calls=3, keep_records=True, block_threads=512,
                                   columns="hbm")
    for k, s in enumerate(seeds):
        o = oracle_ref.run_chain(text, s, 2, 3, maxs=0)
        assert o["rc"] == 0
        np.testing.assert_array_equal(ri[k], o["rec_int"], err_msg="%s seed %d" % (name, s))
        assert np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64)), (name, s)
        assert summ[k]["consistent"] == 0


# Ragged split halves (round 5 audit, DESIGN.md 4 "cross-thread orderings"): the second half starts at
# olo = sr_sp_half(M), not a multiple of the block, so the Gibbs step's rounds of TB taxa (taken when 2M words
# exceed the resident RNG ring, M > 1360) hand some of the half's taxa to threads other than their owners in
# phases A / C; a barrier orders those writes before phase C.  One geometry per case: Gibbs rounds touching the
# half (1, 2, 3), block 1024 or the opt-in 512 (several taxa per thread), more than 64 hard sites (the bitmap
# paths) -- name, N, M, nh, block_threads, SR_SPLIT, Gibbs rounds inside the second half.
RAGGED = [("r1-nh100", 150, 1000, 100, 1024, "1", 1), ("r2-nh80", 120, 1700, 80, 1024, "-1", 2),
          ("r2-tb512-nh70", 100, 1500, 70, 512, "2", 2), ("r3-tb512-nh66", 100, 1900, 66, 512, "2", 3)]


def _sp_half(M):
    return (((M + 1) // 2) + 63) & ~63


@pytest.mark.parametrize("name,N,M,nh,tb,split,rounds", RAGGED, ids=["ragged-" + c[0] for c in RAGGED])
def test_split_ragged_half_geometries(monkeypatch, name, N, M, nh, tb, split, rounds):
    olo = _sp_half(M)
    assert olo % tb != 0   # the ragged second half
    ring_rounds = 1 if 2 * M + 1024 <= 7 * 624 - 623 else -(-M // tb)
    touching = 1 if ring_rounds == 1 else len({m // tb for m in range(olo, M)})
    assert touching == rounds, (name, touching)
    if split == "-1":
        monkeypatch.delenv("SR_SPLIT", raising=False)
    else:
        monkeypatch.setenv("SR_SPLIT", split)
    text = make_text(N, M, nh, seed=N * 1000 + M + 5)
    ds = sa.Dataset.parse(text, maxs=0)
    seeds = [3, 8, 30]
    with sa.Session(ds, seeds, block_threads=tb, columns="hbm") as s:
        assert s.variant == "hbm" and s.kernel == "split" and s.block_threads == tb
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=2, sample_calls=3, keep_records=True, block_threads=tb,
                                   columns="hbm")
    for k, sd_ in enumerate(seeds):
        o = oracle_ref.run_chain(text, sd_, 2, 3, maxs=0)
        assert o["rc"] == 0
        np.testing.assert_array_equal(ri[k], o["rec_int"], err_msg="%s seed %d" % (name, sd_))
        assert np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64)), (name, sd_)
        assert summ[k]["consistent"] == 0


def test_checkpoint_resume_continues_exactly(tmp_path):
    """sr_session_checkpoint after 10 calls + sr_session_restore + 20 calls == 30 calls straight."""
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "datasets", "g5s5.txt")
    ds = sa.Dataset.load(path)
    seeds = [1, 2, 3, 4]
    with sa.Session(ds, seeds, calls_per_launch=30) as s:
        s.run(30, save=True)
        ab_full, cdl_full = s.fetch_records()
    ck = str(tmp_path / "chains.srck")
    with sa.Session(ds, seeds, calls_per_launch=30) as s:
        s.run(10, save=False)
        s.checkpoint(ck)
    r = sa.Session.restore(ds, ck, calls_per_launch=30)
    try:
        assert r.n == len(seeds)
        r.run(20, save=True)
        ab2, cdl2 = r.fetch_records()
    finally:
        r.close()
    assert np.array_equal(ab_full[:, 10:], ab2)
    assert np.array_equal(cdl_full[:, 10:].view(np.uint64), cdl2.view(np.uint64))


@pytest.mark.parametrize("manycd", [0, 1])
def test_checkpoint_carries_records(tmp_path, manycd):
    """Checkpoints keep the buffered records and the record capacity (version 7 / 8): 500 saved calls + checkpoint
    + restore + 500 saved calls give the same 1000 records and the same exp_data rows (compute_exp_data over the
    whole sampling phase, mcmc.c:53-67) bit for bit as 1000 calls straight -- manycd sessions with their per-taxon
    c, d too.  The restore passes default options: the checkpointed session's capacity (1000) comes back with it."""
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "datasets", "g10s10.txt")
    ds = sa.Dataset.load(path)
    seeds = [5, 6, 7]
    T, H = (1000, 500) if not manycd else (60, 25)
    with sa.Session(ds, seeds, calls_per_launch=T, manycd=manycd) as s:
        s.run(T, save=True)
        ab_full, cdl_full = s.fetch_records()
        sum_full = s.summaries()
        cv_full = s.fetch_cd_vectors() if manycd else None
    ck = str(tmp_path / "rec.srck")
    with sa.Session(ds, seeds, calls_per_launch=T, manycd=manycd) as s:
        s.run(H, save=True)
        s.checkpoint(ck)
    with open(ck, "rb") as fh:
        head = fh.read(40)
    assert np.frombuffer(head, "<u4", 1, 4)[0] == (8 if manycd else 7)
    assert np.frombuffer(head, "<i4", 2, 32).tolist() == [H, T]
    r = sa.Session.restore(ds, ck, manycd=manycd)
    try:
        assert L.lib().sr_session_records(r.h) == H and r.record_capacity >= T
        r.run(T - H, save=True)
        ab2, cdl2 = r.fetch_records()
        sum2 = r.summaries()
        cv2 = r.fetch_cd_vectors() if manycd else None
    finally:
        r.close()
    assert np.array_equal(ab_full, ab2)
    assert np.array_equal(cdl_full.view(np.uint64), cdl2.view(np.uint64))
    assert np.array_equal(sum_full.view(np.uint64), sum2.view(np.uint64))
    if manycd:
        assert np.array_equal(cv_full.view(np.uint64), cv2.view(np.uint64))


def _all_ones_text(N, M, hard_rows):
    lines = ["%d %d" % (N, M)] + [" ".join("1" * M) + (" *" if i in hard_rows else "") for i in range(N)]
    return ("\n".join(lines) + "\n").encode()


@pytest.mark.parametrize("columns", ["lds", "hbm"])
def test_johnk_beta_branch(columns):
    """An all-ones matrix: every taxon spans every site (a = 0, b = N), so t0a = f1a = 0 and
    mcmc_samplec's gsl_ran_beta(1 + 0, 1 + 0) takes GSL's Johnk branch (both shapes <= 1), not the
    gamma ratio -- every word it consumes must match the oracle's restatement (oracle/om_gsl.h)."""
    text = _all_ones_text(40, 24, {5, 17, 30})
    ds = sa.Dataset.parse(text, maxs=0)
    seeds = [2, 9, 31]
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=3, sample_calls=6, keep_records=True, columns=columns)
    for k, s in enumerate(seeds):
        o = oracle_ref.run_chain(text, s, 3, 6, maxs=0)
        assert o["rc"] == 0
        np.testing.assert_array_equal(ri[k], o["rec_int"], err_msg="seed %d" % s)
        assert np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64)), s
        assert summ[k]["consistent"] == 0


PAIR_CASES = [("synth-like", 256, 512, 12), ("m300", 200, 300, 5), ("n287", 287, 400, 9), ("nh0", 128, 260, 0)]


@pytest.mark.parametrize("name,N,M,nh", PAIR_CASES, ids=[c[0] for c in PAIR_CASES])
def test_pair_kernel_parity(monkeypatch, name, N, M, nh):
    """The opt-in pair kernel (SR_KERNEL=pair: two lanes per taxon, each walking half of a Gibbs
    column; proposal terms in slot pairs) is bit-exact too (it is slower: DESIGN.md section 4)."""
    monkeypatch.setenv("SR_KERNEL", "pair")
    text = make_text(N, M, nh, seed=N * 1000 + M + 7)
    ds = sa.Dataset.parse(text, maxs=0)
    seeds = [4, 19]
    with sa.Session(ds, seeds) as s:
        assert s.kernel == "pair" and s.block_threads == 1024
    summ, (ri, rd) = sa.run_chains(ds, seeds, burnin_calls=3, sample_calls=4, keep_records=True)
    for k, s in enumerate(seeds):
        o = oracle_ref.run_chain(text, s, 3, 4, maxs=0)
        assert o["rc"] == 0
        np.testing.assert_array_equal(ri[k], o["rec_int"], err_msg="%s seed %d" % (name, s))
        assert np.array_equal(rd[k].view(np.uint64), o["rec_dbl"].view(np.uint64)), (name, s)
        assert summ[k]["consistent"] == 0


def test_taxa_beyond_int16():
    """M = 40 000 taxa (beyond int16; the records hold positions only): HBM columns, one workgroup of 1024
    threads with ~40 taxa per thread, one chain x (1 + 2) calls equal to the oracle bit for bit."""
    N, M = 40, 40000
    text = make_text(N, M, 3, seed=4040000)
    ds = sa.Dataset.parse(text, maxs=0)
    with sa.Session(ds, [2]) as s:
        assert s.variant == "hbm" and s.block_threads == 1024
    summ, (ri, rd) = sa.run_chains(ds, [2], burnin_calls=1, sample_calls=2, keep_records=True)
    o = oracle_ref.run_chain(text, 2, 1, 2, maxs=0)
    assert o["rc"] == 0
    np.testing.assert_array_equal(ri[0], o["rec_int"])
    assert np.array_equal(rd[0].view(np.uint64), o["rec_dbl"].view(np.uint64))
    assert summ[0]["consistent"] == 0
