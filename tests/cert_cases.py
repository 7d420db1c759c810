"""Adversarial inputs for the certification self-tests -- TEST INFRASTRUCTURE.

The sampler's fast paths are exact only because two analytic error bounds hold:
  * the Gibbs pick (mcmc_auxa + mcmc_logtop + mcmc_randompick, mcmc.c:828-915): the fast walk's CDF F^ is within
    REL * min(F, S - F) + ABS of the reference's sequentially summed, clamped CDF (csrc/sr_device.hip, draw_fast /
    walk_pick_s), so a pick is accepted only when u lies farther than that from both neighbouring boundaries;
  * phase C's decision (mcmc.c:492 / 569 / 637: delta >= 0 || delta > log u): the exact sum S of the exact terms is
    within Eb = (Knz + 16) 2^-52 B of the reference's rounded, sequentially summed delta (pc_classify / pc_resolve).
A uniform u lands in the band where an understated bound would answer wrongly about once in 1e13 draws, so chain
parity cannot see one.  These generators put the inputs on the band: u on the reference's own CDF boundaries
(found by bisection over the doubles with the oracle's exact pick) and at a ladder of distances around them, from
one ulp to twice the margin; and term lists whose reference delta crosses 0 or log u (c, d chosen by bisection), at
a ladder of ulp distances in d around the crossing.  Every expected answer is the oracle's (oracle/om_mcmc.c).
"""
import math

import numpy as np

import oracle_ref

MINC, MAXC = -6.9077552789821368, -2.3025850929940455   # mcmc.h:27-28 (log .001, log .1)
MIND, MAXD = -1.6094379124341003, -0.22314355131420971  # mcmc.h:29-30 (log .2, log .8)
LOGEPS = -32.236191301916641                            # mcmc.h:26


def _step(x, k):
    b = int(np.array([x], np.float64).view(np.int64)[0])
    if x < 0:
        raise ValueError("non-negative only")
    return float(np.array([max(0, b + k)], np.int64).view(np.float64)[0])


def cd_grid():
    """(c, d) pairs: the corners of mcmc_samplebeta's bounds (the steepest and flattest walks) and interior points."""
    cs = [MINC, MAXC, math.log(0.01), math.log(0.03)]
    ds = [MIND, MAXD, math.log(0.5), math.log(0.35)]
    return [(c, d) for c in cs for d in ds]


# ----------------------------------------------------------------------------------------------- Gibbs picks
def _margin(N):
    """The product's absolute slack ABS (draw_fast: (N + 1) 2^-39 + 2^-46), the scale of the u ladder."""
    return (N + 1) * 2.0 ** -39 + 2.0 ** -46


def u_ladder(ub, N):
    """u values around a boundary ub: the boundary itself and +-1, 2, 4, 16, 256 ulps, +-f * ABS for f from 2 down
    to 2^-11 in quarter-octave steps (the band an understated bound, e.g. ABS / 2^8, fails in), and from 2^1.5 up to
    2^10.5 in half-octave steps (where the fast path certifies)."""
    out = {ub}
    for k in (1, 2, 4, 16, 256):
        out.add(_step(ub, k))
        if ub > 0:
            out.add(_step(ub, -k))
    A = _margin(N)
    for q in range(0, 49):
        f = 2.0 ** (1 - q / 4.0)
        out.add(ub + f * A)
        out.add(ub - f * A)
    for q in range(3, 22):   # and out to 2^10 ABS: the fast path certifies there (its picks are checked too)
        f = 2.0 ** (q / 2.0)
        out.add(ub + f * A)
        out.add(ub - f * A)
    return sorted(u for u in out if 0.0 <= u < 1.0)


def walk_bits(col, N, rev, L):
    """Walk-order bits x[0..L) of a position-ordered column (rev: walk entry w = position N - 1 - w)."""
    col = np.asarray(col, np.int32)
    return (col[::-1] if rev else col)[:L].copy()


def _boundaries(x, o, c, d, extra):
    """Entries whose upper CDF boundary the ladder probes: the heaviest few, the ends of the mass, and `extra`."""
    _, p = oracle_ref.auxa_pick(x, o, c, d, 0.5, want_p=True)
    L = len(x)
    order = list(np.argsort(-p, kind="stable"))
    pick = set(int(i) for i in order[:4])
    big = np.nonzero(p > p.max() * 2.0 ** -30)[0]
    for i in (big[0] - 1, big[0], big[-1] - 1, big[-1], big[-1] + 1, o - 1, o):
        pick.add(int(i))
    pick.update(int(i) for i in extra)
    return sorted(i for i in pick if 0 <= i < L)


def gibbs_block_columns(kind, N, rng):
    """One column (position order, 0/1 int32) and a walk (rev, o, L) of the given kind:
       "random"  -- density ~ U(0.05, 0.6) inside a random interval, ~0.02 outside (the synthetic data's shape);
       "tail"    -- a short heavy region at the start of the walk, then a long run of ones: every later entry is
                    clamped at e^LOGEPS by the reference (the clamped mass is what ABS covers);
       "steep"   -- long runs of zeros (q climbs |vA| bits per entry: the y chain spans the widest range);
       "rise"    -- zeros after the start (for N in the thousands the window's q range passes SR_QSPAN: trims)."""
    col = np.zeros(N, np.int32)
    if kind == "random":
        lo = int(rng.integers(0, N // 2))
        hi = int(rng.integers(lo + 1, N + 1))
        col = (rng.random(N) < 0.02).astype(np.int32)
        col[lo:hi] = (rng.random(hi - lo) < rng.uniform(0.05, 0.6)).astype(np.int32)
        rev = bool(rng.integers(0, 2))
        L = int(rng.integers(max(1, N // 4), N + 1))
        o = int(rng.integers(0, L + 1))
    elif kind == "tail":
        rev = bool(rng.integers(0, 2))
        L, o = N, 0
        x = np.ones(L, np.int32)
        x[:6] = rng.integers(0, 2, 6)
        x[0] = 0
        col = x[::-1].copy() if rev else x
    elif kind == "steep":
        rev = bool(rng.integers(0, 2))
        L = N
        o = int(rng.integers(0, N // 8 + 1))
        x = (rng.random(L) < 0.03).astype(np.int32)
        col = x[::-1].copy() if rev else x
    elif kind == "rise":
        rev = False
        L = N
        o = 0
        col = (rng.random(N) < 0.002).astype(np.int32)
    else:
        raise ValueError(kind)
    return col, rev, o, L


def gibbs_cases(N, kinds, seed, blocks_per_kind):
    """Blocks of 64 cases sharing (c, d) and one column; returns dict of arrays for sr_device_selftest_gibbs plus
    the oracle's expected picks."""
    rng = np.random.default_rng(seed)
    grid = cd_grid()
    cols, cidx, cds, oo, LL, rv, uu, exp = [], [], [], [], [], [], [], []
    b = 0
    for kind in kinds:
        for _ in range(blocks_per_kind):
            c, d = grid[(b * 7 + seed) % len(grid)]
            b += 1
            col, rev, o, L = gibbs_block_columns(kind, N, rng)
            cols.append(col)
            x = walk_bits(col, N, rev, L)
            us = []
            for i in _boundaries(x, o, c, d, rng.integers(0, L, 2)):
                ub = oracle_ref.auxa_boundary(x, o, c, d, i)
                if 0.0 <= ub <= 1.0:
                    us.extend(u_ladder(ub, N))
            us = [0.0, 0.5, float(np.nextafter(1.0, 0.0))] + us
            rng.shuffle(us)
            # whole blocks of 64 lanes, each lane one u on this column
            for k0 in range(0, len(us), 64):
                chunk = us[k0:k0 + 64]
                chunk += [0.5] * (64 - len(chunk))
                cds.append((c, d))
                for u in chunk:
                    cidx.append(len(cols) - 1)
                    oo.append(o)
                    LL.append(L)
                    rv.append(1 if rev else 0)
                    uu.append(u)
                    exp.append(oracle_ref.auxa_pick(x, o, c, d, u))
    n = len(uu)
    NW = (N + 31) // 32
    ncol = len(cols)
    bits = np.zeros((ncol, NW * 32), np.uint8)
    bits[:, :N] = np.array(cols, np.uint8)
    words = (bits.reshape(ncol, NW, 32).astype(np.uint64) << np.arange(32, dtype=np.uint64)).sum(-1).astype(np.uint32)
    ones = np.concatenate([np.zeros((ncol, 1), np.int64), np.cumsum(bits.reshape(ncol, NW, 32).sum(-1), axis=1)], axis=1)
    ci = np.array(cidx)
    P = np.ascontiguousarray(words[ci].T)                                  # [NW][n]: bit p of word w = position 32w + p
    pre = np.ascontiguousarray(ones[ci].astype(np.uint16).T)               # [NW + 1][n]: ones before position 32w
    return dict(N=N, n=n, P=P, pre=pre, cd=np.array(cds, np.float64), o=np.array(oo, np.int32),
                L=np.array(LL, np.int32), rev=np.array(rv, np.int32), u=np.array(uu, np.float64),
                expected=np.array(exp, np.int32), cols=cols, cidx=ci)


def pick_counts(col, N, rev, o, r):
    """mcmc_auxa's dt0, df0, dt1, df1 at the pick r from limit o (the oracle's dt arrays at r)."""
    x = walk_bits(col, N, rev, max(o, r))
    if r == o:
        return 0, 0, 0, 0
    if r < o:
        O = int(x[r:o].sum())
        Z = (o - r) - O
        return -Z, Z, O, -O
    O = int(x[o:r].sum())
    Z = (r - o) - O
    return Z, -Z, -O, O


# ------------------------------------------------------------------------------------------ phase C decisions
def _log(v):
    """glibc-exact log (the oracle's om_log = the device's sr_log_m)."""
    return float(oracle_ref.exp_log(np.array([v]))[1][0])


def term_list(kind, rng, X0, X1, K):
    """Per-taxon (dt0, dt1) lists with the signal sums (X0, X1):
       "plain" -- the signal alone, spread one unit per taxon;
       "cancel" -- heavy terms that grow the partial sums and bring them back, then the signal (the sequential sum's
                   rounding is largest here: the bound's K-dependence is what it covers);
       "mixed" -- random small terms summing to the signal."""
    if kind == "plain":
        t0 = [int(np.sign(X0))] * abs(X0)
        t1 = [0] * abs(X0)
        t0 += [0] * abs(X1)
        t1 += [int(np.sign(X1))] * abs(X1)
        return np.array(t0 or [0], np.int32), np.array(t1 or [0], np.int32)
    if kind == "cancel":
        # K / 2 terms of dt1 = +2 grow the partial sums, K terms of dt1 = -1 bring them back: the sequential
        # rounding of the reference's sum accumulates over the climb and the descent separately (their residuals
        # modulo the ulp differ), up to ~1 % of Eb -- then the signal terms
        h = K // 2
        s0 = [int(np.sign(X0))] * abs(X0) + [0] * abs(X1)
        s1 = [0] * abs(X0) + [int(np.sign(X1))] * abs(X1)
        t0 = np.concatenate([np.zeros(3 * h, np.int64), s0]).astype(np.int32)
        t1 = np.concatenate([np.full(h, 2), np.full(2 * h, -1), s1]).astype(np.int32)
        return t0, t1
    if kind == "mixed":
        t0 = rng.integers(-2, 3, K).astype(np.int32)
        t1 = rng.integers(-1, 2, K).astype(np.int32)
        t0[-1] += X0 - int(t0.sum())
        t1[-1] += X1 - int(t1.sum())
        return t0, t1
    raise ValueError(kind)


def _d_crossing(t0, t1, c, target):
    """d in [MIND, MAXD] where the reference delta(d) - target changes sign (bisection over the ordered doubles of
    the interval, all negative: larger bit patterns are more negative); None when the ends do not bracket it."""
    f = lambda d: oracle_ref.delta_terms(t0, t1, c, d) - target
    lo, hi = MIND, MAXD
    flo, fhi = f(lo), f(hi)
    if (flo > 0) == (fhi > 0):
        return None
    blo = int(np.array([lo]).view(np.int64)[0])
    bhi = int(np.array([hi]).view(np.int64)[0])   # (bits(MIND) > bits(MAXD): the negative doubles order reversed)
    while blo - bhi > 1:
        mid = (blo + bhi) // 2
        dm = float(np.array([mid], np.int64).view(np.float64)[0])
        if (f(dm) > 0) == (flo > 0):
            blo = mid
        else:
            bhi = mid
    return float(np.array([bhi], np.int64).view(np.float64)[0])


def d_ladder(d):
    b = int(np.array([d]).view(np.int64)[0])
    out = {d}
    for k in [0] + [1 << j for j in range(0, 31)]:
        for s in (k, -k):
            v = float(np.array([b + s], np.int64).view(np.float64)[0])
            if MIND <= v <= MAXD:
                out.add(v)
    return sorted(out)


def _exact_ratio(t0, t1, c, d):
    """|reference delta - exact sum of the exact terms| / Eb at (c, d): how much of the bound the reference's own
    rounding uses (exact rationals; cc, dd as the oracle computes them)."""
    from fractions import Fraction as F
    e = oracle_ref.exp_log(np.array([c, d]))[0]
    cc, dd = (float(v) for v in oracle_ref.exp_log(1.0 - e)[1])
    X0, X1 = int(t0.sum()), int(t1.sum())
    ex = X0 * (F(cc) - F(d)) + X1 * (F(dd) - F(c))
    Y = int(np.abs(t0).sum() + np.abs(t1).sum())
    Eb = (2 * Y + 16) * 2.0 ** -52 * Y * (abs(cc) + abs(d) + abs(dd) + abs(c))
    return abs(float(F(oracle_ref.delta_terms(t0, t1, c, d)) - ex)) / Eb


def decide_cases(seed, n_combos=40, K=2000, tries=12):
    """Proposals whose reference delta crosses 0 or log u: returns dict(sums [n][4] int32, cd [n][2], uw [n] uint32,
    expected [n]: 1 accepted without u, 2 accepted with u, 0 rejected).  For the "cancel" term lists, `tries` values
    of c are drawn and the one whose crossing uses the largest share of Eb (the reference's rounding furthest from
    the exact sum) is kept."""
    rng = np.random.default_rng(seed)
    sums, cds, uws, exp = [], [], [], []
    kinds = ["cancel", "plain", "cancel", "mixed"]
    for t in range(n_combos):
        kind = kinds[t % 4]
        if t % 2 == 0:   # threshold 0: X0 A + X1 B = 0 needs opposite signs (A = cc - d > 0, B = dd - c > 0)
            X0 = int(rng.integers(1, 6))
            X1 = -int(rng.integers(1, 4))
            uw0 = int(rng.integers(1, 1 << 32))
        else:           # threshold log u: delta < 0
            X0 = -int(rng.integers(1, 4))
            X1 = int(rng.integers(-1, 1))
            uw0 = None
        t0, t1 = term_list(kind, rng, X0, X1, K)
        best = None
        for _ in range(tries if kind == "cancel" else 1):
            c = float(rng.uniform(MINC, MAXC))
            uw, target = uw0, 0.0
            if uw is None:
                # a u whose log lies between delta(MIND) and delta(MAXD), so a crossing exists
                a, b = oracle_ref.delta_terms(t0, t1, c, MIND), oracle_ref.delta_terms(t0, t1, c, MAXD)
                lo, hi = min(a, b), max(a, b)
                if hi >= 0 or lo < -21:
                    continue
                uw = max(1, min((1 << 32) - 1, int(math.exp(rng.uniform(lo, hi)) * 4294967296.0)))
                target = _log(uw / 4294967296.0)
            d0 = _d_crossing(t0, t1, c, target)
            if d0 is None:
                continue
            r = _exact_ratio(t0, t1, c, d0) if kind == "cancel" else 0.0
            if best is None or r > best[0]:
                best = (r, c, d0, uw)
        if best is None:
            continue
        _, c, d0, uw = best
        X0s, X1s = int(t0.sum()), int(t1.sum())
        Y = int(np.abs(t0).sum() + np.abs(t1).sum())
        for d in d_ladder(d0):
            delta = oracle_ref.delta_terms(t0, t1, c, d)
            sums.append((X0s, X1s, Y, Y))
            cds.append((c, d))
            uws.append(uw)
            exp.append(oracle_ref.mh_outcome(delta, uw / 4294967296.0))
    return dict(n=len(exp), sums=np.array(sums, np.int32), cd=np.array(cds, np.float64),
                uw=np.array(uws, np.uint32), expected=np.array(exp, np.int32))


def emulate_decide(cs, shift=0):
    """pc_classify + pc_resolve restated on the host (numpy f64; the f32 log's slack taken from its definition):
    0 / 1 / 2 as the oracle's outcomes, 3 = undecided (the exact delta decides).  shift: margins / 2^shift."""
    out = np.zeros(cs["n"], np.int32)
    for k in range(cs["n"]):
        X0, X1, Y0, Y1 = (int(v) for v in cs["sums"][k])
        c, d = (float(v) for v in cs["cd"][k])
        e = oracle_ref.exp_log(np.array([c, d]))[0]
        cc, dd = (float(v) for v in oracle_ref.exp_log(1.0 - e)[1])
        S = (float(X0) * cc - float(X0) * d) + (float(X1) * dd - float(X1) * c)
        aC, aD = abs(cc) + abs(d), abs(dd) + abs(c)
        B = float(Y0) * aC + float(Y1) * aD
        Knz = Y0 + Y1
        Eb = (float(Knz) + 16.0) * 2.0 ** -52 * B * 2.0 ** -shift
        u = float(cs["uw"][k]) / 4294967296.0
        lu = _log(u)
        if Knz == 0 or S > Eb:
            out[k] = 1
        elif S < -Eb and S - Eb > lu:
            out[k] = 2
        elif S < -Eb and S + Eb < lu:
            out[k] = 0
        else:
            out[k] = 3
    return out
