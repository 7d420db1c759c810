#!/usr/bin/env python3
"""Generate the constant tables shared (by value) between the CPU oracle and the HIP sampler.

Two headers are written from the same numbers, one per consumer, so the oracle never
includes product code and the product never includes oracle code:

  oracle/om_tables.h                                            (prefix om_)
  seriation-in-paleontological-data-using-mcmc_amd/csrc/sr_tables.h  (prefix sr_)

Contents
--------
1. GSL 2.6 ``gsl_ran_gaussian_ziggurat`` tables (randist/gausszig.c).  GSL is a
   third-party dependency of the reference (``mcmc.c:43`` includes gsl_randist.h;
   the shipped binary links libgsl.so.25 = GSL 2.6) and is not under
   /root/reference, so the tables are regenerated from their construction:
   128 equal-area strips of f(x)=exp(-x^2/2), base strip = [0,R] rectangle plus an
   exponential wedge exp(-R(x-R/2)) of area f(R)/R, with R the exact root that
   makes ytab[0] == 1 (GSL prints it rounded as 3.44428647676).  ytab/wtab are
   rounded to 12 significant digits, ktab = floor(2^24 x_i/x_{i+1}).  Pinned: this
   reproduces the published GSL values ytab[0..15], ktab[0..15], wtab[0..7]
   (asserted below); the remaining entries follow from the same construction.

2. glibc's exp/log tables (the reference calls glibc exp()/log(); its binary imports
   exp@GLIBC_2.29): __exp_data.tab is computed from its definition and cross-checked
   against this machine's libm.so.6; __log_data.tab {invc, logc} comes out of a search
   procedure with no closed form, so it is read from libm.so.6 (Ubuntu glibc 2.35), located
   by the struct's leading constants.  oracle/om_libm.h and csrc/sr_math.h restate the
   x86-64 FMA ifunc variant of glibc's exp/log on these tables; tests/test_host.py checks
   both equal glibc bit for bit.
"""
import os
import sys
from mpmath import mp, mpf, exp, log, sqrt, findroot, floor

mp.dps = 60
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "seriation-in-paleontological-data-using-mcmc_amd")


def zig_tables():
    f = lambda x: exp(-x * x / 2)

    def build(R):
        V = R * f(R) + f(R) / R
        x = [None] * 129
        y = [None] * 128
        x[127] = R
        y[127] = f(R)
        for i in range(126, -1, -1):
            y[i] = y[i + 1] + V / x[i + 1]
            x[i] = sqrt(-2 * log(y[i])) if y[i] < 1 else mpf(0)
        x[128] = V / f(R)
        return x, y

    R = findroot(lambda r: build(r)[1][0] - 1, mpf("3.44428647676"))
    x, y = build(R)
    y[0] = mpf(1)
    x[0] = mpf(0)
    ktab = [int(floor(mpf(2) ** 24 * x[i] / x[i + 1])) for i in range(127)]
    ktab.append(int(floor(mpf(2) ** 24 * R / x[128])))
    wtab = [x[i + 1] * mpf(2) ** -24 for i in range(128)]
    return y, ktab, wtab


def sig12(v):
    if v == 0:
        return "0"
    s = mp.nstr(v, 12, min_fixed=0, max_fixed=0)  # scientific, 12 significant digits
    return s


# values recalled from the published GSL 2.6 gausszig.c (pins for the regeneration)
PIN_Y = ["1", "0.963598623011", "0.936280813353", "0.913041104253", "0.892278506696",
         "0.873239356919", "0.855496407634", "0.838778928349", "0.822902083699",
         "0.807732738234", "0.793171045519", "0.779139726505", "0.765577436082",
         "0.752434456248", "0.739669787677", "0.727249120285"]
PIN_K = [0, 12590644, 14272653, 14988939, 15384584, 15635009, 15807561, 15933577,
         16029594, 16105155, 16166147, 16216399, 16258508, 16294295, 16325078, 16351831]
PIN_W = ["1.62318314817e-08", "2.16291505214e-08", "2.54246305087e-08", "2.84579525938e-08",
         "3.10340022482e-08", "3.33011726243e-08", "3.53439060345e-08", "3.72152672658e-08"]


def hexd(v):
    return float(v).hex()


def dd(v):
    hi = float(v)
    lo = float(v - mpf(hi))
    return hi, lo


GLIBC_LIBM = "/lib/x86_64-linux-gnu/libm.so.6"

# glibc >= 2.28 exp/log (the ARM optimized-routines code; the reference binary imports
# exp@GLIBC_2.29 / log@GLIBC_2.29): sysdeps/ieee754/dbl-64/e_exp.c, e_log.c with
# EXP_TABLE_BITS = LOG_TABLE_BITS = 7, EXP_POLY_ORDER = 5, LOG_POLY_ORDER = 6,
# LOG_POLY1_ORDER = 12.  Scalar constants (published in e_exp_data.c / e_log_data.c):
EXP_CONST = dict(invln2N="0x1.71547652b82fep7", shift="0x1.8p52", negln2hiN="-0x1.62e42fefa0000p-8",
                 negln2loN="-0x1.cf79abc9e3b3ap-47", C2="0x1.ffffffffffdbdp-2", C3="0x1.555555555543cp-3",
                 C4="0x1.55555cf172b91p-5", C5="0x1.1111167a4d017p-7")
LOG_CONST = dict(ln2hi="0x1.62e42fefa3800p-1", ln2lo="0x1.ef35793c76730p-45")
LOG_A = ["-0x1.0000000000001p-1", "0x1.555555551305bp-2", "-0x1.fffffffeb459p-3", "0x1.999b324f10111p-3",
         "-0x1.55575e506c89fp-3"]
LOG_B = ["-0x1p-1", "0x1.5555555555577p-2", "-0x1.ffffffffffdcbp-3", "0x1.999999995dd0cp-3",
         "-0x1.55555556745a7p-3", "0x1.24924a344de3p-3", "-0x1.fffffa4423d65p-4", "0x1.c7184282ad6cap-4",
         "-0x1.999eb43b068ffp-4", "0x1.78182f7afd085p-4", "-0x1.5521375d145cdp-4"]


def _u64(x):
    import struct
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def _libm_bytes():
    with open(GLIBC_LIBM, "rb") as fh:
        return fh.read()


def _find_block(data, head):
    """offset of the data block whose leading doubles are `head` (hex strings); unique or error"""
    import struct
    pat = b"".join(struct.pack("<d", float.fromhex(h)) for h in head)
    i = data.find(pat)
    if i < 0 or data.find(pat, i + 1) >= 0:
        raise SystemExit("gen_tables: cannot locate a unique %s... block in %s" % (head[0], GLIBC_LIBM))
    return i


def exp_tables():
    """__exp_data.tab: for k < 128, tab[2k] = bits of the tail (2^(k/128) - H_k) / H_k and
    tab[2k+1] = bits of H_k - (k << 45), H_k = 2^(k/128) rounded to nearest.  Computed here
    from the definition and checked against the table inside this machine's libm.so.6."""
    import struct
    mp.dps = 80
    tab = []
    for k in range(128):
        v = mpf(2) ** (mpf(k) / 128)
        H = float(v)
        tail = float((v - mpf(H)) / mpf(H))
        tab.append(_u64(tail))
        tab.append((_u64(H) - (k << 45)) & 0xFFFFFFFFFFFFFFFF)
    mp.dps = 60
    if os.path.exists(GLIBC_LIBM):
        data = _libm_bytes()
        e = _find_block(data, [EXP_CONST["invln2N"], EXP_CONST["shift"], EXP_CONST["negln2hiN"]])
        # struct exp_data: invln2N, shift, negln2hiN, negln2loN, poly[4], exp2_shift, exp2_poly[5], tab[256]
        head = struct.unpack("<8d", data[e:e + 64])
        want = [float.fromhex(EXP_CONST[k]) for k in ("invln2N", "shift", "negln2hiN", "negln2loN", "C2", "C3", "C4",
                                                       "C5")]
        assert list(head) == want, "exp constants differ from " + GLIBC_LIBM
        got = list(struct.unpack("<256Q", data[e + 14 * 8:e + 14 * 8 + 256 * 8]))
        assert got == tab, "computed exp table differs from " + GLIBC_LIBM
    return tab


def log_tables():
    """__log_data.tab[128] = {invc, logc}: chosen by glibc's search procedure (not a closed
    form), so they are read from this machine's libm.so.6 (located by the leading constants
    ln2hi, ln2lo, A[0..4], B[0..10] of struct log_data, which are checked)."""
    import struct
    data = _libm_bytes()
    head = [LOG_CONST["ln2hi"], LOG_CONST["ln2lo"]] + LOG_A + LOG_B
    L = _find_block(data, head)
    t = list(struct.unpack("<256d", data[L + 18 * 8:L + 18 * 8 + 256 * 8]))
    for i in range(128):   # invc ~ 1/c with c inside interval i of [0x1.6p-1, 0x1.6p0)
        z0 = struct.unpack("<d", struct.pack("<Q", 0x3FE6000000000000 + (i << 45)))[0]
        assert 1 / t[2 * i] >= z0 * (1 - 2 ** -7) and 1 / t[2 * i] <= z0 * 2 ** (1 / 64) * (1 + 2 ** -7), i
        assert abs(float(log(1 / mpf(t[2 * i]))) - t[2 * i + 1]) < 2 ** -40, i
    return t


def emit(prefix, guard, path):
    y, k, w = zig_tables()
    ys = [sig12(v) for v in y]
    ys[0] = "1"
    ws = [sig12(v) for v in w]
    for i, p in enumerate(PIN_Y):
        assert float(ys[i]) == float(p), (i, ys[i], p)
    for i, p in enumerate(PIN_K):
        assert k[i] == p, (i, k[i], p)
    for i, p in enumerate(PIN_W):
        assert float(ws[i]) == float(p), (i, ws[i], p)
    etab = exp_tables()
    ltab = log_tables()
    P = prefix
    U = P.upper()
    out = []

    def arr(ctype, name, items, fmt=str):
        rows = []
        for j in range(0, len(items), 4):
            rows.append("  " + ", ".join(fmt(v) for v in items[j:j + 4]) + ("," if j + 4 < len(items) else ""))
        out.append("#define %s%s_INIT { \\\n%s }" % (U, name.upper(), " \\\n".join(rows)))
        out.append("#ifndef %sTABLES_NO_ARRAYS" % U)
        out.append("static const %s %s%s[%d] = %s%s_INIT;" % (ctype, P, name, len(items), U, name.upper()))
        out.append("#endif")

    out.append("/* GENERATED by tools/gen_tables.py -- do not edit. */")
    out.append("#ifndef %s\n#define %s" % (guard, guard))
    out.append("/* GSL 2.6 gausszig.c construction (see tools/gen_tables.py). */")
    out.append("#define %sZIG_R 3.44428647676" % U)
    arr("double", "zig_ytab", ys)
    arr("unsigned int", "zig_ktab", k, lambda v: "%du" % v)
    arr("double", "zig_wtab", ws)
    out.append("/* glibc exp (e_exp.c, N = 128): scalar constants and __exp_data.tab[2N] (tail, scale bits). */")
    for name, h in EXP_CONST.items():
        out.append("#define %sGEXP_%s %s" % (U, name.upper(), float.fromhex(h).hex()))
    arr("unsigned long long", "exp_tab", etab, lambda v: "0x%016xULL" % v)
    out.append("/* glibc log (e_log.c, N = 128): ln2 split, poly A[5] (|x-1| >= 0x1p-4 path), poly1 B[11]")
    out.append("   (near 1), __log_data.tab[N] = {invc, logc} interleaved. */")
    for name, h in LOG_CONST.items():
        out.append("#define %sGLOG_%s %s" % (U, name.upper(), float.fromhex(h).hex()))
    for i, h in enumerate(LOG_A):
        out.append("#define %sGLOG_A%d %s" % (U, i, float.fromhex(h).hex()))
    for i, h in enumerate(LOG_B):
        out.append("#define %sGLOG_B%d %s" % (U, i, float.fromhex(h).hex()))
    arr("double", "log_tab", ltab, hexd)
    out.append("#endif")
    with open(path, "w") as fh:
        fh.write("\n".join(out) + "\n")


if __name__ == "__main__":
    emit("om_", "OM_TABLES_H", os.path.join(ROOT, "oracle", "om_tables.h"))
    emit("sr_", "SR_TABLES_H", os.path.join(PKG, "csrc", "sr_tables.h"))
    print("tables written")
