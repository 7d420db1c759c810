/*
 * oracle/om_libm.h -- TEST INFRASTRUCTURE ONLY (the CPU oracle).  Never linked into the product.
 *
 * glibc's exp()/log(), restated.  The reference calls them in every Gibbs draw and accept
 * test (mcmc.c:644, 734, 757-760, 847-848, 1214, 1261, 1441, 1636; the shipped binary imports
 * exp@GLIBC_2.29 / log@GLIBC_2.29, i.e. the table-driven code glibc took from ARM's
 * optimized-routines in 2.28: sysdeps/ieee754/dbl-64/e_exp.c, e_log.c).  On x86-64 glibc
 * dispatches to the build of that code compiled with -mfma -mavx2 (ifunc "fma" variant,
 * chosen on every CPU with FMA and AVX2), in which gcc contracted a*b+c into fused
 * multiply-adds; the fma() calls below are exactly the contractions of that build (read off
 * its machine code: tools/README.md), and tests/test_host.py checks these functions equal
 * this machine's libm.so.6 bit for bit on >= 10^7 inputs.  The device restatement is
 * csrc/sr_math.h (same operation sequence).
 *
 * Tables: om_tables.h (tools/gen_tables.py).  Compile with -ffp-contract=off: the only
 * fused operations are the explicit ones.
 */
#ifndef OM_LIBM_H
#define OM_LIBM_H
#include <stdint.h>
#include <string.h>
#include <math.h>
#include "om_tables.h"

static inline uint64_t om_bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static inline double om_from_bits(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }

/* e_exp.c: exp(x) = 2^(k/128) * exp(r), r in [-ln2/256, ln2/256] */
static inline double om_exp(double x)
{
  uint32_t abstop = (uint32_t)(om_bits(x) >> 52) & 0x7ff;
  if (abstop - 0x3c9u >= 0x408u - 0x3c9u) {          /* |x| < 2^-54 or |x| >= 512 */
    if ((int32_t)(abstop - 0x3c9u) < 0) return 1.0 + x;
    if (abstop >= 0x409u) {                           /* |x| >= 1024 */
      if (om_bits(x) == om_bits(-INFINITY)) return 0.0;
      if (abstop >= 0x7ffu) return 1.0 + x;
      return (om_bits(x) >> 63) ? 0.0 : INFINITY;
    }
    abstop = 0;                                       /* large |x|: specialcase below */
  }
  double kd = __builtin_fma(x, OM_GEXP_INVLN2N, OM_GEXP_SHIFT);
  const uint64_t ki = om_bits(kd);
  kd -= OM_GEXP_SHIFT;
  double r = __builtin_fma(kd, OM_GEXP_NEGLN2HIN, x);
  r = __builtin_fma(kd, OM_GEXP_NEGLN2LON, r);
  const uint64_t idx = 2 * (ki % 128), top = ki << 45;
  const double tail = om_from_bits(om_exp_tab[idx]);
  uint64_t sbits = om_exp_tab[idx + 1] + top;
  const double r2 = r * r;
  const double p1 = __builtin_fma(r, OM_GEXP_C3, OM_GEXP_C2);
  const double p2 = __builtin_fma(r, OM_GEXP_C5, OM_GEXP_C4);
  double tmp = __builtin_fma(r2, p1, tail + r);
  tmp = __builtin_fma(r2 * r2, p2, tmp);
  if (abstop == 0) {                                  /* specialcase() */
    if ((ki & 0x80000000u) == 0) {                    /* k > 0 */
      sbits -= 1009ull << 52;
      const double scale = om_from_bits(sbits);
      return 0x1p1009 * __builtin_fma(scale, tmp, scale);
    }
    sbits += 1022ull << 52;                           /* k < 0: this branch is not contracted */
    const double scale = om_from_bits(sbits);
    const double st = scale * tmp;
    double y = scale + st;
    if (y < 1.0) {
      double lo = scale - y + st;
      const double hi = 1.0 + y;
      lo = 1.0 - hi + y + lo;
      y = (hi + lo) - 1.0;
      if (y == 0.0) y = 0.0;
    }
    return 0x1p-1022 * y;
  }
  const double scale = om_from_bits(sbits);
  return __builtin_fma(scale, tmp, scale);
}

/* e_log.c: log(x) = k ln2 + log(c) + log1p(z/c - 1), x = 2^k z */
static inline double om_log(double x)
{
  uint64_t ix = om_bits(x);
  const uint32_t top = (uint32_t)(ix >> 48);
  if (ix - 0x3FEE000000000000ULL < 0x3FF1090000000000ULL - 0x3FEE000000000000ULL) {   /* x in [1-2^-4, 1+0x1.09p-4) */
    if (ix == 0x3FF0000000000000ULL) return 0.0;
    const double r = x - 1.0, r2 = r * r, r3 = r * r2;
    double p = __builtin_fma(r, OM_GLOG_B8, OM_GLOG_B7);
    p = __builtin_fma(r2, OM_GLOG_B9, p);
    p = __builtin_fma(r3, OM_GLOG_B10, p);
    double q = __builtin_fma(r, OM_GLOG_B5, OM_GLOG_B4);
    q = __builtin_fma(r2, OM_GLOG_B6, q);
    q = __builtin_fma(p, r3, q);
    double s = __builtin_fma(r, OM_GLOG_B2, OM_GLOG_B1);
    s = __builtin_fma(r2, OM_GLOG_B3, s);
    const double P = __builtin_fma(q, r3, s);
    const double rhi = __builtin_fma(-0x1p27, r, __builtin_fma(r, 0x1p27, r));
    const double rlo = r - rhi;
    const double rr = rhi * rhi;
    const double hi = __builtin_fma(rr, OM_GLOG_B0, r);
    double lo = __builtin_fma(rr, OM_GLOG_B0, r - hi);
    lo = __builtin_fma(OM_GLOG_B0 * rlo, rhi + r, lo);
    const double y = __builtin_fma(P, r3, lo);
    return y + hi;
  }
  if (top - 0x0010u >= 0x7ff0u - 0x0010u) {
    if (ix * 2 == 0) return -INFINITY;
    if (ix == 0x7FF0000000000000ULL) return x;
    if ((top & 0x8000u) || (top & 0x7ff0u) == 0x7ff0u) return (x - x) / (x - x);
    ix = om_bits(x * 0x1p52);                         /* subnormal: normalise */
    ix -= 52ULL << 52;
  }
  const uint64_t tmp = ix - 0x3FE6000000000000ULL;
  const int i = (int)((tmp >> 45) % 128);
  const int64_t k = (int64_t)tmp >> 52;
  const uint64_t iz = ix - (tmp & (0xFFFULL << 52));
  const double invc = om_log_tab[2 * i], logc = om_log_tab[2 * i + 1];
  const double z = om_from_bits(iz);
  const double r = __builtin_fma(z, invc, -1.0);
  const double kd = (double)k;
  const double w = __builtin_fma(kd, OM_GLOG_LN2HI, logc);
  const double hi = w + r;
  const double lo = __builtin_fma(kd, OM_GLOG_LN2LO, w - hi + r);
  const double r2 = r * r;
  const double q = __builtin_fma(r2, __builtin_fma(r, OM_GLOG_A4, OM_GLOG_A3), __builtin_fma(r, OM_GLOG_A2, OM_GLOG_A1));
  return __builtin_fma(r * r2, q, __builtin_fma(r2, OM_GLOG_A0, lo)) + hi;
}

#endif
