/*
 * oracle/om_libm.h -- TEST INFRASTRUCTURE ONLY (the CPU oracle).  Never linked into the product.
 *
 * Deterministic exp/log for the oracle.  The reference calls glibc exp()/log()
 * (mcmc.c:644, 734, 760, 847-848, 1214, 1261, ...; the shipped binary imports
 * exp@GLIBC_2.29).  glibc's results depend on the host's FMA ifunc variant and are
 * not reproducible on a GPU, so the oracle and the HIP sampler both use this
 * algorithm (table-driven, ~0.51 ulp, built only from IEEE +,-,*,/,fma,rint and bit
 * operations).  Any IEEE-754 machine executing these operations in this order gets
 * bitwise-identical results; the device copy lives in the product's csrc/sr_math.h
 * and tests/test_math.py checks the two agree bit-for-bit.
 *
 * Compile with -ffp-contract=off (no implicit FMA contraction, as in the
 * reference binary, which contains no vfmadd).
 */
#ifndef OM_LIBM_H
#define OM_LIBM_H
#include <stdint.h>
#include <string.h>
#include <math.h>
#include "om_tables.h"

static inline uint64_t om_bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static inline double om_from_bits(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }

static inline double om_exp(double x)
{
  if (x != x) return x;
  if (x > 709.782712893384) return HUGE_VAL;
  if (x < -745.1332191019412) return 0.0;
  double kd = __builtin_rint(x * OM_EXP_INVL);
  int k = (int)kd;
  double r = __builtin_fma(-kd, OM_EXP_L1, x);
  r = __builtin_fma(-kd, OM_EXP_L2, r);
  int idx = k & 127;
  int e = (k - idx) / 128;
  double r2 = r * r;
  double h = __builtin_fma(r, 1.0 / 720.0, 1.0 / 120.0);
  h = __builtin_fma(r, h, 1.0 / 24.0);
  h = __builtin_fma(r, h, 1.0 / 6.0);
  h = __builtin_fma(r, h, 0.5);
  double p = __builtin_fma(r2, h, r);
  double thi = om_exp_thi[idx];
  double tmp = __builtin_fma(thi, p, om_exp_tlo[idx]);
  double res = thi + tmp;
  if (e > 1000)
    return (res * om_from_bits((uint64_t)(e - 1 + 1023) << 52)) * 2.0;
  if (e >= -1022)
    return res * om_from_bits((uint64_t)(e + 1023) << 52);
  return (res * om_from_bits((uint64_t)(e + 600 + 1023) << 52)) * 0x1p-600;
}

static inline double om_log(double x)
{
  if (x != x) return x;
  if (x <= 0.0) return x == 0.0 ? -HUGE_VAL : (x - x) / (x - x);
  if (x == HUGE_VAL) return x;
  if (x > 0.96875 && x < 1.03125) {
    /* log1p series on r = x - 1 (exact by Sterbenz), |r| < 2^-5 */
    double r = x - 1.0;
    double P = __builtin_fma(r, -1.0 / 14.0, 1.0 / 13.0);
    P = __builtin_fma(r, P, -1.0 / 12.0);
    P = __builtin_fma(r, P, 1.0 / 11.0);
    P = __builtin_fma(r, P, -1.0 / 10.0);
    P = __builtin_fma(r, P, 1.0 / 9.0);
    P = __builtin_fma(r, P, -1.0 / 8.0);
    P = __builtin_fma(r, P, 1.0 / 7.0);
    P = __builtin_fma(r, P, -1.0 / 6.0);
    P = __builtin_fma(r, P, 1.0 / 5.0);
    P = __builtin_fma(r, P, -1.0 / 4.0);
    P = __builtin_fma(r, P, 1.0 / 3.0);
    P = __builtin_fma(r, P, -0.5);
    double r2 = r * r;
    return __builtin_fma(r2, P, r);
  }
  uint64_t ix = om_bits(x);
  int64_t kadj = 0;
  if (ix < 0x0010000000000000ULL) { /* subnormal */
    ix = om_bits(x * 0x1p52);
    kadj = -52;
  }
  uint64_t tmp = ix - OM_LOG_OFF;
  int i = (int)((tmp >> 45) & 127);
  int64_t k = ((int64_t)tmp >> 52) + kadj;
  uint64_t iz = ix - (tmp & (0xFFFULL << 52));
  double z = om_from_bits(iz);
  double r = __builtin_fma(z, om_log_invc[i], -1.0);
  double kd = (double)k;
  double w1 = kd * OM_LOG_LN2HI;
  double lhi = om_log_lhi[i];
  double w = w1 + lhi;
  double bb = w - w1;
  double werr = (w1 - (w - bb)) + (lhi - bb);
  double hi = w + r;
  double b2 = hi - w;
  double e2 = (w - (hi - b2)) + (r - b2);
  double P = __builtin_fma(r, -1.0 / 8.0, 1.0 / 7.0);
  P = __builtin_fma(r, P, -1.0 / 6.0);
  P = __builtin_fma(r, P, 1.0 / 5.0);
  P = __builtin_fma(r, P, -1.0 / 4.0);
  P = __builtin_fma(r, P, 1.0 / 3.0);
  P = __builtin_fma(r, P, -0.5);
  double r2 = r * r;
  double lo = werr + e2;
  lo = __builtin_fma(kd, OM_LOG_LN2LO, lo);
  lo = lo + om_log_llo[i];
  lo = __builtin_fma(r2, P, lo);
  return hi + lo;
}

#endif
