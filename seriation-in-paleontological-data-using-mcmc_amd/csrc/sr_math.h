/*
 * sr_math.h -- deterministic double-precision exp/log and exact "run" helpers, compiled
 * both for the host (gcc, -ffp-contract=off) and for gfx950 (hipcc, -ffp-contract=off).
 *
 * Why: the reference evaluates glibc exp()/log() inside every accept test and Gibbs
 * draw (mcmc.c:644, 734, 757-760, 847-848, 1214, 1261, 1441, 1636).  A GPU cannot call
 * glibc, and OCML's exp/log differ from it in the last bit, which would flip
 * data-dependent RNG consumption (mcmc.c:1261 draws uniform_pos only when delta < 0).
 * So the sampler restates glibc's own algorithm (the x86-64 FMA build of e_exp.c / e_log.c,
 * built only from correctly rounded IEEE operations and explicit fma); host, device and
 * this machine's libm.so.6 produce bitwise-identical results (tests/test_host.py,
 * tests/test_gpu_parity.py).
 *
 * sr_run_add / sr_run_sub reproduce L sequential roundings x = fl(x + e) / r = fl(r - p)
 * in O(binades) instead of O(L) steps: inside one binade every step moves x by the same
 * representable increment RN(e/ulp)*ulp (ties handled step-by-step).  They let the
 * device skip the long runs of clamped exp(LOGEPSILON) terms in mcmc_logtop /
 * mcmc_randompick (mcmc.c:731-737, 909-913) while producing the exact sequential result.
 */
#ifndef SR_MATH_H
#define SR_MATH_H
#include <stdint.h>
#include "sr_tables.h"

#ifdef __HIPCC__
#define SR_HD __host__ __device__ __forceinline__
#else
#define SR_HD static inline
#endif

#if defined(__cplusplus)
SR_HD uint64_t sr_bits(double x) { return __builtin_bit_cast(uint64_t, x); }
SR_HD double sr_from_bits(uint64_t u) { return __builtin_bit_cast(double, u); }
#else
SR_HD uint64_t sr_bits(double x) { union { double d; uint64_t u; } v; v.d = x; return v.u; }
SR_HD double sr_from_bits(uint64_t u) { union { double d; uint64_t u; } v; v.u = u; return v.d; }
#endif

#define SR_LOGEPSILON (-32.236191301916641) /* mcmc.h:26 */
#define SR_MINC (-6.9077552789821368)       /* mcmc.h:27 */
#define SR_MAXC (-2.3025850929940455)       /* mcmc.h:28 */
#define SR_MIND (-1.6094379124341003)       /* mcmc.h:29 */
#define SR_MAXD (-0.22314355131420971)      /* mcmc.h:30 */

/* Table pointers: the device passes LDS copies, the host the static tables. */
typedef struct {
  const uint64_t *exp_tab;   /* glibc __exp_data.tab[256] */
  const double *log_tab;     /* glibc __log_data.tab[128] {invc, logc} */
} sr_mtab;

/* glibc exp (sysdeps/ieee754/dbl-64/e_exp.c), x86-64 FMA ifunc build: the fma() calls are that
 * build's contractions; bit-identical to libm.so.6 (tests/test_host.py, tests/test_gpu_parity.py) */
SR_HD double sr_exp_m(double x, const sr_mtab *t)
{
  uint32_t abstop = (uint32_t)(sr_bits(x) >> 52) & 0x7ff;
  if (abstop - 0x3c9u >= 0x408u - 0x3c9u) {          /* |x| < 2^-54 or |x| >= 512 */
    if ((int32_t)(abstop - 0x3c9u) < 0) return 1.0 + x;
    if (abstop >= 0x409u) {
      if (sr_bits(x) == 0xFFF0000000000000ULL) return 0.0;
      if (abstop >= 0x7ffu) return 1.0 + x;
      return (sr_bits(x) >> 63) ? 0.0 : __builtin_inf();
    }
    abstop = 0;
  }
  double kd = __builtin_fma(x, SR_GEXP_INVLN2N, SR_GEXP_SHIFT);
  const uint64_t ki = sr_bits(kd);
  kd -= SR_GEXP_SHIFT;
  double r = __builtin_fma(kd, SR_GEXP_NEGLN2HIN, x);
  r = __builtin_fma(kd, SR_GEXP_NEGLN2LON, r);
  const uint64_t idx = 2 * (ki % 128), top = ki << 45;
  const double tail = sr_from_bits(t->exp_tab[idx]);
  uint64_t sbits = t->exp_tab[idx + 1] + top;
  const double r2 = r * r;
  const double p1 = __builtin_fma(r, SR_GEXP_C3, SR_GEXP_C2);
  const double p2 = __builtin_fma(r, SR_GEXP_C5, SR_GEXP_C4);
  double tmp = __builtin_fma(r2, p1, tail + r);
  tmp = __builtin_fma(r2 * r2, p2, tmp);
  if (abstop == 0) {                                  /* specialcase(): |x| >= 512 */
    if ((ki & 0x80000000u) == 0) {
      sbits -= 1009ull << 52;
      const double scale = sr_from_bits(sbits);
      return 0x1p1009 * __builtin_fma(scale, tmp, scale);
    }
    sbits += 1022ull << 52;                           /* k < 0: not contracted in glibc's build */
    const double scale = sr_from_bits(sbits);
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
  const double scale = sr_from_bits(sbits);
  return __builtin_fma(scale, tmp, scale);
}

/* glibc log (sysdeps/ieee754/dbl-64/e_log.c), x86-64 FMA ifunc build */
SR_HD double sr_log_m(double x, const sr_mtab *t)
{
  uint64_t ix = sr_bits(x);
  const uint32_t top = (uint32_t)(ix >> 48);
  if (ix - 0x3FEE000000000000ULL < 0x3FF1090000000000ULL - 0x3FEE000000000000ULL) {   /* near 1 */
    if (ix == 0x3FF0000000000000ULL) return 0.0;
    const double r = x - 1.0, r2 = r * r, r3 = r * r2;
    double p = __builtin_fma(r, SR_GLOG_B8, SR_GLOG_B7);
    p = __builtin_fma(r2, SR_GLOG_B9, p);
    p = __builtin_fma(r3, SR_GLOG_B10, p);
    double q = __builtin_fma(r, SR_GLOG_B5, SR_GLOG_B4);
    q = __builtin_fma(r2, SR_GLOG_B6, q);
    q = __builtin_fma(p, r3, q);
    double s = __builtin_fma(r, SR_GLOG_B2, SR_GLOG_B1);
    s = __builtin_fma(r2, SR_GLOG_B3, s);
    const double P = __builtin_fma(q, r3, s);
    const double rhi = __builtin_fma(-0x1p27, r, __builtin_fma(r, 0x1p27, r));
    const double rlo = r - rhi;
    const double rr = rhi * rhi;
    const double hi = __builtin_fma(rr, SR_GLOG_B0, r);
    double lo = __builtin_fma(rr, SR_GLOG_B0, r - hi);
    lo = __builtin_fma(SR_GLOG_B0 * rlo, rhi + r, lo);
    const double y = __builtin_fma(P, r3, lo);
    return y + hi;
  }
  if (top - 0x0010u >= 0x7ff0u - 0x0010u) {
    if (ix * 2 == 0) return -__builtin_inf();
    if (ix == 0x7FF0000000000000ULL) return x;
    if ((top & 0x8000u) || (top & 0x7ff0u) == 0x7ff0u) return (x - x) / (x - x);
    ix = sr_bits(x * 0x1p52);
    ix -= 52ULL << 52;
  }
  const uint64_t tmp = ix - 0x3FE6000000000000ULL;
  const int i = (int)((tmp >> 45) % 128);
  const int64_t k = (int64_t)tmp >> 52;
  const uint64_t iz = ix - (tmp & (0xFFFULL << 52));
  const double invc = t->log_tab[2 * i], logc = t->log_tab[2 * i + 1];
  const double z = sr_from_bits(iz);
  const double r = __builtin_fma(z, invc, -1.0);
  const double kd = (double)k;
  const double w = __builtin_fma(kd, SR_GLOG_LN2HI, logc);
  const double hi = w + r;
  const double lo = __builtin_fma(kd, SR_GLOG_LN2LO, w - hi + r);
  const double r2 = r * r;
  const double q = __builtin_fma(r2, __builtin_fma(r, SR_GLOG_A4, SR_GLOG_A3), __builtin_fma(r, SR_GLOG_A2, SR_GLOG_A1));
  return __builtin_fma(r * r2, q, __builtin_fma(r2, SR_GLOG_A0, lo)) + hi;
}

/* ulp of a positive normal double */
SR_HD double sr_ulp(double x) { return sr_from_bits((sr_bits(x) & 0x7FF0000000000000ULL) - (52ULL << 52)); }

/* Result of L sequential steps x = fl(x + e); x >= 0, e > 0 (finite, normal range). */
SR_HD double sr_run_add(double x, double e, long L)
{
  while (L > 0) {
    x = x + e;
    L--;
    if (L == 0) break;
    double u = sr_ulp(x);
    double q = e / u; /* exact: u is a power of two */
    double fq = __builtin_floor(q);
    if (q - fq == 0.5) { /* tie: rounding depends on parity, step explicitly */
      x = x + e;
      L--;
      continue;
    }
    double S = __builtin_rint(q);
    if (S == 0.0) return x;                   /* e no longer moves x */
    int64_t X = (int64_t)(x / u);
    int64_t Si = (int64_t)S;
    int64_t T = ((1LL << 53) - 2 - X) / Si;
    if (T <= 0) continue;
    if (T > L) T = L;
    x = (double)(X + T * Si) * u;
    L -= T;
  }
  return x;
}

/* Up to L sequential steps r = fl(r - p) (r > 0, p > 0), stopping after the first step
 * whose result is <= 0.  Returns the steps taken (== L when no crossing); *rr = final r. */
SR_HD long sr_run_sub(double *rr, double p, long L)
{
  double r = *rr;
  long steps = 0;
  while (steps < L) {
    r = r - p;
    steps++;
    if (r <= 0.0) break;
    if (steps == L) break;
    double u = sr_ulp(r);
    double q = p / u;
    double fq = __builtin_floor(q);
    if (q - fq == 0.5) continue;
    double S = __builtin_rint(q);
    if (S == 0.0) { steps = L; break; }       /* p no longer moves r: never crosses */
    int64_t X = (int64_t)(r / u);
    int64_t Si = (int64_t)S;
    int64_t T = (X - (1LL << 52) - 1) / Si;
    if (T <= 0) continue;
    if (T > L - steps) T = L - steps;
    r = (double)(X - T * Si) * u;
    steps += T;
  }
  *rr = r;
  return steps;
}

#endif
