/*
 * sr_math.h -- deterministic double-precision exp/log and exact "run" helpers, compiled
 * both for the host (gcc, -ffp-contract=off) and for gfx950 (hipcc, -ffp-contract=off).
 *
 * Why: the reference evaluates glibc exp()/log() inside every accept test and Gibbs
 * draw (mcmc.c:644, 734, 757-760, 847-848, 1214, 1261, 1441, 1636).  A GPU cannot call
 * glibc, and OCML's exp/log differ from it in the last bit, which would flip
 * data-dependent RNG consumption (mcmc.c:1261 draws uniform_pos only when delta < 0).
 * So the sampler uses one table-driven algorithm (~0.51 ulp; agrees with glibc on
 * >99.8% of inputs) built only from correctly rounded IEEE operations; host and
 * device produce bitwise-identical results (tests/test_math.py, tests/test_gpu_parity.py).
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
  const double *exp_thi, *exp_tlo, *log_invc, *log_lhi, *log_llo;
} sr_mtab;

SR_HD double sr_exp_t(double x, const double *thi_t, const double *tlo_t)
{
  if (x != x) return x;
  if (x > 709.782712893384) return __builtin_inf();
  if (x < -745.1332191019412) return 0.0;
  double kd = __builtin_rint(x * SR_EXP_INVL);
  int k = (int)kd;
  double r = __builtin_fma(-kd, SR_EXP_L1, x);
  r = __builtin_fma(-kd, SR_EXP_L2, r);
  int idx = k & 127;
  int e = (k - idx) / 128;
  double r2 = r * r;
  double h = __builtin_fma(r, 1.0 / 720.0, 1.0 / 120.0);
  h = __builtin_fma(r, h, 1.0 / 24.0);
  h = __builtin_fma(r, h, 1.0 / 6.0);
  h = __builtin_fma(r, h, 0.5);
  double p = __builtin_fma(r2, h, r);
  double thi = thi_t[idx];
  double tmp = __builtin_fma(thi, p, tlo_t[idx]);
  double res = thi + tmp;
  if (e > 1000) return (res * sr_from_bits((uint64_t)(e - 1 + 1023) << 52)) * 2.0;
  if (e >= -1022) return res * sr_from_bits((uint64_t)(e + 1023) << 52);
  return (res * sr_from_bits((uint64_t)(e + 600 + 1023) << 52)) * 0x1p-600;
}

SR_HD double sr_log_t(double x, const double *invc_t, const double *lhi_t, const double *llo_t)
{
  if (x != x) return x;
  if (x <= 0.0) return x == 0.0 ? -__builtin_inf() : (x - x) / (x - x);
  if (x == __builtin_inf()) return x;
  if (x > 0.96875 && x < 1.03125) {
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
  uint64_t ix = sr_bits(x);
  int64_t kadj = 0;
  if (ix < 0x0010000000000000ULL) {
    ix = sr_bits(x * 0x1p52);
    kadj = -52;
  }
  uint64_t tmp = ix - SR_LOG_OFF;
  int i = (int)((tmp >> 45) & 127);
  int64_t k = ((int64_t)tmp >> 52) + kadj;
  uint64_t iz = ix - (tmp & (0xFFFULL << 52));
  double z = sr_from_bits(iz);
  double r = __builtin_fma(z, invc_t[i], -1.0);
  double kd = (double)k;
  double w1 = kd * SR_LOG_LN2HI;
  double lhi = lhi_t[i];
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
  lo = __builtin_fma(kd, SR_LOG_LN2LO, lo);
  lo = lo + llo_t[i];
  lo = __builtin_fma(r2, P, lo);
  return hi + lo;
}

SR_HD double sr_exp_m(double x, const sr_mtab *t) { return sr_exp_t(x, t->exp_thi, t->exp_tlo); }
SR_HD double sr_log_m(double x, const sr_mtab *t) { return sr_log_t(x, t->log_invc, t->log_lhi, t->log_llo); }

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
