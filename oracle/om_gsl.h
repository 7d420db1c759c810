/*
 * oracle/om_gsl.h -- TEST INFRASTRUCTURE ONLY (CPU oracle).  Never linked into the product.
 *
 * Restatement of the parts of the GNU Scientific Library 2.6 that the reference
 * sampler calls (GSL is an external dependency of /root/reference, not vendored:
 * `readelf -d mcmc` -> libgsl.so.25 = GSL 2.6).  Published algorithms restated:
 *
 *   rng/mt.c            mt19937: Knuth seeding (s==0 -> 4357), 624-word twist, tempering
 *   gsl_rng.h           gsl_rng_uniform      = get()/2^32
 *                       gsl_rng_uniform_pos  = uniform() until != 0
 *                       gsl_rng_uniform_int  = get()/(0xffffffff/n), reject >= n
 *   randist/shuffle.c   gsl_ran_shuffle      (i = n-1..1, swap(i, uniform_int(i+1)))
 *                       gsl_ran_choose       (take src[i] iff (n-i)*uniform() < k-j)
 *   randist/gausszig.c  gsl_ran_gaussian_ziggurat (128 strips, R = 3.44428647676)
 *   randist/gamma.c     gsl_ran_gamma        (Marsaglia-Tsang; a<1 boost branch)
 *   randist/beta.c      gsl_ran_beta         = X/(X+Y), X~Gamma(a), Y~Gamma(b)
 *
 * Reference call sites: mcmc.c:489, 519, 548 (init), 591-592 (setup), 757 (beta),
 * 909 (randompick), 1140-1141, 1261, 1325-1326, 1340, 1360-1361, 1441, 1505-1506,
 * 1561-1562, 1636 (proposals).
 *
 * Parity status: mt19937 / uniform / uniform_int / shuffle / choose are pinned by
 * tests against numpy.random.RandomState (same init_genrand recurrence).  The gamma /
 * ziggurat stream is pinned only through the regenerated tables (tools/gen_tables.py
 * reproduces the published ytab/ktab/wtab head values); GSL itself is absent here.
 * libm exp/log are replaced by om_exp/om_log (om_libm.h).
 */
#ifndef OM_GSL_H
#define OM_GSL_H
#include <stdint.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include "om_libm.h"

#define OM_MT_N 624
#define OM_MT_M 397

typedef struct {
  uint32_t mt[OM_MT_N];
  int mti;
  uint64_t ndraw; /* words drawn so far (diagnostic) */
  /* opt-in Philox mode (the product's SR_F_RNG_PHILOX; not the reference's generator):
     word w = Philox4x32-10(key, counter w / 4)[w % 4] */
  int philox;
  uint32_t pkey[2], pbuf[4];
  uint64_t pw;
} om_rng;

/* Philox4x32-10, restated from its publication (Salmon et al., "Parallel random numbers: as
   easy as 1, 2, 3", SC'11; Random123 philox.h): 10 rounds of two 32x32->64 multiplies by
   0xD2511F53 / 0xCD9E8D57 with the Weyl key schedule 0x9E3779B9 / 0xBB67AE85. */
static inline void om_philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1)
{
  for (int round = 0; round < 10; round++) {
    if (round) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t a = (uint64_t)0xD2511F53u * c[0], b = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(b >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(a >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)b;
    c[3] = (uint32_t)a;
    c[0] = n0;
    c[2] = n2;
  }
}

/* switch a generator to the Philox stream of `seed` (0 -> 4357), word 0 next */
static inline void om_rng_philox(om_rng *r, unsigned long seed)
{
  uint64_t s = seed ? (uint64_t)seed : 4357u;
  r->philox = 1;
  r->pkey[0] = (uint32_t)s;
  r->pkey[1] = (uint32_t)(s >> 32) ^ 0xA511E9B3u;
  r->pw = 0;
}

static inline void om_rng_seed(om_rng *r, unsigned long s)
{
  if (s == 0) s = 4357;
  r->mt[0] = (uint32_t)(s & 0xffffffffUL);
  for (int i = 1; i < OM_MT_N; i++) {
    uint32_t p = r->mt[i - 1];
    r->mt[i] = (uint32_t)(1812433253UL * (p ^ (p >> 30)) + (unsigned long)i);
  }
  r->mti = OM_MT_N;
  r->ndraw = 0;
  r->philox = 0;
}

/* gsl_rng_env_setup (GSL 2.6 rng/env.c; called by mcmc_init, mcmc.c:591-592): GSL_RNG_TYPE names the
   generator among gsl_rng_types_setup's list (rng/types.c order), "GSL_RNG_TYPE=<name>" on stderr when set;
   GSL_RNG_SEED (strtoul base 0) and "GSL_RNG_SEED=<value>" after it.  Returns 0 for mt19937 (unset or named),
   1 for another GSL generator (GSL would run it; the oracle has only mt19937 and refuses, as the product does),
   2 for a name GSL does not know (GSL prints the list and aborts through gsl_error; here: the list, then 2). */
static const char *const om_gsl_rng_names[] = {
    "borosh13", "cmrg", "coveyou", "fishman18", "fishman20", "fishman2x", "gfsr4", "knuthran", "knuthran2",
    "knuthran2002", "lecuyer21", "minstd", "mrg", "mt19937", "mt19937_1999", "mt19937_1998", "r250", "ran0", "ran1",
    "ran2", "ran3", "rand", "rand48", "random128-bsd", "random128-glibc2", "random128-libc5", "random256-bsd",
    "random256-glibc2", "random256-libc5", "random32-bsd", "random32-glibc2", "random32-libc5", "random64-bsd",
    "random64-glibc2", "random64-libc5", "random8-bsd", "random8-glibc2", "random8-libc5", "random-bsd",
    "random-glibc2", "random-libc5", "randu", "ranf", "ranlux", "ranlux389", "ranlxd1", "ranlxd2", "ranlxs0",
    "ranlxs1", "ranlxs2", "ranmar", "slatec", "taus", "taus2", "taus113", "transputer", "tt800", "uni", "uni32",
    "vax", "waterman14", "zuf", 0};

static inline int om_rng_env_setup(unsigned long *seed)
{
  const char *p = getenv("GSL_RNG_TYPE");
  *seed = 0;
  if (p) {
    int known = 0;
    for (int k = 0; om_gsl_rng_names[k]; k++) known |= strcmp(p, om_gsl_rng_names[k]) == 0;
    if (!known) {
      fprintf(stderr, "GSL_RNG_TYPE=%s not recognized\n", p);
      fprintf(stderr, "Valid generator types are:\n");
      for (int k = 0; om_gsl_rng_names[k]; k++) {
        fprintf(stderr, " %18s", om_gsl_rng_names[k]);
        if ((k + 1) % 4 == 0) fputc('\n', stderr);
      }
      fputc('\n', stderr);
      /* Departure (parity unpinned): GSL 2.6 follows the list with GSL_ERROR_VOID("unknown generator"), whose
         default handler prints its own "gsl: env.c:<line>: ERROR: unknown generator" line and abort()s; the
         oracle and the product both return exit status 1 here (no GSL to take the handler's exact text from) */
      return 2;
    }
    if (strcmp(p, "mt19937") != 0) {
      fprintf(stderr, "GSL_RNG_TYPE=%s: generator not available, only mt19937 (GSL's default) is implemented\n", p);
      return 1;
    }
    fprintf(stderr, "GSL_RNG_TYPE=%s\n", p);
  }
  const char *s = getenv("GSL_RNG_SEED");
  if (s) { *seed = strtoul(s, 0, 0); fprintf(stderr, "GSL_RNG_SEED=%lu\n", *seed); }
  return 0;
}

static inline uint32_t om_rng_get(om_rng *r)
{
  if (r->philox) {
    if ((r->pw & 3) == 0) {
      const uint64_t ctr = r->pw >> 2;
      r->pbuf[0] = (uint32_t)ctr; r->pbuf[1] = (uint32_t)(ctr >> 32); r->pbuf[2] = 0; r->pbuf[3] = 0;
      om_philox4x32_10(r->pbuf, r->pkey[0], r->pkey[1]);
    }
    r->ndraw++;
    return r->pbuf[r->pw++ & 3];
  }
  uint32_t *mt = r->mt;
  if (r->mti >= OM_MT_N) {
    int kk;
    for (kk = 0; kk < OM_MT_N; kk++) {
      uint32_t y = (mt[kk] & 0x80000000u) | (mt[(kk + 1) % OM_MT_N] & 0x7fffffffu);
      uint32_t v = mt[(kk + OM_MT_M) % OM_MT_N] ^ (y >> 1);
      if (y & 1u) v ^= 0x9908b0dfu;
      mt[kk] = v;
    }
    r->mti = 0;
  }
  uint32_t k = mt[r->mti++];
  k ^= (k >> 11);
  k ^= (k << 7) & 0x9d2c5680u;
  k ^= (k << 15) & 0xefc60000u;
  k ^= (k >> 18);
  r->ndraw++;
  return k;
}

static inline double om_uniform(om_rng *r) { return om_rng_get(r) / 4294967296.0; }

static inline double om_uniform_pos(om_rng *r)
{
  double x;
  do { x = om_uniform(r); } while (x == 0);
  return x;
}

static inline unsigned long om_uniform_int(om_rng *r, unsigned long n)
{
  unsigned long scale = 0xffffffffUL / n;
  unsigned long k;
  do { k = om_rng_get(r) / scale; } while (k >= n);
  return k;
}

static inline void om_swap_bytes(void *base, size_t size, size_t i, size_t j)
{
  unsigned char *a = (unsigned char *)base + size * i, *b = (unsigned char *)base + size * j;
  for (size_t s = 0; s < size; s++) { unsigned char t = a[s]; a[s] = b[s]; b[s] = t; }
}

static inline void om_shuffle(om_rng *r, void *base, size_t n, size_t size)
{
  for (size_t i = n - 1; i > 0; i--) {
    size_t j = om_uniform_int(r, i + 1);
    om_swap_bytes(base, size, i, j);
  }
}

static inline int om_choose(om_rng *r, void *dest, size_t k, const void *src, size_t n, size_t size)
{
  size_t i, j = 0;
  if (k > n) return -1;
  for (i = 0; i < n && j < k; i++) {
    if ((double)(n - i) * om_uniform(r) < (double)(k - j)) {
      memcpy((char *)dest + size * j, (const char *)src + size * i, size);
      j++;
    }
  }
  return 0;
}

static inline double om_gaussian_ziggurat(om_rng *r, double sigma)
{
  unsigned long i, j;
  int sign;
  double x, y;
  for (;;) {
    unsigned long k = om_rng_get(r);
    i = k & 0xFF;
    j = (k >> 8) & 0xFFFFFF;
    sign = (i & 0x80) ? +1 : -1;
    i &= 0x7f;
    x = j * om_zig_wtab[i];
    if (j < om_zig_ktab[i]) break;
    if (i < 127) {
      double y0 = om_zig_ytab[i], y1 = om_zig_ytab[i + 1];
      double U1 = om_uniform(r);
      y = y1 + (y0 - y1) * U1;
    } else {
      double U1 = 1.0 - om_uniform(r);
      double U2 = om_uniform(r);
      x = OM_ZIG_R - om_log(U1) / OM_ZIG_R;
      y = om_exp(-OM_ZIG_R * (x - 0.5 * OM_ZIG_R)) * U2;
    }
    if (y < om_exp(-0.5 * x * x)) break;
  }
  return sign * sigma * x;
}

static inline double om_gamma(om_rng *r, double a, double b)
{
  if (a < 1) {
    /* GSL boost: gamma(1+a) * pow(u, 1/a).  Unreachable from the sampler (a = 1 + count). */
    double u = om_uniform_pos(r);
    return om_gamma(r, 1.0 + a, b) * om_exp(om_log(u) * (1.0 / a));
  }
  double x, v, u;
  double d = a - 1.0 / 3.0;
  double c = (1.0 / 3.0) / __builtin_sqrt(d);
  for (;;) {
    do {
      x = om_gaussian_ziggurat(r, 1.0);
      v = 1.0 + c * x;
    } while (v <= 0);
    v = v * v * v;
    u = om_uniform_pos(r);
    if (u < 1 - 0.0331 * x * x * x * x) break;
    if (om_log(u) < 0.5 * x * x + d * (1 - v + om_log(v))) break;
  }
  return b * d * v;
}

/* gsl_ran_beta (GSL 2.6 randist/beta.c, restated from its published algorithm): Johnk's method
 * when both shapes are <= 1, else the ratio of two gammas.  The sampler's shapes are 1 + count
 * (mcmc.c:757), so the Johnk branch is reached exactly when both counts are 0 (e.g. every taxon
 * spans every site: t0a = f1a = 0 for c); then a = b = 1 and pow(U, 1/1) = U exactly.  Other
 * shapes <= 1 use libm pow/log/exp (never reached by the sampler; not bit-pinned). */
static inline double om_beta(om_rng *r, double a, double b)
{
  if (a <= 1.0 && b <= 1.0) {
    for (;;) {
      const double U = om_uniform_pos(r), V = om_uniform_pos(r);
      const double X = (a == 1.0) ? U : pow(U, 1.0 / a), Y = (b == 1.0) ? V : pow(V, 1.0 / b);
      if (X + Y <= 1.0) {
        if (X + Y > 0) return X / (X + Y);
        double logX = log(U) / a, logY = log(V) / b;
        const double logM = logX > logY ? logX : logY;
        logX -= logM;
        logY -= logM;
        return exp(logX - log(exp(logX) + exp(logY)));
      }
    }
  }
  double x1 = om_gamma(r, a, 1.0);
  double x2 = om_gamma(r, b, 1.0);
  return x1 / (x1 + x2);
}

#endif
