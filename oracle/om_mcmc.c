/*
 * oracle/om_mcmc.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference sampler C_Implementation/mcmc.c (+ mcmc.h), used
 * as the parity checker for the HIP sampler and as the CPU baseline ("port") in
 * bench.py.  Nothing in the product links, loads or calls this file.
 *
 * It follows the reference's control flow, RNG consumption order and floating-point
 * expression order line by line (each function cites the lines it restates), with
 * these documented differences:
 *   - GSL 2.6 is restated in om_gsl.h (GSL is absent here); glibc exp/log are
 *     restated in om_libm.h (om_exp/om_log: bit-identical to libm.so.6, pinned by
 *     oracle_libm_mismatch in tests/test_host.py);
 *   - plain int arrays instead of gsl_vector/gsl_permutation (same values);
 *   - mcmc_randomize's read of q[nh] past the end (mcmc.c:530, UB) is guarded;
 *   - the library entry points return error codes instead of exit(1).
 * Parity with the reference binary itself is UNPINNED for the gamma/ziggurat stream
 * (GSL is not available in this container); see DESIGN.md "Oracle".
 */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
#include <time.h>
#include "om_gsl.h"

#define OM_MAXS 2000                              /* mcmc.h:25 */
#define OM_LOGEPSILON (-32.236191301916641)        /* mcmc.h:26 */
#define OM_MINC (-6.9077552789821368)              /* mcmc.h:27 */
#define OM_MAXC (-2.3025850929940455)              /* mcmc.h:28 */
#define OM_MIND (-1.6094379124341003)              /* mcmc.h:29 */
#define OM_MAXD (-0.22314355131420971)             /* mcmc.h:30 */

typedef struct {                                   /* mcmc.h:32-45 */
  int N, M;
  int *X;                  /* N*M, row = site */
  int *a, *b;
  int *pi, *rpi;           /* pi[site] = position, rpi[position] = site */
  int *h;
  double *c, *d;
  int manycd;
  double loglik;
  int *t0, *f0, *t1, *f1;
  int t0a, f0a, t1a, f1a;
  int nh;
  /* scratch */
  int *v, *dt0, *df0, *dt1, *df1, *p;
  double *q;
  om_rng rng;
  long long acc[7];        /* cc, cd, cab, cpi1, cpi20, cpi21, cpi3 (mcmc.c:220) */
} om_model;

#define X_(x, n, m) ((x)->X[(size_t)(n) * (x)->M + (m)])

/* diagnostics: how often |delta| is within the device's certification bound */
static long long om_stat[8];
static double om_stat_acc_K, om_stat_A;
static void om_note(double delta, int K, double A)
{
  om_stat[0]++;
  if (K == 0) { om_stat[1]++; return; }
  double E = (K + 64.0) * 0x1p-52 * A;
  if (delta == 0.0) om_stat[2]++;
  if (-E <= delta && delta <= E) om_stat[3]++;
  om_stat_acc_K += K; om_stat_A += A;
}

/* ---------------------------------------------------------------- parsing */

/* fgets(s, maxs, f) over an in-memory buffer; maxs <= 0 means unlimited. */
static int om_fgets(char **s, size_t *cap, int maxs, const char *text, size_t len, size_t *off)
{
  if (*off >= len) return 0;
  size_t lim = (maxs > 0) ? (size_t)(maxs - 1) : (size_t)-1;
  size_t n = 0;
  while (*off < len && n < lim) {
    char ch = text[(*off)++];
    if (n + 2 > *cap) { *cap = *cap * 2 + 64; *s = (char *)realloc(*s, *cap); }
    (*s)[n++] = ch;
    if (ch == '\n') break;
  }
  if (n + 1 > *cap) { *cap = n + 1; *s = (char *)realloc(*s, *cap); }
  (*s)[n] = '\0';
  return 1;
}

static void om_initab(om_model *x);
static void om_count01(om_model *x);
static double om_logl(const om_model *x);

static void om_free(om_model *x)
{
  free(x->X); free(x->a); free(x->b); free(x->pi); free(x->rpi); free(x->h);
  free(x->c); free(x->d); free(x->t0); free(x->f0); free(x->t1); free(x->f1);
  free(x->v); free(x->dt0); free(x->df0); free(x->dt1); free(x->df1); free(x->p); free(x->q);
  memset(x, 0, sizeof(*x));
}

/* mcmc_readmodel, mcmc.c:339-437.  Returns 0 or -1 (read error), -2 (header). */
static int om_readmodel(om_model *x, const char *text, size_t len, int maxs, int manycd)
{
  size_t off = 0, cap = 256;
  char *s = (char *)malloc(cap);
  int n, m, i, j, k;
  memset(x, 0, sizeof(*x));
  if (!om_fgets(&s, &cap, maxs, text, len, &off)) { free(s); return -1; }
  if (sscanf(s, "%d %d", &n, &m) != 2 || n <= 0 || m <= 0) { free(s); return -2; }
  x->N = n; x->M = m; x->nh = 0; x->manycd = manycd;
  x->h = (int *)calloc(n, sizeof(int));
  x->X = (int *)calloc((size_t)n * m, sizeof(int));
  for (i = 0; i < n; i++) {
    if (!om_fgets(&s, &cap, maxs, text, len, &off)) { free(s); om_free(x); return -1; }
    for (j = k = 0; j < m; j++) {
      while (s[k] != '0' && s[k] != '1' && s[k] != '\0') k++;
      if (s[k] == '0') { X_(x, i, j) = 0; k++; }
      else if (s[k] == '1') { X_(x, i, j) = 1; k++; }
    }
    while (s[k] != '*' && s[k] != '\0') k++;
    if (s[k] == '*') { x->h[i] = 1; x->nh++; }
  }
  free(s);
  x->pi = (int *)malloc(n * sizeof(int));
  x->rpi = (int *)malloc(n * sizeof(int));
  for (i = 0; i < n; i++) x->pi[i] = x->rpi[i] = i;
  x->a = (int *)malloc(m * sizeof(int));
  x->b = (int *)malloc(m * sizeof(int));
  om_initab(x);
  x->c = (double *)malloc(m * sizeof(double));
  x->d = (double *)malloc(m * sizeof(double));
  for (i = 0; i < m; i++) { x->c[i] = om_log(.01); x->d[i] = om_log(.3); }   /* mcmc.c:417-421 */
  x->t0 = (int *)malloc(m * sizeof(int)); x->f0 = (int *)malloc(m * sizeof(int));
  x->t1 = (int *)malloc(m * sizeof(int)); x->f1 = (int *)malloc(m * sizeof(int));
  x->v = (int *)malloc(n * sizeof(int)); x->p = (int *)malloc(n * sizeof(int));
  x->dt0 = (int *)malloc((n + 1) * sizeof(int)); x->df0 = (int *)malloc((n + 1) * sizeof(int));
  x->dt1 = (int *)malloc((n + 1) * sizeof(int)); x->df1 = (int *)malloc((n + 1) * sizeof(int));
  x->q = (double *)calloc(n + 1, sizeof(double));
  om_count01(x);
  x->loglik = om_logl(x);
  return 0;
}

/* mcmc_initab, mcmc.c:440-474 (its stderr line, mcmc.c:457, in the CLI build: om_diag) */
static int om_diag = 0;
static void om_initab(om_model *x)
{
  for (int m = 0; m < x->M; m++) {
    int n = 0;
    while (n < x->N && !X_(x, x->rpi[n], m)) n++;
    if (n == x->N) {
      if (om_diag) fprintf(stderr, "mcmc_initab: zero column at %d, continuing.\n", m);
      x->a[m] = 0; x->b[m] = x->N;
    } else {
      x->a[m] = n;
      n = x->N - 1;
      while (n >= 0 && !X_(x, x->rpi[n], m)) n--;
      x->b[m] = n + 1;
    }
  }
}

static void om_inverse(int *dst, const int *src, int n)
{
  for (int i = 0; i < n; i++) dst[src[i]] = i;
}

/* mcmc_randomize, mcmc.c:477-578 */
static int om_randomize(om_model *x)
{
  int i, j, k, *p, *q;
  if (x->nh == 0) {
    om_shuffle(&x->rng, x->pi, x->N, sizeof(int));
    om_inverse(x->rpi, x->pi, x->N);
    om_count01(x);
    x->loglik = om_logl(x);
    return 0;
  } else if (x->nh == x->N) {
    return 0;
  }
  p = (int *)malloc(x->N * sizeof(int));
  q = (int *)malloc(x->nh * sizeof(int));
  for (i = 0; i < x->N; i++) p[i] = i;
  om_choose(&x->rng, q, x->nh, p, x->N, sizeof(int));
  for (i = j = k = 0; i < x->N; i++) {
    if (j < x->nh && i == q[j]) j++;       /* guarded: reference reads q[nh] (mcmc.c:530) */
    else p[k++] = i;
  }
  om_shuffle(&x->rng, p, x->N - x->nh, sizeof(int));
  for (i = j = k = 0; i < x->N; i++) {
    if (x->h[i]) x->pi[i] = q[j++];
    else x->pi[i] = p[k++];
  }
  om_inverse(x->rpi, x->pi, x->N);
  free(p); free(q);
  om_initab(x);
  om_count01(x);
  x->loglik = om_logl(x);
  return 0;
}

/* mcmc_logl, mcmc.c:625-648 */
static double om_logl(const om_model *x)
{
  double loglik = 0., c, d;
  for (int m = 0; m < x->M; m++) {
    c = x->c[m];
    d = x->d[m];
    loglik += x->t0[m] * om_log(1. - om_exp(c)) + x->f0[m] * d + x->t1[m] * om_log(1. - om_exp(d)) + x->f1[m] * c;
  }
  return loglik;
}

/* mcmc_count01, mcmc.c:651-708 */
static void om_count01(om_model *x)
{
  x->t0a = x->f0a = x->t1a = x->f1a = 0;
  for (int m = 0; m < x->M; m++) {
    int t0 = 0, f0 = 0, t1 = 0, f1 = 0;
    for (int n = 0; n < x->N; n++) {
      if (x->a[m] <= x->pi[n] && x->pi[n] < x->b[m]) {
        if (X_(x, n, m)) t1++; else f0++;
      } else {
        if (X_(x, n, m)) f1++; else t0++;
      }
    }
    x->t0a += t0; x->f0a += f0; x->t1a += t1; x->f1a += f1;
    x->t0[m] = t0; x->f0[m] = f0; x->t1[m] = t1; x->f1[m] = f1;
  }
}

/* mcmc_logtop, mcmc.c:711-748 */
static void om_logtop(double *p, int n)
{
  int i;
  double x, y, z;
  z = p[0];
  for (i = 1; i < n; i++)
    if (p[i] > z) z = p[i];
  x = 0.;
  for (i = 0; i < n; i++) {
    double t = p[i] - z;
    y = om_exp(OM_LOGEPSILON > t ? OM_LOGEPSILON : t);    /* GSL_MAX(LOGEPSILON, .) */
    p[i] = y;
    x += y;
  }
  for (i = 0; i < n; i++) p[i] = p[i] / x;
}

/* mcmc_samplebeta, mcmc.c:751-765 */
static double om_samplebeta(om_model *mo, double *x, double a, double b, double low, double high)
{
  double y = om_beta(&mo->rng, 1. + a, 1. + b);
  if (y > 0.) {
    y = om_log(y);
    if (low <= y && y <= high) *x = y;
  }
  return *x;
}

/* mcmc_samplec, mcmc.c:768-795 */
static int om_samplec(om_model *x)
{
  double y;
  if (x->manycd) {
    for (int m = 0; m < x->M; m++) {
      y = x->c[m];
      om_samplebeta(x, &y, x->f1[m], x->t0[m], OM_MINC, OM_MAXC);
      x->c[m] = y;
    }
    return x->M;
  }
  y = x->c[0];
  om_samplebeta(x, &y, x->f1a, x->t0a, OM_MINC, OM_MAXC);
  for (int m = 0; m < x->M; m++) x->c[m] = y;
  return 1;
}

/* mcmc_sampled, mcmc.c:798-825 */
static int om_sampled(om_model *x)
{
  double y;
  if (x->manycd) {
    for (int m = 0; m < x->M; m++) {
      y = x->d[m];
      om_samplebeta(x, &y, x->f0[m], x->t1[m], OM_MIND, OM_MAXD);
      x->d[m] = y;
    }
    return x->M;
  }
  y = x->d[0];
  om_samplebeta(x, &y, x->f0a, x->t1a, OM_MIND, OM_MAXD);
  for (int m = 0; m < x->M; m++) x->d[m] = y;
  return 1;
}

/* mcmc_randompick, mcmc.c:901-915, with the uniform given (om_pick_u) or drawn */
static int om_pick_u(const double *p, int n, double u)
{
  int i = 0;
  double x = u - p[0];
  while (x > 0. && i < n - 1) x -= p[++i];
  return i;
}

static int om_randompick(om_model *mo, const double *p, int n)
{
  return om_pick_u(p, n, om_uniform(&mo->rng));
}

/* mcmc_auxa's weights (mcmc.c:828-897 up to the randompick): the count deltas dt0..df1[0..b] of moving the limit
 * from *a to each entry and q[0..b] = the pick probabilities after mcmc_logtop */
static void om_auxa_weights(const int *x, int b, int a, double c, double d, double *q, int *dt0, int *df0, int *dt1,
                            int *df1)
{
  int i;
  double cc, dd;
  q[a] = 0.;
  dt0[a] = df0[a] = dt1[a] = df1[a] = 0;
  cc = om_log(1. - om_exp(c));
  dd = om_log(1. - om_exp(d));
  for (i = a - 1; i >= 0; i--) {
    if (x[i]) {
      dt0[i] = dt0[i + 1]; df0[i] = df0[i + 1];
      dt1[i] = dt1[i + 1] + 1; df1[i] = df1[i + 1] - 1;
    } else {
      dt0[i] = dt0[i + 1] - 1; df0[i] = df0[i + 1] + 1;
      dt1[i] = dt1[i + 1]; df1[i] = df1[i + 1];
    }
  }
  for (i = a + 1; i <= b; i++) {
    if (x[i - 1]) {
      dt0[i] = dt0[i - 1]; df0[i] = df0[i - 1];
      dt1[i] = dt1[i - 1] - 1; df1[i] = df1[i - 1] + 1;
    } else {
      dt0[i] = dt0[i - 1] + 1; df0[i] = df0[i - 1] - 1;
      dt1[i] = dt1[i - 1]; df1[i] = df1[i - 1];
    }
  }
  for (i = 0; i <= b; i++)
    q[i] = dt0[i] * cc + df0[i] * d + dt1[i] * dd + df1[i] * c;
  om_logtop(q, b + 1);
}

/* mcmc_auxa, mcmc.c:828-898 */
static void om_auxa(om_model *mo, const int *x, int b, double c, double d,
                    int *a, int *t0, int *f0, int *t1, int *f1)
{
  double *q = mo->q;
  int *dt0 = mo->dt0, *df0 = mo->df0, *dt1 = mo->dt1, *df1 = mo->df1;
  om_auxa_weights(x, b, *a, c, d, q, dt0, df0, dt1, df1);
  *a = om_randompick(mo, q, b + 1);
  *t0 += dt0[*a]; *f0 += df0[*a]; *t1 += dt1[*a]; *f1 += df1[*a];
}

/* mcmc_sampleab, mcmc.c:918-996 */
static int om_sampleab(om_model *x)
{
  int m, t, count = 0, t0, f0, t1, f1, n;
  double c, d;
  int *v = x->v;
  for (m = 0; m < x->M; m++) {
    for (n = 0; n < x->N; n++) v[n] = X_(x, x->rpi[n], m);   /* get_col + permute(rpi) */
    t = x->a[m];
    t0 = x->t0[m]; f0 = x->f0[m]; t1 = x->t1[m]; f1 = x->f1[m];
    c = x->c[m]; d = x->d[m];
    om_auxa(x, v, x->b[m], c, d, &t, &t0, &f0, &t1, &f1);
    if (t != x->a[m]) { x->a[m] = t; count++; }
    for (n = 0; n < x->N / 2; n++) { int s = v[n]; v[n] = v[x->N - 1 - n]; v[x->N - 1 - n] = s; }
    t = x->N - x->b[m];
    om_auxa(x, v, x->N - x->a[m], c, d, &t, &t0, &f0, &t1, &f1);
    x->t0[m] = t0; x->f0[m] = f0; x->t1[m] = t1; x->f1[m] = f1;
    if (t != x->N - x->b[m]) { x->b[m] = x->N - t; count++; }
  }
  x->t0a = x->f0a = x->t1a = x->f1a = 0;
  for (m = 0; m < x->M; m++) {
    x->t0a += x->t0[m]; x->f0a += x->f0[m]; x->t1a += x->t1[m]; x->f1a += x->f1[m];
  }
  x->loglik = om_logl(x);
  return count;
}

/* mcmc_consistent, mcmc.c:999-1094.  mutate!=0 reproduces the reference exactly
 * (recount + loglik := logl); mutate==0 checks without touching the model. */
static int om_consistent(om_model *x, int mutate, int verbose)
{
  int flag = 0, i, n, m;
  for (m = 0; m < x->M; m++) {
    int a = x->a[m], b = x->b[m];
    if (!(0 <= a && a <= b && b <= x->N)) {
      if (verbose) fprintf(stderr, "mcmc_consistent: error. a(%d) = %d  b(%d) = %d\n", m, a, m, b);
      flag = 1;
    }
  }
  int *seen = (int *)calloc(x->N, sizeof(int));
  for (n = 0; n < x->N; n++) {
    if (x->pi[n] < 0 || x->pi[n] >= x->N || seen[x->pi[n]]++) {
      if (verbose) fprintf(stderr, "mcmc_consistent: invalid permutation.\n");
      flag = 1; break;
    }
  }
  free(seen);
  for (n = 0; n < x->N; n++) {
    if (x->pi[n] >= 0 && x->pi[n] < x->N && x->rpi[x->pi[n]] != n) {
      if (verbose) fprintf(stderr, "mcmc_consistent: rpi is not inverse of pi.\n");
      flag = 1; break;
    }
  }
  m = -1; i = 0;
  for (n = 0; n < x->N; n++) {
    if (x->h[n]) {
      i++;
      if (m >= 0 && x->pi[n] < m) {
        if (verbose) fprintf(stderr, "mcmc_consistent: hard site order is incorrect %d %d %d.\n", n, x->pi[n], m);
        flag = 1;
      }
      m = x->pi[n];
    }
  }
  if (i != x->nh) { if (verbose) fprintf(stderr, "mcmc_consistent: incorrect number of hard sites.\n"); flag = 1; }
  int t0 = x->t0a, f0 = x->f0a, t1 = x->t1a, f1 = x->f1a;
  double loglik = x->loglik;
  if (mutate) {
    om_count01(x);
    x->loglik = om_logl(x);
    double delta = loglik - x->loglik;
    if (delta < 0.) delta = -delta;
    if (t0 != x->t0a || f0 != x->f0a || t1 != x->t1a || f1 != x->f1a || delta > 1e-8) {
      if (verbose) fprintf(stderr, "mcmc_consistent: inconsistent parameters.\n");
      flag = 1;
    }
  } else {
    int *sv = (int *)malloc(4 * x->M * sizeof(int));
    memcpy(sv, x->t0, x->M * sizeof(int)); memcpy(sv + x->M, x->f0, x->M * sizeof(int));
    memcpy(sv + 2 * x->M, x->t1, x->M * sizeof(int)); memcpy(sv + 3 * x->M, x->f1, x->M * sizeof(int));
    om_count01(x);
    double l2 = om_logl(x);
    double delta = loglik - l2;
    if (delta < 0.) delta = -delta;
    if (t0 != x->t0a || f0 != x->f0a || t1 != x->t1a || f1 != x->f1a || delta > 1e-8 ||
        memcmp(sv, x->t0, x->M * sizeof(int)) || memcmp(sv + x->M, x->f0, x->M * sizeof(int)) ||
        memcmp(sv + 2 * x->M, x->t1, x->M * sizeof(int)) || memcmp(sv + 3 * x->M, x->f1, x->M * sizeof(int))) {
      if (verbose) fprintf(stderr, "mcmc_consistent: inconsistent parameters.\n");
      flag = 1;
    }
    free(sv);
  }
  return flag;
}

/* mcmc_ininterval, mcmc.c:1097-1124 */
static int om_ininterval(int i, int a, int b, int inc1, int inc2)
{
  int r;
  if (a > b) { r = a; a = b; b = r; }
  r = inc1 ? (a <= i) : (a < i);
  if (r) r = inc2 ? (i <= b) : (i < b);
  return r;
}

/* mcmc_samplepi1, mcmc.c:1127-1308 */
static int om_samplepi1(om_model *x)
{
  int n, m, i, j, ii, jj, a, b, ain, bin, t;
  int dt0, df0, dt1, df1;
  double delta, c, d, aA_ = 0.0;
  int nK_ = 0;
  const int *v;
  i = (int)om_uniform_int(&x->rng, x->N);
  j = (int)om_uniform_int(&x->rng, x->N - 1);
  if (j >= i) j++;
  if (i < j) { ii = i; jj = j; } else { ii = j; jj = i; }
  if (x->h[x->rpi[i]]) {
    m = 0;
    for (n = ii; n <= jj; n++) {
      m += x->h[x->rpi[n]];
      if (m > 1) return 0;
    }
  }
  v = &X_(x, x->rpi[i], 0);
  delta = 0.;
  for (m = 0; m < x->M; m++) {
    dt0 = df0 = dt1 = df1 = 0;
    a = x->a[m]; b = x->b[m];
    if (i < j) {
      ain = (ii < a && a <= jj + 1);
      bin = (ii < b && b <= jj + 1);
      if (ain && !bin) {
        if (v[m]) { dt1++; df1--; } else { dt0--; df0++; }
      } else if (!ain && bin) {
        if (v[m]) { dt1--; df1++; } else { dt0++; df0--; }
      }
    } else {
      ain = (ii <= a && a <= jj);
      bin = (ii <= b && b <= jj);
      if (!ain && bin) {
        if (v[m]) { dt1++; df1--; } else { dt0--; df0++; }
      } else if (ain && !bin) {
        if (v[m]) { dt1--; df1++; } else { dt0++; df0--; }
      }
    }
    c = x->c[m]; d = x->d[m];
    { double t_ = dt0 * om_log(1. - om_exp(c)) + df0 * d + dt1 * om_log(1. - om_exp(d)) + df1 * c;
      delta += t_; if (t_ != 0.0) { nK_++; aA_ += t_ < 0 ? -t_ : t_; } }
  }
  om_note(delta, nK_, aA_);
  if (delta >= 0. || delta > om_log(om_uniform_pos(&x->rng))) {
    if (i < j) {
      for (m = 0; m < x->M; m++) {
        a = x->a[m]; b = x->b[m];
        if (ii < a && a <= jj + 1) x->a[m] = a - 1;
        if (ii < b && b <= jj + 1) x->b[m] = b - 1;
      }
      t = x->rpi[i];
      for (n = i; n < j; n++) x->rpi[n] = x->rpi[n + 1];
      x->rpi[j] = t;
    } else {
      for (m = 0; m < x->M; m++) {
        a = x->a[m]; b = x->b[m];
        if (ii <= a && a <= jj) x->a[m] = a + 1;
        if (ii <= b && b <= jj) x->b[m] = b + 1;
      }
      t = x->rpi[i];
      for (n = i; n > j; n--) x->rpi[n] = x->rpi[n - 1];
      x->rpi[j] = t;
    }
    om_inverse(x->pi, x->rpi, x->N);
    x->loglik += delta;
    om_count01(x);
    return 1;
  }
  return 0;
}

/* mcmc_samplepi2, mcmc.c:1311-1486 */
static int om_samplepi2(om_model *x, int swap)
{
  int i, j, n, m, a, b, inc1, inc2, ain, bin;
  int dt0, df0, dt1, df1;
  double delta, c, d, aA_ = 0.0;
  int nK_ = 0;
  if (!swap) {
    i = (int)om_uniform_int(&x->rng, x->N);
    j = (int)om_uniform_int(&x->rng, x->N - 1);
    if (j >= i) j++;
    else { n = i; i = j; j = n; }
  } else {
    i = (int)om_uniform_int(&x->rng, x->N - 1);
    j = i + 1;
  }
  m = 0;
  for (n = i; n <= j; n++) {
    m += x->h[x->rpi[n]];
    if (m > 1) return 0;
  }
  inc1 = (int)om_uniform_int(&x->rng, 2);
  inc2 = (int)om_uniform_int(&x->rng, 2);
  delta = 0.;
  for (m = 0; m < x->M; m++) {
    dt0 = df0 = dt1 = df1 = 0;
    a = x->a[m]; b = x->b[m];
    ain = om_ininterval(a, i, j + 1, inc1, inc2);
    bin = om_ininterval(b, i, j + 1, inc1, inc2);
    if (ain && !bin) {
      for (n = i; n < a; n++) {
        if (X_(x, x->rpi[n], m)) { dt1++; df1--; } else { dt0--; df0++; }
      }
      for (n = a; n <= j; n++) {
        if (X_(x, x->rpi[n], m)) { dt1--; df1++; } else { dt0++; df0--; }
      }
    } else if (!ain && bin) {
      for (n = i; n < b; n++) {
        if (X_(x, x->rpi[n], m)) { dt1--; df1++; } else { dt0++; df0--; }
      }
      for (n = b; n <= j; n++) {
        if (X_(x, x->rpi[n], m)) { dt1++; df1--; } else { dt0--; df0++; }
      }
    }
    c = x->c[m]; d = x->d[m];
    { double t_ = dt0 * om_log(1. - om_exp(c)) + df0 * d + dt1 * om_log(1. - om_exp(d)) + df1 * c;
      delta += t_; if (t_ != 0.0) { nK_++; aA_ += t_ < 0 ? -t_ : t_; } }
  }
  om_note(delta, nK_, aA_);
  if (delta >= 0. || delta > om_log(om_uniform_pos(&x->rng))) {
    for (m = 0; m < x->M; m++) {
      a = x->a[m]; b = x->b[m];
      ain = om_ininterval(a, i, j + 1, inc1, inc2);
      bin = om_ininterval(b, i, j + 1, inc1, inc2);
      if (ain && !bin) x->a[m] = i + j + 1 - a;
      else if (!ain && bin) x->b[m] = i + j + 1 - b;
      else if (ain && bin) { x->b[m] = i + j + 1 - a; x->a[m] = i + j + 1 - b; }
    }
    for (n = i; n <= (i + j) / 2; n++) {
      m = x->rpi[n]; x->rpi[n] = x->rpi[i + j - n]; x->rpi[i + j - n] = m;
    }
    om_inverse(x->pi, x->rpi, x->N);
    x->loglik += delta;
    om_count01(x);
    return 1;
  }
  return 0;
}

/* mcmc_samplepi3, mcmc.c:1489-1682 */
static int om_samplepi3(om_model *x)
{
  int i, j, n, m, a, b, nn, na, nb, inc1, inc2, ain, bin, wasalive, isalive;
  int dt0, df0, dt1, df1;
  double delta, c, d, aA_ = 0.0;
  int nK_ = 0;
  int *p = x->p;
  if (x->N - x->nh < 2) return 0;
  n = (int)om_uniform_int(&x->rng, x->N - x->nh);
  m = (int)om_uniform_int(&x->rng, x->N - x->nh - 1);
  if (n <= m) { i = n; j = m + 1; } else { i = m; j = n; }
  n = 0;
  while (n <= i) { if (x->h[x->rpi[n]]) { i++; j++; } n++; }
  while (n <= j) { if (x->h[x->rpi[n]]) j++; n++; }
  n = i; m = j;
  while (n <= m) {
    if (x->h[x->rpi[n]]) { p[n] = n; n++; }
    else if (x->h[x->rpi[m]]) { p[m] = m; m--; }
    else { p[n] = m; p[m] = n; n++; m--; }
  }
  inc1 = (int)om_uniform_int(&x->rng, 2);
  inc2 = (int)om_uniform_int(&x->rng, 2);
  delta = 0.;
  for (m = 0; m < x->M; m++) {
    dt0 = df0 = dt1 = df1 = 0;
    a = x->a[m]; b = x->b[m];
    ain = om_ininterval(a, i, j + 1, inc1, inc2);
    bin = om_ininterval(b, i, j + 1, inc1, inc2);
    if (ain && !bin) { na = i + j + 1 - a; nb = b; }
    else if (!ain && bin) { na = a; nb = i + j + 1 - b; }
    else if (ain && bin) { na = i + j + 1 - b; nb = i + j + 1 - a; }
    else { na = a; nb = b; }
    for (n = i; n <= j; n++) {
      nn = p[n];
      wasalive = (a <= n && n < b);
      isalive = (na <= nn && nn < nb);
      if (wasalive && !isalive) {
        if (X_(x, x->rpi[n], m)) { dt1--; df1++; } else { df0--; dt0++; }
      } else if (!wasalive && isalive) {
        if (X_(x, x->rpi[n], m)) { dt1++; df1--; } else { df0++; dt0--; }
      }
    }
    c = x->c[m]; d = x->d[m];
    { double t_ = dt0 * om_log(1. - om_exp(c)) + df0 * d + dt1 * om_log(1. - om_exp(d)) + df1 * c;
      delta += t_; if (t_ != 0.0) { nK_++; aA_ += t_ < 0 ? -t_ : t_; } }
  }
  om_note(delta, nK_, aA_);
  if (delta >= 0. || delta > om_log(om_uniform_pos(&x->rng))) {
    for (m = 0; m < x->M; m++) {
      a = x->a[m]; b = x->b[m];
      ain = om_ininterval(a, i, j + 1, inc1, inc2);
      bin = om_ininterval(b, i, j + 1, inc1, inc2);
      if (ain && !bin) x->a[m] = i + j + 1 - a;
      else if (!ain && bin) x->b[m] = i + j + 1 - b;
      else if (ain && bin) { x->b[m] = i + j + 1 - a; x->a[m] = i + j + 1 - b; }
    }
    for (n = i; n <= j; n++) { a = p[n]; p[n] = x->rpi[a]; }
    for (n = i; n <= j; n++) x->rpi[n] = p[n];
    om_inverse(x->pi, x->rpi, x->N);
    x->loglik += delta;
    om_count01(x);
    return 1;
  }
  return 0;
}

/* mcmc_sample, mcmc.c:214-258 (sweeps = 10 in the reference) */
static int om_sample(om_model *x, int sweeps)
{
  for (int i = 0; i < sweeps; i++) {
    x->acc[0] += om_samplec(x);
    x->acc[1] += om_sampled(x);
    x->acc[2] += om_sampleab(x);
    x->acc[5] += om_samplepi2(x, 1);
    for (int j = 0; j < 5; j++) {
      x->acc[3] += om_samplepi1(x);
      x->acc[4] += om_samplepi2(x, 0);
      x->acc[6] += om_samplepi3(x);
    }
  }
  return 0;
}

/* ------------------------------------------------------------ library API */


#define OM_API __attribute__((visibility("default")))

OM_API void oracle_stats(long long *out8, double *meanK_meanA)
{
  for (int k = 0; k < 8; k++) out8[k] = om_stat[k];
  meanK_meanA[0] = om_stat_acc_K; meanK_meanA[1] = om_stat_A;
  for (int k = 0; k < 8; k++) om_stat[k] = 0;
  om_stat_acc_K = om_stat_A = 0;
}

/* Parse a dataset (reference text format).  X_out may be NULL (dims only). */
OM_API int oracle_parse(const char *text, long len, int maxs, int *N, int *M, int *nh,
                        int32_t *X_out, int32_t *h_out)
{
  om_model x;
  int rc = om_readmodel(&x, text, (size_t)len, maxs, 0);
  if (rc) return rc;
  *N = x.N; *M = x.M; *nh = x.nh;
  if (X_out) for (size_t k = 0; k < (size_t)x.N * x.M; k++) X_out[k] = x.X[k];
  if (h_out) for (int k = 0; k < x.N; k++) h_out[k] = x.h[k];
  om_free(&x);
  return 0;
}

/*
 * Run one chain exactly as `main` does (mcmc.c:102-210): init, randomize, tb burn-in
 * calls of mcmc_sample, then ts calls each followed by a saved record.
 *   init_out (optional): 2M+N ints = a, b, pi after randomize; init_dbl: c0, d0, loglik
 *   rec_int  (optional): ts*(2M+N) ints = a, b, pi per saved sample
 *   rec_dbl  (optional): ts*3 doubles  = c[0], d[0], loglik per saved sample
 *   exp_out  (optional): exp_loglik, exp_c, exp_d exactly as print_exp_data (/1000)
 *   acc_out  (optional): 7 cumulative acceptance counters; rng_words: words drawn
 *   check:   1 = verify mcmc_consistent (non-mutating) after every call
 * Returns 0, parse error (<0), or 1 if the final/check consistency test failed.
 */
/* 1: the sampling phase of oracle_run_chain draws from the Philox stream (the product's opt-in
 * SR_F_RNG_PHILOX mode), initialisation stays MT19937; 0: the reference's MT19937 throughout */
static int g_rng_philox = 0;
OM_API void oracle_set_rng(int philox) { g_rng_philox = philox ? 1 : 0; }

/* wall seconds of the last oracle_run_chain(_v) on this thread: [0] the tb burn-in calls, [1] the ts saved calls
 * (bench.py's cpu_baseline times the calls after the GPU's warm-up window, mcmc.c:140-185's two loops) */
static __thread double om_phase_s[2];
static double om_now(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
OM_API void oracle_phase_seconds(double *out2) { out2[0] = om_phase_s[0]; out2[1] = om_phase_s[1]; }

/* rec_cdv (optional, manycd runs): ts*2M doubles = every taxon's c then d per saved sample */
OM_API int oracle_run_chain_v(const char *text, long len, int maxs, unsigned long seed, int manycd,
                              int tb, int ts, int sweeps, int check,
                              int32_t *init_out, double *init_dbl,
                              int32_t *rec_int, double *rec_dbl, double *rec_cdv, double *exp_out,
                              long long *acc_out, unsigned long long *rng_words);

OM_API int oracle_run_chain(const char *text, long len, int maxs, unsigned long seed, int manycd,
                            int tb, int ts, int sweeps, int check,
                            int32_t *init_out, double *init_dbl,
                            int32_t *rec_int, double *rec_dbl, double *exp_out,
                            long long *acc_out, unsigned long long *rng_words)
{
  return oracle_run_chain_v(text, len, maxs, seed, manycd, tb, ts, sweeps, check, init_out, init_dbl, rec_int, rec_dbl,
                            NULL, exp_out, acc_out, rng_words);
}

OM_API int oracle_run_chain_v(const char *text, long len, int maxs, unsigned long seed, int manycd,
                              int tb, int ts, int sweeps, int check,
                              int32_t *init_out, double *init_dbl,
                              int32_t *rec_int, double *rec_dbl, double *rec_cdv, double *exp_out,
                              long long *acc_out, unsigned long long *rng_words)
{
  om_model x;
  int rc = om_readmodel(&x, text, (size_t)len, maxs, manycd);
  if (rc) return rc;
  om_rng_seed(&x.rng, seed);
  om_randomize(&x);
  if (g_rng_philox) om_rng_philox(&x.rng, seed);
  int bad = om_consistent(&x, 1, 0);
  const int N = x.N, M = x.M, W = 2 * M + N;
  if (init_out) {
    for (int m = 0; m < M; m++) { init_out[m] = x.a[m]; init_out[M + m] = x.b[m]; }
    for (int n = 0; n < N; n++) init_out[2 * M + n] = x.pi[n];
  }
  if (init_dbl) { init_dbl[0] = x.c[0]; init_dbl[1] = x.d[0]; init_dbl[2] = x.loglik; }
  const double t0 = om_now();
  for (int i = 0; i < tb; i++) {
    om_sample(&x, sweeps);
    if (check && om_consistent(&x, 0, 1)) bad = 1;
  }
  const double t1 = om_now();
  double ls = 0, cs = 0, ds = 0;
  for (int i = 0; i < ts; i++) {
    om_sample(&x, sweeps);
    if (check && om_consistent(&x, 0, 1)) bad = 1;
    if (rec_int) {
      int32_t *r = rec_int + (size_t)i * W;
      for (int m = 0; m < M; m++) { r[m] = x.a[m]; r[M + m] = x.b[m]; }
      for (int n = 0; n < N; n++) r[2 * M + n] = x.pi[n];
    }
    if (rec_dbl) { rec_dbl[3 * i] = x.c[0]; rec_dbl[3 * i + 1] = x.d[0]; rec_dbl[3 * i + 2] = x.loglik; }
    if (rec_cdv) {
      memcpy(rec_cdv + (size_t)i * 2 * M, x.c, (size_t)M * sizeof(double));
      memcpy(rec_cdv + (size_t)i * 2 * M + M, x.d, (size_t)M * sizeof(double));
    }
    ls += -(x.loglik);                  /* compute_exp_data, mcmc.c:53-58 (libm exp there) */
    cs += exp(x.c[0]);
    ds += exp(x.d[0]);
  }
  om_phase_s[0] = t1 - t0;
  om_phase_s[1] = om_now() - t1;
  if (exp_out) { exp_out[0] = ls / 1000; exp_out[1] = cs / 1000; exp_out[2] = ds / 1000; }
  if (acc_out) memcpy(acc_out, x.acc, sizeof(x.acc));
  if (rng_words) *rng_words = x.rng.ndraw;
  if (om_consistent(&x, 1, 1)) bad = 1;
  om_free(&x);
  return bad ? 1 : 0;
}

/* ---- references of the device certification self-tests (tests/test_gpu_cert.py) ----
 * oracle_auxa_pick: mcmc_auxa + mcmc_logtop + mcmc_randompick (mcmc.c:828-915) over walk-order bits x[0..b) from
 * limit a, with the uniform u given instead of drawn; returns the pick, p_out (optional, b + 1) the probabilities
 * randompick subtracts.  oracle_auxa_boundary: the smallest u in [0, 1] whose pick exceeds entry i -- the
 * reference's own CDF boundary, with its sequential subtractions -- by bisection over the ordered doubles of [0, 1]
 * (each subtraction is monotone in its minuend, so the pick is monotone in u). */
static int om_auxa_alloc(int b, double **q, int **dt)
{
  *q = (double *)malloc(sizeof(double) * (size_t)(b + 1));
  *dt = (int *)malloc(sizeof(int) * 4 * (size_t)(b + 1));
  return *q && *dt;
}

OM_API int oracle_auxa_pick(const int32_t *x, int b, int a, double c, double d, double u, double *p_out)
{
  double *q;
  int *dt;
  if (b < 0 || a < 0 || a > b || !om_auxa_alloc(b, &q, &dt)) return -1;
  om_auxa_weights(x, b, a, c, d, q, dt, dt + b + 1, dt + 2 * (b + 1), dt + 3 * (b + 1));
  const int r = om_pick_u(q, b + 1, u);
  if (p_out) memcpy(p_out, q, sizeof(double) * (size_t)(b + 1));
  free(q); free(dt);
  return r;
}

OM_API double oracle_auxa_boundary(const int32_t *x, int b, int a, double c, double d, int i)
{
  double *q;
  int *dt;
  if (b < 0 || a < 0 || a > b || i < 0 || i >= b || !om_auxa_alloc(b, &q, &dt)) return -1.0;
  om_auxa_weights(x, b, a, c, d, q, dt, dt + b + 1, dt + 2 * (b + 1), dt + 3 * (b + 1));
  double one = 1.0;
  uint64_t lo = 0, hi;
  memcpy(&hi, &one, 8);
  double r = 2.0;
  if (om_pick_u(q, b + 1, 1.0) > i) {
    while (lo < hi) {   /* invariant: pick(bits hi) > i */
      const uint64_t mid = lo + (hi - lo) / 2;
      double um;
      memcpy(&um, &mid, 8);
      if (om_pick_u(q, b + 1, um) > i) hi = mid; else lo = mid + 1;
    }
    memcpy(&r, &hi, 8);
  }
  free(q); free(dt);
  return r;   /* 2.0: no u in [0, 1] picks beyond i */
}

/* a proposal's delta as the reference sums it (mcmc_samplepi1 / pi2 / pi3 / swap, e.g. mcmc.c:1300-1304): per
 * taxon dt0 cc + df0 d + dt1 dd + df1 c with df0 = -dt0, df1 = -dt1 (cc = log(1 - e^c), dd = log(1 - e^d)), added
 * in taxon order; and its acceptance (mcmc.c:492): 1 accepted without drawing u (delta >= 0), 2 accepted with the
 * uniform_pos u drawn (delta > log u), 0 rejected */
OM_API double oracle_delta_terms(const int32_t *dt0, const int32_t *dt1, long K, double c, double d)
{
  const double cc = om_log(1. - om_exp(c)), dd = om_log(1. - om_exp(d));
  double delta = 0.;
  for (long m = 0; m < K; m++) {
    const int df0 = -dt0[m], df1 = -dt1[m];
    delta += dt0[m] * cc + df0 * d + dt1[m] * dd + df1 * c;
  }
  return delta;
}

OM_API int oracle_mh_outcome(double delta, double u)
{
  if (delta >= 0.) return 1;
  return delta > om_log(u) ? 2 : 0;
}

/* Philox4x32-10 block probe (known-answer tests) */
OM_API void oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4])
{
  uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
  om_philox4x32_10(c, key[0], key[1]);
  memcpy(out, c, sizeof c);
}

/* RNG probes for the unit tests. kind: 0 raw u32, 1 uniform, 2 uniform_pos,
 * 3 uniform_int(n), 4 gaussian_ziggurat(1), 5 gamma(a), 6 beta(a, b). */
OM_API void oracle_rng_stream(unsigned long seed, int kind, double a, double b, long count,
                              double *out, unsigned long long *words)
{
  om_rng r;
  om_rng_seed(&r, seed);
  for (long k = 0; k < count; k++) {
    switch (kind) {
    case 0: out[k] = (double)om_rng_get(&r); break;
    case 1: out[k] = om_uniform(&r); break;
    case 2: out[k] = om_uniform_pos(&r); break;
    case 3: out[k] = (double)om_uniform_int(&r, (unsigned long)a); break;
    case 4: out[k] = om_gaussian_ziggurat(&r, 1.0); break;
    case 5: out[k] = om_gamma(&r, a, 1.0); break;
    default: out[k] = om_beta(&r, a, b); break;
    }
  }
  if (words) *words = r.ndraw;
}

OM_API void oracle_shuffle(unsigned long seed, int32_t *base, long n)
{
  om_rng r;
  om_rng_seed(&r, seed);
  om_shuffle(&r, base, (size_t)n, sizeof(int32_t));
}

OM_API int oracle_choose(unsigned long seed, int32_t *dest, long k, const int32_t *src, long n)
{
  om_rng r;
  om_rng_seed(&r, seed);
  return om_choose(&r, dest, (size_t)k, src, (size_t)n, sizeof(int32_t));
}

OM_API void oracle_exp_log(const double *in, long n, double *out_exp, double *out_log)
{
  for (long k = 0; k < n; k++) {
    if (out_exp) out_exp[k] = om_exp(in[k]);
    if (out_log) out_log[k] = om_log(in[k]);
  }
}

/* The pin of om_libm.h: count inputs where om_exp / om_log differ (bitwise, NaN == NaN) from
 * this machine's glibc exp() / log(), the functions the reference calls.  Called through a
 * volatile pointer so the compiler neither folds nor inlines them. */
static int om_same(double a, double b) { return om_bits(a) == om_bits(b) || (a != a && b != b); }
OM_API void oracle_libm_mismatch(const double *in, long n, long *bad_exp, long *bad_log)
{
  double (*volatile gexp)(double) = exp, (*volatile glog)(double) = log;
  long be = 0, bl = 0;
  for (long k = 0; k < n; k++) {
    be += !om_same(om_exp(in[k]), gexp(in[k]));
    bl += !om_same(om_log(in[k]), glog(in[k]));
  }
  *bad_exp = be;
  *bad_log = bl;
}

/* ---------------------------------------------------------------- CLI */
#ifdef OM_MAIN
/* The reference CLI (mcmc.c:102-210): `mcmc_oracle [chain_index]` reading the dataset
 * on stdin, seed from GSL_RNG_SEED, writing Chains/chain_XX/{taxa,sites,hard_sites,
 * exp_data,chain_data}.csv exactly as the reference formats them. */
static void om_save_chain(const om_model *x, FILE *f)                 /* mcmc.c:69-92 */
{
  int i;
  for (i = 0; i < x->M; i++) fprintf(f, "%d ", x->a[i]);
  fprintf(f, ",");
  for (i = 0; i < x->M; i++) fprintf(f, "%d ", x->b[i]);
  fprintf(f, ",");
  for (i = 0; i < x->N; i++) fprintf(f, "%d ", x->pi[i]);
  fprintf(f, ",");
  for (i = 0; i < x->M; i++) fprintf(f, "%.14f ", exp(x->c[i]));
  fprintf(f, ",");
  for (i = 0; i < x->M; i++) fprintf(f, "%.14f ", exp(x->d[i]));
  fprintf(f, ",%.14f\n", x->loglik);
}

int main(int argc, char *argv[])
{
  int tb = 1000, ts = 1000, manycd = 0;
  const char *chain_index = NULL;
  FILE *lf = fopen("mcmc_c.log", "a");
  if (lf) fclose(lf);
  switch (argc) {
  case 1: break;
  case 2: chain_index = argv[1]; break;
  case 4:
    if (sscanf(argv[1], "%d", &manycd) && sscanf(argv[2], "%d", &tb) == 1 && tb >= 0 &&
        sscanf(argv[3], "%d", &ts) == 1 && ts >= 0) break;
    /* fallthrough */
  default:
    fprintf(stderr, "usage: %s [manycd Tburnin T]\n", argv[0]);
    return 1;
  }
  unsigned long seed = 0;
  if (om_rng_env_setup(&seed)) return 1;   /* mcmc_init, mcmc.c:591-592 */
  size_t cap = 1 << 16, len = 0;
  char *text = (char *)malloc(cap);
  size_t got;
  while ((got = fread(text + len, 1, cap - len, stdin)) > 0) {
    len += got;
    if (len == cap) { cap *= 2; text = (char *)realloc(text, cap); }
  }
  om_model x;
  om_diag = 1;
  int rc = om_readmodel(&x, text, len, OM_MAXS, manycd);
  free(text);
  if (rc == -2) { fprintf(stderr, "mcmc_readmodel: read error at header.\n"); return 1; }
  if (rc) { fprintf(stderr, "mcmc_readmodel: read error.\n"); return 1; }
  om_rng_seed(&x.rng, seed);
  om_randomize(&x);
  om_consistent(&x, 1, 1);
  for (int i = 0; i < tb; i++) om_sample(&x, 10);
  char dir[64];
  int idx = chain_index ? atoi(chain_index) : 0;
  if (idx > 9) snprintf(dir, sizeof dir, "Chains/chain_%c%c", chain_index[0], chain_index[1]);
  else snprintf(dir, sizeof dir, "Chains/chain_0%c", chain_index ? chain_index[0] : '0');
  char path[128];
  snprintf(path, sizeof path, "%s/chain_data.csv", dir);
  FILE *fchain = fopen(path, "w");
  if (!fchain) { fprintf(stderr, "cannot open %s\n", path); return 1; }
  double ls = 0, cs = 0, ds = 0;
  for (int i = 0; i < ts; i++) {
    om_sample(&x, 10);
    om_save_chain(&x, fchain);
    ls += -(x.loglik); cs += exp(x.c[0]); ds += exp(x.d[0]);
  }
  FILE *f1, *f2, *f3, *f4;
  snprintf(path, sizeof path, "%s/taxa.csv", dir); f1 = fopen(path, "w");
  snprintf(path, sizeof path, "%s/sites.csv", dir); f2 = fopen(path, "w");
  snprintf(path, sizeof path, "%s/hard_sites.csv", dir); f3 = fopen(path, "w");
  snprintf(path, sizeof path, "%s/exp_data.csv", dir); f4 = fopen(path, "w");
  ls /= 1000; cs /= 1000; ds /= 1000;                               /* mcmc.c:60-67 */
  fprintf(f4, "exp_loglik,exp_c,exp_d\n");
  fprintf(f4, "%.14f,%.14f,%.14f", ls, cs, ds);
  fprintf(f1, "a,b,c,d\n");                                          /* mcmc.c:261-293 */
  for (int i = 0; i < x.M; i++) fprintf(f1, "%d,%d,%.14f,%.14f\n", x.a[i], x.b[i], exp(x.c[i]), exp(x.d[i]));
  fprintf(f2, "sites\n");
  for (int i = 0; i < x.N; i++) fprintf(f2, "%d\n", x.pi[i]);
  fprintf(f3, "i,pi_i\n");
  for (int i = 0; i < x.N; i++) if (x.h[i]) fprintf(f3, "%d,%d\n", i, x.pi[i]);
  fclose(f1); fclose(f2); fclose(f3); fclose(f4); fclose(fchain);
  if (om_consistent(&x, 1, 1)) { fprintf(stderr, "main: error.\n"); return 1; }
  om_free(&x);
  return 0;
}
#endif
