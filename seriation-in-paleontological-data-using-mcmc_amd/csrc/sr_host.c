/*
 * sr_host.c -- C host layer of libseriation.so (implements include/seriation.h).
 *
 * Responsibilities (reference file:line in C_Implementation/mcmc.c):
 *   parsing                 mcmc_readmodel            :339-437  (fgets(MAXS) semantics)
 *   chain initialisation    mcmc_init/initab/randomize/count01/logl  :440-593, 625-708
 *   device state build      P columns in position order, hard positions, MT ring
 *   run loop                main()'s burn-in + sampling loops  :140-185 (on the GPU)
 *   summaries               compute_exp_data/print_exp_data    :53-67
 *   consistency             mcmc_consistent                    :999-1094
 *   output files            mcmc_save_chain / mcmc_save         :69-92, 261-293
 * The sweep itself runs only in sr_device.hip; there is no CPU fallback: without a
 * usable gfx950 device every run entry point returns SR_EDEVICE.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <math.h>
#include <errno.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <pthread.h>
#include <sched.h>
#include <unistd.h>
#include "seriation.h"
#include "sr_internal.h"
#include "sr_math.h"
#include "sr_rng.h"

#define SR_API __attribute__((visibility("default")))
#define SR_MAX_WRITERS 64   /* chain_data.csv formatting threads (SR_WRITER_THREADS, default = online CPUs) */

static const sr_mtab SR_HOST_TAB = {(const uint64_t *)sr_exp_tab, sr_log_tab};
static double h_exp(double x) { return sr_exp_m(x, &SR_HOST_TAB); }
static double h_log(double x) { return sr_log_m(x, &SR_HOST_TAB); }

SR_API const char *sr_version(void) { return "seriation-mi355x 0.1"; }

SR_API const char *sr_strerror(int code)
{
  switch (code) {
  case SR_OK: return "ok";
  case SR_EINVAL: return "invalid argument";
  case SR_EPARSE: return "mcmc_readmodel: read error.";
  case SR_EHEADER: return "mcmc_readmodel: read error at header.";
  case SR_ENOMEM: return "out of memory";
  case SR_EDEVICE: return "HIP device error (no usable gfx950 device?)";
  case SR_EUNSUPPORTED: return "configuration not supported by the kernel";
  case SR_EIO: return "cannot open or write an output file";
  case SR_EINCONSISTENT: return "mcmc_consistent: inconsistent chain state";
  default: return "unknown error";
  }
}

SR_API int sr_device_count(void) { return srk_device_count(); }

/* ------------------------------------------------------- GSL_RNG_TYPE / GSL_RNG_SEED */
/* gsl_rng_env_setup's contract (GSL 2.6 rng/env.c; the reference's mcmc_init calls it, mcmc.c:591-592): the
   generator named by GSL_RNG_TYPE out of gsl_rng_types_setup's list (rng/types.c, in its order), MT19937 when
   unset.  The sampler implements MT19937 (and the opt-in Philox stream) only, so any other generator is
   refused instead of silently sampling MT19937. */
static const char *const sr_gsl_rng_names[] = {
    "borosh13", "cmrg", "coveyou", "fishman18", "fishman20", "fishman2x", "gfsr4", "knuthran", "knuthran2",
    "knuthran2002", "lecuyer21", "minstd", "mrg", "mt19937", "mt19937_1999", "mt19937_1998", "r250", "ran0", "ran1",
    "ran2", "ran3", "rand", "rand48", "random128-bsd", "random128-glibc2", "random128-libc5", "random256-bsd",
    "random256-glibc2", "random256-libc5", "random32-bsd", "random32-glibc2", "random32-libc5", "random64-bsd",
    "random64-glibc2", "random64-libc5", "random8-bsd", "random8-glibc2", "random8-libc5", "random-bsd",
    "random-glibc2", "random-libc5", "randu", "ranf", "ranlux", "ranlux389", "ranlxd1", "ranlxd2", "ranlxs0",
    "ranlxs1", "ranlxs2", "ranmar", "slatec", "taus", "taus2", "taus113", "transputer", "tt800", "uni", "uni32",
    "vax", "waterman14", "zuf", NULL};

static int rng_type_check(int verbose)
{
  const char *p = getenv("GSL_RNG_TYPE");
  if (!p) return SR_OK;
  int known = 0;
  for (int k = 0; sr_gsl_rng_names[k]; k++) known |= strcmp(p, sr_gsl_rng_names[k]) == 0;
  if (!known) {   /* GSL: this list, then gsl_error("unknown generator") */
    if (verbose) {
      fprintf(stderr, "GSL_RNG_TYPE=%s not recognized\n", p);
      fprintf(stderr, "Valid generator types are:\n");
      for (int k = 0; sr_gsl_rng_names[k]; k++) {
        fprintf(stderr, " %18s", sr_gsl_rng_names[k]);
        if ((k + 1) % 4 == 0) fputc('\n', stderr);
      }
      fputc('\n', stderr);
    }
    return SR_EINVAL;
  }
  if (strcmp(p, "mt19937") != 0) {
    if (verbose)
      fprintf(stderr, "GSL_RNG_TYPE=%s: generator not available, only mt19937 (GSL's default) is implemented\n", p);
    return SR_EUNSUPPORTED;
  }
  if (verbose) fprintf(stderr, "GSL_RNG_TYPE=%s\n", p);
  return SR_OK;
}

SR_API int sr_rng_env_setup(uint64_t *seed, int32_t verbose)
{
  const int rc = rng_type_check(verbose);
  if (rc) return rc;
  unsigned long v = 0;
  const char *s = getenv("GSL_RNG_SEED");
  if (s) {
    v = strtoul(s, 0, 0);
    if (verbose) fprintf(stderr, "GSL_RNG_SEED=%lu\n", v);
  }
  if (seed) *seed = (uint64_t)v;
  return SR_OK;
}

/* ------------------------------------------------------------------ parsing */

/* one fgets(s, maxs, f) over the buffer; returns line length or -1 at EOF */
static long next_line(const char *text, size_t len, size_t *off, int maxs, char **buf, size_t *cap)
{
  if (*off >= len) return -1;
  size_t lim = maxs > 0 ? (size_t)maxs - 1 : (size_t)-1, n = 0;
  while (*off < len && n < lim) {
    char ch = text[(*off)++];
    if (n + 2 > *cap) {
      *cap = *cap * 2 + 256;
      char *nb = (char *)realloc(*buf, *cap);
      if (!nb) return -2;
      *buf = nb;
    }
    (*buf)[n++] = ch;
    if (ch == '\n') break;
  }
  (*buf)[n] = '\0';
  return (long)n;
}

SR_API void sr_free_dataset(sr_dataset *ds)
{
  if (!ds) return;
  free(ds->X);
  free(ds->hard);
  memset(ds, 0, sizeof(*ds));
}

SR_API int sr_parse_dataset(const char *text, size_t len, int32_t maxs, sr_dataset *out)
{
  if (!text || !out) return SR_EINVAL;
  memset(out, 0, sizeof(*out));
  size_t off = 0, cap = 256;
  char *s = (char *)malloc(cap);
  if (!s) return SR_ENOMEM;
  long got = next_line(text, len, &off, maxs, &s, &cap);
  if (got < 0) { free(s); return got == -2 ? SR_ENOMEM : SR_EPARSE; }
  int n, m;
  if (sscanf(s, "%d %d", &n, &m) != 2 || n <= 0 || m <= 0) { free(s); return SR_EHEADER; }
  out->N = n; out->M = m; out->nh = 0;
  out->X = (uint8_t *)calloc((size_t)n * m, 1);
  out->hard = (uint8_t *)calloc((size_t)n, 1);
  if (!out->X || !out->hard) { free(s); sr_free_dataset(out); return SR_ENOMEM; }
  for (int i = 0; i < n; i++) {
    got = next_line(text, len, &off, maxs, &s, &cap);
    if (got < 0) { free(s); sr_free_dataset(out); return got == -2 ? SR_ENOMEM : SR_EPARSE; }
    int k = 0;
    for (int j = 0; j < m; j++) {
      while (s[k] != '0' && s[k] != '1' && s[k] != '\0') k++;
      if (s[k] == '0') { out->X[(size_t)i * m + j] = 0; k++; }
      else if (s[k] == '1') { out->X[(size_t)i * m + j] = 1; k++; }
    }
    while (s[k] != '*' && s[k] != '\0') k++;
    if (s[k] == '*') { out->hard[i] = 1; out->nh++; }
  }
  free(s);
  return SR_OK;
}

/* ---- binary bit-packed datasets ----
 * "SRBX", u32 version 1, i32 N, i32 M, N hard-flag bytes, then N rows of (M + 7) / 8 bytes with
 * X[n][m] = bit (m & 7) of byte m >> 3 (little-endian host).  32x smaller than the reference's
 * text and no line limit; sr_load_dataset recognises it by the magic. */
static const char SRB_MAGIC[4] = {'S', 'R', 'B', 'X'};

SR_API int sr_save_dataset_bin(const sr_dataset *ds, const char *path)
{
  if (!ds || !path || ds->N < 1 || ds->M < 1 || !ds->X || !ds->hard) return SR_EINVAL;
  FILE *f = fopen(path, "wb");
  if (!f) return SR_EIO;
  const int32_t hdr[3] = {1, ds->N, ds->M};
  const size_t rb = ((size_t)ds->M + 7) / 8;
  uint8_t *row = (uint8_t *)calloc(rb, 1);
  int ok = row && fwrite(SRB_MAGIC, 1, 4, f) == 4 && fwrite(hdr, 4, 3, f) == 3 &&
           fwrite(ds->hard, 1, (size_t)ds->N, f) == (size_t)ds->N;
  for (int n = 0; ok && n < ds->N; n++) {
    memset(row, 0, rb);
    for (int m = 0; m < ds->M; m++)
      if (ds->X[(size_t)n * ds->M + m]) row[m >> 3] |= (uint8_t)(1u << (m & 7));
    ok = fwrite(row, 1, rb, f) == rb;
  }
  free(row);
  if (fclose(f) != 0) ok = 0;
  return ok ? SR_OK : SR_EIO;
}

static int load_bin(FILE *f, sr_dataset *out)
{
  int32_t hdr[3];
  if (fread(hdr, 4, 3, f) != 3 || hdr[0] != 1 || hdr[1] < 1 || hdr[2] < 1 || hdr[1] > (1 << 20) || hdr[2] > (1 << 20))
    return SR_EHEADER;
  const int N = hdr[1], M = hdr[2];
  const size_t rb = ((size_t)M + 7) / 8;
  out->N = N; out->M = M; out->nh = 0;
  out->X = (uint8_t *)malloc((size_t)N * M);
  out->hard = (uint8_t *)malloc((size_t)N);
  uint8_t *row = (uint8_t *)malloc(rb);
  if (!out->X || !out->hard || !row) { free(row); sr_free_dataset(out); return SR_ENOMEM; }
  int rc = SR_OK;
  if (fread(out->hard, 1, (size_t)N, f) != (size_t)N) rc = SR_EPARSE;
  for (int n = 0; rc == SR_OK && n < N; n++) {
    if (fread(row, 1, rb, f) != rb) { rc = SR_EPARSE; break; }
    for (int m = 0; m < M; m++) out->X[(size_t)n * M + m] = (row[m >> 3] >> (m & 7)) & 1u;
  }
  free(row);
  if (rc) { sr_free_dataset(out); return rc; }
  for (int n = 0; n < N; n++) { out->hard[n] = out->hard[n] ? 1 : 0; out->nh += out->hard[n]; }
  return SR_OK;
}

SR_API int sr_load_dataset_bin(const char *path, sr_dataset *out)
{
  if (!path || !out) return SR_EINVAL;
  memset(out, 0, sizeof *out);
  FILE *f = fopen(path, "rb");
  if (!f) return SR_EIO;
  char mg[4];
  int rc = (fread(mg, 1, 4, f) == 4 && memcmp(mg, SRB_MAGIC, 4) == 0) ? load_bin(f, out) : SR_EHEADER;
  fclose(f);
  return rc;
}

SR_API int sr_load_dataset(const char *path, int32_t maxs, sr_dataset *out)
{
  FILE *f = fopen(path, "rb");
  if (!f) return SR_EIO;
  {
    char mg[4];
    if (fread(mg, 1, 4, f) == 4 && memcmp(mg, SRB_MAGIC, 4) == 0) {
      memset(out, 0, sizeof *out);
      int rc = load_bin(f, out);
      fclose(f);
      return rc;
    }
    rewind(f);
  }
  size_t cap = 1 << 16, len = 0, got;
  char *t = (char *)malloc(cap);
  if (!t) { fclose(f); return SR_ENOMEM; }
  while ((got = fread(t + len, 1, cap - len, f)) > 0) {
    len += got;
    if (len == cap) {
      cap *= 2;
      char *nt = (char *)realloc(t, cap);
      if (!nt) { free(t); fclose(f); return SR_ENOMEM; }
      t = nt;
    }
  }
  fclose(f);
  int rc = sr_parse_dataset(t, len, maxs, out);
  free(t);
  return rc;
}

SR_API void sr_default_opts(sr_run_opts *o)
{
  memset(o, 0, sizeof(*o));
  o->burnin_calls = 1000;
  o->sample_calls = 1000;
  o->sweeps_per_call = 10;
}

/* ------------------------------------------------------------ chain init */
typedef struct {
  int N, M, nh;
  const uint8_t *X, *hard;
  int32_t *pi, *rpi, *a, *b, *t0, *f0, *t1, *f1;
  int t0a, f0a, t1a, f1a;
  double c, d, loglik;
  const double *cv;         /* manycd: per-taxon c[M], d[M] (mcmc.h:38-39 vectors), else NULL: c, d shared */
  int diag;                 /* SR_F_DIAG: the reference's stderr diagnostics */
} hmodel;

static void h_initab(hmodel *x)                       /* mcmc_initab, mcmc.c:440-474 */
{
  for (int m = 0; m < x->M; m++) {
    int n = 0;
    while (n < x->N && !x->X[(size_t)x->rpi[n] * x->M + m]) n++;
    if (n == x->N) {
      if (x->diag) fprintf(stderr, "mcmc_initab: zero column at %d, continuing.\n", m);   /* mcmc.c:457 */
      x->a[m] = 0; x->b[m] = x->N;
    }
    else {
      x->a[m] = n;
      n = x->N - 1;
      while (n >= 0 && !x->X[(size_t)x->rpi[n] * x->M + m]) n--;
      x->b[m] = n + 1;
    }
  }
}

static void h_count01(hmodel *x)                      /* mcmc_count01, mcmc.c:651-708 */
{
  x->t0a = x->f0a = x->t1a = x->f1a = 0;
  for (int m = 0; m < x->M; m++) {
    int t0 = 0, f0 = 0, t1 = 0, f1 = 0;
    for (int n = 0; n < x->N; n++) {
      int v = x->X[(size_t)n * x->M + m];
      if (x->a[m] <= x->pi[n] && x->pi[n] < x->b[m]) { if (v) t1++; else f0++; }
      else { if (v) f1++; else t0++; }
    }
    x->t0a += t0; x->f0a += f0; x->t1a += t1; x->f1a += f1;
    x->t0[m] = t0; x->f0[m] = f0; x->t1[m] = t1; x->f1[m] = f1;
  }
}

static double h_logl(const hmodel *x)                 /* mcmc_logl, mcmc.c:625-648 */
{
  double loglik = 0.;
  for (int m = 0; m < x->M; m++) {
    const double c = x->cv ? x->cv[m] : x->c, d = x->cv ? x->cv[x->M + m] : x->d;   /* mcmc.c:641-642 */
    loglik += x->t0[m] * h_log(1. - h_exp(c)) + x->f0[m] * d + x->t1[m] * h_log(1. - h_exp(d)) + x->f1[m] * c;
  }
  return loglik;
}

/* mcmc_randomize (mcmc.c:477-578); the read of q[nh] past the end (:530) is guarded */
static int h_randomize(hmodel *x, sr_hrng *r)
{
  const int N = x->N, nh = x->nh;
  if (nh == 0) {
    sr_hrng_shuffle(r, x->pi, (size_t)N);
    for (int i = 0; i < N; i++) x->rpi[x->pi[i]] = i;
    h_count01(x);
    x->loglik = h_logl(x);
    return 0;
  } else if (nh == N) {
    return 0;
  }
  int32_t *p = (int32_t *)malloc(N * sizeof(int32_t)), *q = (int32_t *)malloc(nh * sizeof(int32_t));
  if (!p || !q) { free(p); free(q); return SR_ENOMEM; }
  for (int i = 0; i < N; i++) p[i] = i;
  sr_hrng_choose(r, q, (size_t)nh, p, (size_t)N);
  int j = 0, k = 0;
  for (int i = 0; i < N; i++) {
    if (j < nh && i == q[j]) j++;
    else p[k++] = i;
  }
  sr_hrng_shuffle(r, p, (size_t)(N - nh));
  j = k = 0;
  for (int i = 0; i < N; i++) x->pi[i] = x->hard[i] ? q[j++] : p[k++];
  for (int i = 0; i < N; i++) x->rpi[x->pi[i]] = i;
  free(p); free(q);
  h_initab(x);
  h_count01(x);
  x->loglik = h_logl(x);
  return 0;
}

static void hmodel_free(hmodel *x)
{
  free(x->pi); free(x->rpi); free(x->a); free(x->b);
  free(x->t0); free(x->f0); free(x->t1); free(x->f1);
}

static int hmodel_alloc(hmodel *x, const sr_dataset *ds)
{
  memset(x, 0, sizeof(*x));
  x->N = ds->N; x->M = ds->M; x->nh = ds->nh; x->X = ds->X; x->hard = ds->hard;
  x->pi = (int32_t *)malloc(ds->N * 4); x->rpi = (int32_t *)malloc(ds->N * 4);
  x->a = (int32_t *)malloc(ds->M * 4); x->b = (int32_t *)malloc(ds->M * 4);
  x->t0 = (int32_t *)malloc(ds->M * 4); x->f0 = (int32_t *)malloc(ds->M * 4);
  x->t1 = (int32_t *)malloc(ds->M * 4); x->f1 = (int32_t *)malloc(ds->M * 4);
  if (!x->pi || !x->rpi || !x->a || !x->b || !x->t0 || !x->f0 || !x->t1 || !x->f1) { hmodel_free(x); return SR_ENOMEM; }
  return SR_OK;
}

/* ---------------------------------------------------------------- sessions */
struct sr_session {
  sr_dataset ds;            /* private copy */
  int nchains;
  sr_chain_spec *specs;
  sr_run_opts opts;
  srk_dev *dev;
  int rec_cap, nrec;
  long debug_calls;         /* mcmc_sample calls checked by SR_F_DEBUG_CHECK in this session */
  uint64_t *acc0;           /* SR_F_DEBUG_CHECK: acceptance counters at session creation (a restored
                               state carries its counters over; the rates cover this session's calls) */
  uint8_t *dbg_bad;         /* SR_F_DEBUG_CHECK: chain failed mcmc_consistent after some call (sticky) */
};

static void state_free(sr_state_host *st)
{
  free(st->P); free(st->rpi); free(st->hp); free(st->ab); free(st->cnt);
  free(st->cdl); free(st->mt); free(st->rng); free(st->acc); free(st->cdv);
  memset(st, 0, sizeof(*st));
}

static int state_alloc(sr_state_host *st, int N, int M, int nh, int C, int manycd)
{
  memset(st, 0, sizeof(*st));
  st->N = N; st->M = M; st->NW = (N + 31) / 32; st->nh = nh; st->nchains = C; st->manycd = manycd != 0;
  if (st->manycd && !(st->cdv = (double *)calloc((size_t)C * 2 * M, 8))) return SR_ENOMEM;
  st->P = (uint32_t *)calloc((size_t)C * st->NW * M, 4);
  st->rpi = (int32_t *)calloc((size_t)C * N, 4);
  st->hp = (int32_t *)calloc((size_t)C * SR_NHCAP(nh), 4);
  st->ab = (int32_t *)calloc((size_t)C * 2 * M, 4);
  st->cnt = (int32_t *)calloc((size_t)C * 4 * M, 4);
  st->cdl = (double *)calloc((size_t)C * 4, 8);
  st->mt = (uint32_t *)calloc((size_t)C * SR_RING * SR_MT_N, 4);
  st->rng = (uint64_t *)calloc((size_t)C * 2, 8);
  st->acc = (uint64_t *)calloc((size_t)C * SR_NACC, 8);
  if (!st->P || !st->rpi || !st->hp || !st->ab || !st->cnt || !st->cdl || !st->mt || !st->rng || !st->acc) {
    state_free(st);
    return SR_ENOMEM;
  }
  return SR_OK;
}

/* initialise one chain exactly as main() does before the burn-in (mcmc.c:127-135) */
static int init_chain(const sr_dataset *ds, uint64_t seed, sr_state_host *st, int c, int diag)
{
  hmodel x;
  int rc = hmodel_alloc(&x, ds);
  if (rc) return rc;
  x.diag = diag;
  const int N = ds->N, M = ds->M, NW = st->NW;
  for (int i = 0; i < N; i++) x.pi[i] = x.rpi[i] = i;      /* mcmc.c:405-407 */
  h_initab(&x);
  x.c = h_log(.01);                                           /* mcmc.c:417-421 */
  x.d = h_log(.3);
  h_count01(&x);
  x.loglik = h_logl(&x);
  sr_hrng r;
  sr_hrng_seed(&r, (unsigned long)seed);
  rc = h_randomize(&x, &r);
  if (rc) { hmodel_free(&x); return rc; }
  /* device state */
  uint32_t *P = st->P + (size_t)c * NW * M;
  for (int p = 0; p < N; p++) {
    const uint8_t *row = ds->X + (size_t)x.rpi[p] * M;
    for (int m = 0; m < M; m++)
      if (row[m]) P[(size_t)(p >> 5) * M + m] |= 1u << (p & 31);
  }
  memcpy(st->rpi + (size_t)c * N, x.rpi, N * 4);
  int k = 0;
  for (int s = 0; s < N; s++)
    if (ds->hard[s]) st->hp[(size_t)c * SR_NHCAP(ds->nh) + k++] = x.pi[s];
  memcpy(st->ab + (size_t)c * 2 * M, x.a, M * 4);
  memcpy(st->ab + (size_t)c * 2 * M + M, x.b, M * 4);
  memcpy(st->cnt + (size_t)c * 4 * M, x.t0, M * 4);
  memcpy(st->cnt + (size_t)c * 4 * M + M, x.f0, M * 4);
  memcpy(st->cnt + (size_t)c * 4 * M + 2 * M, x.t1, M * 4);
  memcpy(st->cnt + (size_t)c * 4 * M + 3 * M, x.f1, M * 4);
  st->cdl[(size_t)c * 4 + 0] = x.c;
  st->cdl[(size_t)c * 4 + 1] = x.d;
  st->cdl[(size_t)c * 4 + 2] = x.loglik;
  if (st->manycd)   /* every taxon starts at log .01 / log .3 (mcmc.c:417-421): the same loglik */
    for (int m = 0; m < M; m++) { st->cdv[(size_t)c * 2 * M + m] = x.c; st->cdv[(size_t)c * 2 * M + M + m] = x.d; }
  memcpy(st->mt + ((size_t)c * SR_RING + (r.bidx % SR_RING)) * SR_MT_N, r.blk, sizeof(r.blk));
  st->rng[(size_t)c * 2 + 0] = r.pos;
  st->rng[(size_t)c * 2 + 1] = r.bidx + 1;
  hmodel_free(&x);
  return SR_OK;
}

/* The chains' initialisation (mcmc_readmodel's state, initab, randomize, count01, logl and the position-ordered bit
   columns: O(N M) per chain, ~20 ms at 1024 x 2048) on several host threads: chains are independent (own RNG, own
   slice of st), so the state is the serial loop's bit for bit.  Threads: the CPUs this process may run on (its
   affinity mask, and OMP_NUM_THREADS when set), at most 32 and one per chain; SR_INIT_THREADS overrides; serial
   when the initab notes go to stderr (their order is the reference's) or for one chain. */
typedef struct {
  const sr_dataset *ds;
  const sr_chain_spec *specs;
  sr_state_host *st;
  int n, diag, next, rc;
  pthread_mutex_t mu;
} init_work;

static void *init_main(void *arg)
{
  init_work *w = (init_work *)arg;
  for (;;) {
    pthread_mutex_lock(&w->mu);
    const int c = (w->rc == SR_OK && w->next < w->n) ? w->next++ : -1;
    pthread_mutex_unlock(&w->mu);
    if (c < 0) return NULL;
    const int rc = init_chain(w->ds, w->specs[c].seed, w->st, c, w->diag);
    if (rc) {
      pthread_mutex_lock(&w->mu);
      if (w->rc == SR_OK) w->rc = rc;
      pthread_mutex_unlock(&w->mu);
    }
  }
}

static int init_chains(const sr_dataset *ds, const sr_chain_spec *specs, int n, sr_state_host *st, int diag)
{
  int nt = 1;
  cpu_set_t cs;
  if (sched_getaffinity(0, sizeof cs, &cs) == 0) nt = CPU_COUNT(&cs);
  const char *omp = getenv("OMP_NUM_THREADS");   /* a launcher's thread budget (the GPU box's CPU share) */
  if (omp && atoi(omp) > 0 && atoi(omp) < nt) nt = atoi(omp);
  const char *e = getenv("SR_INIT_THREADS");
  if (e && atoi(e) > 0) nt = atoi(e);
  if (nt > 32) nt = 32;
  if (nt > n) nt = n;
  if (diag || nt <= 1) {
    for (int c = 0; c < n; c++) {
      const int rc = init_chain(ds, specs[c].seed, st, c, diag);
      if (rc) return rc;
    }
    return SR_OK;
  }
  init_work w = {ds, specs, st, n, diag, 0, SR_OK, PTHREAD_MUTEX_INITIALIZER};
  pthread_t th[32];
  int started = 0;
  for (; started < nt - 1; started++)
    if (pthread_create(&th[started], NULL, init_main, &w) != 0) break;
  init_main(&w);   /* this thread works too (and alone if no thread could be started) */
  for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
  return w.rc;
}

static int auto_calls_per_launch(const sr_run_opts *o)
{
  return o->calls_per_launch > 0 ? o->calls_per_launch : 100;
}

/* The shape-specialised sweep kernel is the default (sr_spec.c; identical results); SR_F_GENERIC_KERNEL or
   SR_JIT=0 in the environment select the generic one. */
static int sr_want_specialized(const sr_run_opts *o)
{
  if (o->flags & SR_F_GENERIC_KERNEL) return 0;
  const char *e = getenv("SR_JIT");
  return !(e && e[0] == '0' && e[1] == 0);
}

/* A session over `ds`: every chain initialised as main() does (restore == NULL), or its state
   filled by restore(ctx, st) (a checkpoint). */
static int session_new(const sr_dataset *ds, const sr_chain_spec *specs, int32_t n_chains, const sr_run_opts *opts,
                       int (*restore)(void *, sr_state_host *), void *restore_ctx, sr_session **out)
{
  if (!ds || !specs || n_chains <= 0 || !out || ds->N < 2 || ds->M < 1) return SR_EINVAL;
  sr_run_opts o;
  if (opts) o = *opts; else sr_default_opts(&o);
  if (o.sweeps_per_call <= 0) return SR_EINVAL;
  o.manycd = o.manycd != 0;   /* mcmc_readmodel stores the flag; any nonzero value means per-taxon c, d */
  /* nh <= 64 hard sites (a 64-bit mask per taxon), N <= 4095 (12-bit positions in the packed proposal
     records, int16 a, b, pi records), M <= SR_MMAX taxa (several per thread beyond the block; the records hold
     positions only).  The LDS layout must also fit 160 KB (srk_create), else HBM columns. */
  if (ds->N > 4095 || ds->M > SR_MMAX) return SR_EUNSUPPORTED;
  /* the environment names another GSL generator (mcmc.c:591-592): a session that samples MT19937's stream is
     refused; an opt-in Philox session (SR_F_RNG_PHILOX) samples no GSL stream and ignores the variable */
  if (!(o.flags & SR_F_RNG_PHILOX)) {
    const int rt = rng_type_check(0);
    if (rt) return rt;
  }
  sr_session *s = (sr_session *)calloc(1, sizeof(*s));
  if (!s) return SR_ENOMEM;
  s->ds.N = ds->N; s->ds.M = ds->M; s->ds.nh = ds->nh;
  s->ds.X = (uint8_t *)malloc((size_t)ds->N * ds->M);
  s->ds.hard = (uint8_t *)malloc((size_t)ds->N);
  s->specs = (sr_chain_spec *)malloc(sizeof(sr_chain_spec) * n_chains);
  if (!s->ds.X || !s->ds.hard || !s->specs) { sr_free_dataset(&s->ds); free(s->specs); free(s); return SR_ENOMEM; }
  memcpy(s->ds.X, ds->X, (size_t)ds->N * ds->M);
  memcpy(s->ds.hard, ds->hard, (size_t)ds->N);
  memcpy(s->specs, specs, sizeof(sr_chain_spec) * n_chains);
  s->nchains = n_chains;
  s->opts = o;
  sr_state_host st;
  int rc = state_alloc(&st, ds->N, ds->M, ds->nh, n_chains, o.manycd);
  if (rc) { sr_session_destroy(s); return rc; }
  const int philox = (o.flags & SR_F_RNG_PHILOX) != 0;
  if (restore) rc = restore(restore_ctx, &st);
  else {
    rc = init_chains(ds, specs, n_chains, &st, (o.flags & SR_F_DIAG) != 0);
    for (int c = 0; c < n_chains && rc == SR_OK && philox; c++) {
      /* sampling draws from the chain's Philox stream, word 0 on (init stays GSL MT19937) */
      st.rng[(size_t)c * 2 + 0] = 0;
      st.rng[(size_t)c * 2 + 1] = 0;
      st.cdl[(size_t)c * 4 + 3] = 1.0;   /* the stream kind travels with the state (checkpoints) */
    }
  }
  /* a restored state keeps its stream: the caller's flag must name the same one */
  for (int c = 0; c < n_chains && rc == SR_OK; c++)
    if ((st.cdl[(size_t)c * 4 + 3] == 1.0) != philox) rc = SR_EINVAL;
  uint32_t *pkey = NULL;
  if (rc == SR_OK && philox) {
    pkey = (uint32_t *)malloc(sizeof(uint32_t) * 2 * n_chains);
    if (!pkey) rc = SR_ENOMEM;
    for (int c = 0; c < n_chains && pkey; c++) sr_philox_key(specs[c].seed, pkey + 2 * c);
  }
  if (rc) { state_free(&st); sr_session_destroy(s); return rc; }
  if (o.flags & SR_F_DEBUG_CHECK) {
    s->acc0 = (uint64_t *)malloc(sizeof(uint64_t) * SR_NACC * n_chains);
    s->dbg_bad = (uint8_t *)calloc(n_chains, 1);
    if (!s->acc0 || !s->dbg_bad) { state_free(&st); free(pkey); sr_session_destroy(s); return SR_ENOMEM; }
    memcpy(s->acc0, st.acc, sizeof(uint64_t) * SR_NACC * n_chains);
  }
  s->rec_cap = auto_calls_per_launch(&o);
  const int gm_force = (o.flags & SR_F_HBM_COLUMNS) ? 1 : ((o.flags & SR_F_LDS_COLUMNS) ? 0 : -1);
  rc = srk_create(&st, o.device, o.block_threads, s->rec_cap, gm_force, pkey, sr_want_specialized(&o), &s->dev);
  free(pkey);
  state_free(&st);
  if (rc) { sr_session_destroy(s); return rc == -6 ? SR_EUNSUPPORTED : SR_EDEVICE; }
  *out = s;
  return SR_OK;
}

SR_API int sr_session_create(const sr_dataset *ds, const sr_chain_spec *specs, int32_t n_chains,
                             const sr_run_opts *opts, sr_session **out)
{
  return session_new(ds, specs, n_chains, opts, NULL, NULL, out);
}

SR_API int sr_session_set_stream(sr_session *s, void *hip_stream)
{
  if (!s) return SR_EINVAL;
  return srk_set_stream(s->dev, hip_stream) ? SR_EDEVICE : SR_OK;
}

static int download(sr_session *s, sr_state_host *st);
static int check_chain(const sr_dataset *ds, const sr_state_host *st, int c);

/* SR_F_DEBUG_CHECK after one mcmc_sample call of every chain: the reference's MCMCDEBUG block
 * (mcmc.c:249-255) -- the running acceptance rates on stderr (counters and calls of this session,
 * as its static ones count the process's calls; sweeps_per_call sweeps per call where the
 * reference hard-codes 10; one line per chain in chain order) and mcmc_consistent on the
 * downloaded state.  Like the reference (which ignores that check's result there and runs on), a
 * failing chain does not stop the run: it is flagged (dbg_bad, sticky) and SR_EINCONSISTENT
 * returned after every chain was checked. */
static int debug_check(sr_session *s)
{
  sr_state_host st;
  int rc = download(s, &st);
  if (rc) return rc;
  s->debug_calls++;
  const double n = (double)s->debug_calls, M = (double)s->ds.M, spc = (double)s->opts.sweeps_per_call;
  for (int c = 0; c < s->nchains; c++) {
    const uint64_t *a = st.acc + (size_t)c * SR_NACC, *a0 = s->acc0 + (size_t)c * SR_NACC;
    double r[7];
    for (int k = 0; k < 7; k++) r[k] = (double)(a[k] - a0[k]);
    if (s->opts.flags & SR_F_DEBUG_PRINT)
      fprintf(stderr, "mcmc_sample: %f %f %f %f %f %f %f\n", r[0] / (spc * n), r[1] / (spc * n), r[2] / (2. * spc * n * M),
              r[3] / (spc * 5 * n), r[4] / (spc * 5 * n), r[5] / (spc * 5 * n), r[6] / (spc * 5 * n));
    if (check_chain(&s->ds, &st, c)) { s->dbg_bad[c] = 1; rc = SR_EINCONSISTENT; }
  }
  state_free(&st);
  return rc;
}

SR_API int sr_session_run(sr_session *s, int32_t calls, int32_t save)
{
  if (!s || calls < 0) return SR_EINVAL;
  if (save && s->nrec + calls > s->rec_cap) return SR_EINVAL;
  const int dbg = (s->opts.flags & SR_F_DEBUG_CHECK) != 0;
  int bad = 0;
  for (int done = 0; done < calls;) {   /* debug: one call per launch, each followed by the check */
    const int k = dbg ? 1 : calls;
    int rc = srk_run(s->dev, k, s->opts.sweeps_per_call, save ? 1 : 0, s->nrec);
    if (rc) return rc == -1 ? SR_EINVAL : SR_EDEVICE;
    if (save) s->nrec += k;
    done += k;
    if (dbg && (rc = debug_check(s))) {
      if (rc != SR_EINCONSISTENT) return rc;
      bad = 1;   /* flagged; the calls still run (mcmc.c:254 ignores the check's result) */
    }
  }
  return bad ? SR_EINCONSISTENT : SR_OK;
}

SR_API int sr_session_debug_flagged(const sr_session *s, int32_t chain)
{
  if (!s || chain < 0 || chain >= s->nchains) return SR_EINVAL;
  return (s->dbg_bad && s->dbg_bad[chain]) ? 1 : 0;
}

SR_API int sr_session_sync(sr_session *s) { return (!s) ? SR_EINVAL : (srk_sync(s->dev) ? SR_EDEVICE : SR_OK); }
SR_API int32_t sr_session_records(const sr_session *s) { return s ? s->nrec : 0; }
SR_API int32_t sr_session_record_capacity(const sr_session *s) { return s ? s->rec_cap : 0; }
SR_API int32_t sr_session_block_threads(const sr_session *s) { return s ? srk_block_threads(s->dev) : 0; }
SR_API int32_t sr_session_variant(const sr_session *s) { return s ? srk_variant(s->dev) : -1; }
SR_API int32_t sr_session_specialized(const sr_session *s) { return s ? srk_specialized(s->dev) != 0 : 0; }
/* test hook: 1 when the session's specialised code object is the one embedded in the library (no compiler,
   no cache at run time), 0 otherwise */
SR_API int32_t sr_session_spec_embedded(const sr_session *s) { return s ? srk_specialized(s->dev) == 2 : 0; }
/* test hook: 1 when the library embeds the specialised code object a session of this shape would run */
SR_API int sr_spec_is_embedded(int N, int M, int nh, int block_threads)
{
  sr_spec_shape sh;
  size_t bytes = 0;
  return srk_plan(N, M, nh, block_threads, -1, 0, &sh) == 1 && sr_spec_embedded(&sh, &bytes) != NULL && bytes > 0;
}
SR_API double sr_session_last_kernel_ms(sr_session *s) { return s ? srk_last_ms(s->dev) : -1.0; }

SR_API int sr_session_fetch_records(sr_session *s, int32_t first, int32_t count, int16_t *ab_pi, double *cdl)
{
  if (!s || first < 0 || count < 0 || first + count > s->nrec) return SR_EINVAL;
  return srk_fetch_records(s->dev, first, count, ab_pi, cdl) ? SR_EDEVICE : SR_OK;
}

SR_API int sr_session_fetch_chain_records(sr_session *s, int32_t chain, int32_t first, int32_t count, int16_t *ab_pi,
                                         double *cdl)
{
  if (!s || chain < 0 || chain >= s->nchains || first < 0 || count < 0 || first + count > s->nrec) return SR_EINVAL;
  return srk_fetch_chain_records(s->dev, chain, first, count, ab_pi, cdl) ? SR_EDEVICE : SR_OK;
}

SR_API int sr_session_copy_chain_records(sr_session *s, int32_t chain, int32_t first, int32_t count, int16_t *dev_ab_pi,
                                        double *dev_cdl)
{
  if (!s || chain < 0 || chain >= s->nchains || first < 0 || count < 0 || first + count > s->nrec) return SR_EINVAL;
  return srk_copy_chain_records(s->dev, chain, first, count, dev_ab_pi, dev_cdl) ? SR_EDEVICE : SR_OK;
}

SR_API int sr_session_fetch_cd_vectors(sr_session *s, int32_t first, int32_t count, double *cdv)
{
  if (!s || !cdv || first < 0 || count < 0 || first + count > s->nrec) return SR_EINVAL;
  if (!s->opts.manycd) return SR_EINVAL;
  return srk_fetch_cdv(s->dev, first, count, cdv) ? SR_EDEVICE : SR_OK;
}

SR_API int32_t sr_session_manycd(const sr_session *s) { return s ? s->opts.manycd : 0; }

/* compute_exp_data + print_exp_data (mcmc.c:53-67) over the buffered records [first, first + count)
 * of every chain: sums of -loglik, e^c, e^d in sample order (C library exp, as the reference),
 * divided by the reference's hard-coded 1000.  consistent is left 0 (no check is run). */
SR_API int sr_session_summaries(sr_session *s, int32_t first, int32_t count, sr_chain_summary *out)
{
  if (!s || !out || first < 0 || count < 0 || first + count > s->nrec) return SR_EINVAL;
  /* the sums on the device, in the reference's row order (srk_exp_data); only they are copied back */
  double *sm = (double *)calloc((size_t)3 * s->nchains, sizeof(double));
  if (!sm) return SR_ENOMEM;
  int rc = count ? srk_exp_data(s->dev, first, count, sm) : 0;
  if (rc) { free(sm); return SR_EDEVICE; }
  for (int c = 0; c < s->nchains; c++) {
    out[c].chain_id = s->specs[c].chain_id;
    out[c].consistent = 0;
    out[c].exp_loglik = sm[3 * c] / 1000;   /* print_exp_data divides by 1000 (mcmc.c:62-64) */
    out[c].exp_c = sm[3 * c + 1] / 1000;
    out[c].exp_d = sm[3 * c + 2] / 1000;
  }
  free(sm);
  return SR_OK;
}

SR_API int sr_session_reset_records(sr_session *s)
{
  if (!s) return SR_EINVAL;
  s->nrec = 0;
  return SR_OK;
}

static int download(sr_session *s, sr_state_host *st)
{
  int rc = state_alloc(st, s->ds.N, s->ds.M, s->ds.nh, s->nchains, s->opts.manycd);
  if (rc) return rc;
  if (srk_download_state(s->dev, st)) { state_free(st); return SR_EDEVICE; }
  return SR_OK;
}

/* ---- checkpoint / resume (the reference restarts every run; optional here) ----
 * File: "SRCK" | u32 version | i32 N, M, nh, nchains | u64 FNV-1a of the dataset (X, hard) | [v5-v8: i32 nrec]
 * | [v7, v8: i32 record capacity of the checkpointed session]
 * | sr_chain_spec[nchains] | the device state as sr_state_host arrays (P, rpi, hp, ab, cnt, cdl, mt, rng, acc;
 * manycd: cdv) | [v5-v8: the session's buffered records: ab_pi [nchains][nrec][2M+N] i16, cdl [nchains][nrec][3]
 * f64, manycd: cdv [nchains][nrec][2M] f64], little-endian.  A restore keeps at least the checkpointed session's
 * record capacity, so the saves that session could still make fit without the caller re-supplying
 * calls_per_launch.  Restoring uploads the same words, so the continued
 * chains are the ones an uninterrupted session produces, and summaries over the records (compute_exp_data,
 * mcmc.c:53-67) span the whole sampling phase across the interruption (tests/test_gpu_edge.py). */
static uint64_t dataset_hash(const sr_dataset *ds)
{
  uint64_t h = 1469598103934665603ULL;
  for (size_t k = 0; k < (size_t)ds->N * ds->M; k++) { h ^= ds->X[k]; h *= 1099511628211ULL; }
  for (int k = 0; k < ds->N; k++) { h ^= ds->hard[k]; h *= 1099511628211ULL; }
  return h;
}

typedef struct { size_t bytes; void *p; } ck_part;
#define SR_CK_VERSION 3   /* 2: SR_NACC counters per chain; 3: SR_NHMAX = 64 hard positions per chain */
#define SR_CK_VERSION_MANYCD 4   /* version 3 + the per-taxon c, d of every chain (manycd sessions) */
#define SR_CK_VERSION_REC 5      /* version 3 + the buffered records (written since round 5) */
#define SR_CK_VERSION_REC_MANYCD 6   /* version 4 + the buffered records */
#define SR_CK_VERSION_CAP 7      /* version 5 + the record capacity (written since round 6) */
#define SR_CK_VERSION_CAP_MANYCD 8   /* version 6 + the record capacity */
#define SR_CK_PARTS 10

static int ck_parts(sr_state_host *st, ck_part *pt)
{
  const size_t C = (size_t)st->nchains;
  ck_part q[SR_CK_PARTS] = {
    {C * st->NW * st->M * 4, st->P}, {C * st->N * 4, st->rpi}, {C * SR_NHCAP(st->nh) * 4, st->hp},
    {C * 2 * st->M * 4, st->ab}, {C * 4 * st->M * 4, st->cnt}, {C * 4 * 8, st->cdl},
    {C * SR_RING * SR_MT_N * 4, st->mt}, {C * 2 * 8, st->rng}, {C * SR_NACC * 8, st->acc},
    {C * 2 * st->M * 8, st->cdv}};
  memcpy(pt, q, sizeof q);
  return st->manycd ? 10 : 9;
}

typedef struct { int32_t nrec, cap; int16_t *ab; double *cdl, *cdv; } ck_records;

static int ck_write(const char *path, const sr_dataset *ds, const sr_chain_spec *specs, int32_t n, sr_state_host *st,
                    const ck_records *rec)
{
  FILE *f = fopen(path, "wb");
  if (!f) return SR_EIO;
  const uint32_t ver = st->manycd ? SR_CK_VERSION_CAP_MANYCD : SR_CK_VERSION_CAP;
  const int32_t dims[4] = {ds->N, ds->M, ds->nh, n};
  const uint64_t h = dataset_hash(ds);
  const int32_t nrec = rec ? rec->nrec : 0, cap = rec ? rec->cap : 0;
  int ok = fwrite("SRCK", 1, 4, f) == 4 && fwrite(&ver, 4, 1, f) == 1 && fwrite(dims, 4, 4, f) == 4 &&
           fwrite(&h, 8, 1, f) == 1 && fwrite(&nrec, 4, 1, f) == 1 && fwrite(&cap, 4, 1, f) == 1 &&
           fwrite(specs, sizeof(sr_chain_spec), n, f) == (size_t)n;
  ck_part pt[SR_CK_PARTS];
  const int np = ck_parts(st, pt);
  for (int k = 0; k < np && ok; k++) ok = fwrite(pt[k].p, 1, pt[k].bytes, f) == pt[k].bytes;
  if (ok && nrec > 0) {
    const size_t rows = (size_t)n * nrec, W = 2 * (size_t)ds->M + ds->N;
    ok = fwrite(rec->ab, 2 * W, rows, f) == rows && fwrite(rec->cdl, 24, rows, f) == rows &&
         (!st->manycd || fwrite(rec->cdv, 16 * (size_t)ds->M, rows, f) == rows);
  }
  if (fclose(f) != 0) ok = 0;
  return ok ? SR_OK : SR_EIO;
}

SR_API int sr_session_checkpoint(sr_session *s, const char *path)
{
  if (!s || !path) return SR_EINVAL;
  sr_state_host st;
  int rc = download(s, &st);
  if (rc) return rc;
  ck_records r = {s->nrec, s->rec_cap, NULL, NULL, NULL};
  if (r.nrec > 0) {   /* the buffered records travel with the state (v5 / v6) */
    const size_t rows = (size_t)s->nchains * r.nrec, W = 2 * (size_t)s->ds.M + s->ds.N;
    r.ab = (int16_t *)malloc(rows * W * 2);
    r.cdl = (double *)malloc(rows * 24);
    r.cdv = s->opts.manycd ? (double *)malloc(rows * 16 * (size_t)s->ds.M) : NULL;
    if (!r.ab || !r.cdl || (s->opts.manycd && !r.cdv)) rc = SR_ENOMEM;
    else if (srk_fetch_records(s->dev, 0, r.nrec, r.ab, r.cdl) || (r.cdv && srk_fetch_cdv(s->dev, 0, r.nrec, r.cdv)))
      rc = SR_EDEVICE;
  }
  if (!rc) rc = ck_write(path, &s->ds, s->specs, s->nchains, &st, &r);
  free(r.ab); free(r.cdl); free(r.cdv);
  state_free(&st);
  return rc;
}

/* test hook: a checkpoint of freshly initialised chains (main()'s initial state), written on
   the host without a device (restore validation tests) */
SR_API int sr_host_initial_checkpoint(const sr_dataset *ds, const sr_chain_spec *specs, int32_t n_chains, const char *path)
{
  if (!ds || !specs || n_chains <= 0 || !path) return SR_EINVAL;
  sr_state_host st;
  int rc = state_alloc(&st, ds->N, ds->M, ds->nh, n_chains, 0);
  if (rc) return rc;
  rc = init_chains(ds, specs, n_chains, &st, 0);
  if (rc == SR_OK) rc = ck_write(path, ds, specs, n_chains, &st, NULL);
  state_free(&st);
  return rc;
}

typedef struct { FILE *f; const sr_dataset *ds; int records; } ck_reader;

static int check_chain(const sr_dataset *ds, const sr_state_host *st, int c);

/* A restored state is uploaded into kernels that use hp and the RNG cursor as LDS indices and
 * a, b, pi as positions: every chain must pass the mcmc_consistent port (limits, permutation,
 * hard-site order, counts, loglik, P == X in position order), its hard positions must be the
 * ascending positions of the hard sites, and its RNG cursor must lie inside the generated ring. */
static int ck_validate(const sr_dataset *ds, const sr_state_host *st)
{
  const int N = ds->N, nh = ds->nh;
  for (int c = 0; c < st->nchains; c++) {
    if (check_chain(ds, st, c)) return SR_EPARSE;
    const int32_t *hp = st->hp + (size_t)c * SR_NHCAP(nh), *rpi = st->rpi + (size_t)c * N;
    for (int k = 0; k < nh; k++)
      if (hp[k] < 0 || hp[k] >= N || (k > 0 && hp[k] <= hp[k - 1]) || !ds->hard[rpi[hp[k]]]) return SR_EPARSE;
    const uint64_t pos = st->rng[(size_t)c * 2 + 0], gen = st->rng[(size_t)c * 2 + 1];
    const uint64_t blk = pos / SR_MT_N;
    const double kind = st->cdl[(size_t)c * 4 + 3];   /* 0 MT19937 (a seeded block exists), 1 Philox */
    if ((kind != 0.0 && kind != 1.0) || (kind == 0.0 && gen < 1) || blk > gen || gen - blk > SR_RING || gen > 0xffffffffULL)
      return SR_EPARSE;
  }
  return SR_OK;
}

static int ck_restore(void *ctx, sr_state_host *st)
{
  ck_reader *r = (ck_reader *)ctx;
  ck_part pt[SR_CK_PARTS];
  const int np = ck_parts(st, pt);
  for (int k = 0; k < np; k++)
    if (fread(pt[k].p, 1, pt[k].bytes, r->f) != pt[k].bytes) return SR_EPARSE;
  if (!r->records && fgetc(r->f) != EOF) return SR_EPARSE;   /* (v5 / v6: the records follow) */
  return ck_validate(r->ds, st);
}

SR_API int sr_session_restore(const sr_dataset *ds, const char *path, const sr_run_opts *opts, sr_session **out)
{
  if (!ds || !path || !out) return SR_EINVAL;
  FILE *f = fopen(path, "rb");
  if (!f) return SR_EIO;
  char magic[4];
  uint32_t ver = 0;
  int32_t dims[4], nrec = 0, cap = 0;
  uint64_t h = 0;
  int rc = SR_OK;
  sr_chain_spec *specs = NULL;
  int16_t *rab = NULL;
  double *rcd = NULL, *rcv = NULL;
  if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "SRCK", 4) != 0 || fread(&ver, 4, 1, f) != 1 ||
      ver < SR_CK_VERSION || ver > SR_CK_VERSION_CAP_MANYCD ||
      fread(dims, 4, 4, f) != 4 || fread(&h, 8, 1, f) != 1 || dims[3] <= 0)
    rc = SR_EPARSE;
  const int with_rec = ver >= SR_CK_VERSION_REC, with_cap = ver >= SR_CK_VERSION_CAP;
  const int mcd = ver == SR_CK_VERSION_MANYCD || ver == SR_CK_VERSION_REC_MANYCD || ver == SR_CK_VERSION_CAP_MANYCD;
  if (rc == SR_OK && with_rec && (fread(&nrec, 4, 1, f) != 1 || nrec < 0)) rc = SR_EPARSE;
  if (rc == SR_OK && with_cap && (fread(&cap, 4, 1, f) != 1 || cap < nrec)) rc = SR_EPARSE;
  if (rc) { fclose(f); return rc; }
  if (dims[0] != ds->N || dims[1] != ds->M || dims[2] != ds->nh || h != dataset_hash(ds))
    rc = SR_EINVAL;   /* the checkpoint belongs to another dataset */
  else if (!(specs = (sr_chain_spec *)malloc(sizeof(sr_chain_spec) * dims[3])))
    rc = SR_ENOMEM;
  else if (fread(specs, sizeof(sr_chain_spec), dims[3], f) != (size_t)dims[3])
    rc = SR_EPARSE;
  if (rc == SR_OK) {   /* the checkpoint's kind (manycd or not) decides; a caller's opts naming the other is an error */
    sr_run_opts o;
    if (opts) o = *opts; else sr_default_opts(&o);
    if (opts && (o.manycd != 0) != mcd) rc = SR_EINVAL;
    o.manycd = mcd;
    /* the record buffer holds the checkpoint's records and the caller's further calls: at least the checkpointed
       session's capacity (v7 / v8), the caller's calls_per_launch, and the records themselves */
    const int want = cap > nrec ? cap : nrec;
    if (auto_calls_per_launch(&o) < want) o.calls_per_launch = want;
    ck_reader r = {f, ds, with_rec};
    if (rc == SR_OK) rc = session_new(ds, specs, dims[3], &o, ck_restore, &r, out);
  }
  if (rc == SR_OK && with_rec) {   /* the buffered records, uploaded into the new session's record buffer */
    const size_t rows = (size_t)dims[3] * nrec, W = 2 * (size_t)ds->M + ds->N;
    if (rows) {
      rab = (int16_t *)malloc(rows * W * 2);
      rcd = (double *)malloc(rows * 24);
      rcv = mcd ? (double *)malloc(rows * 16 * (size_t)ds->M) : NULL;
      if (!rab || !rcd || (mcd && !rcv)) rc = SR_ENOMEM;
      else if (fread(rab, 2 * W, rows, f) != rows || fread(rcd, 24, rows, f) != rows ||
               (mcd && fread(rcv, 16 * (size_t)ds->M, rows, f) != rows))
        rc = SR_EPARSE;
    }
    if (rc == SR_OK && fgetc(f) != EOF) rc = SR_EPARSE;
    if (rc == SR_OK && rows && srk_upload_records((*out)->dev, nrec, rab, rcd, rcv)) rc = SR_EDEVICE;
    if (rc == SR_OK) (*out)->nrec = nrec;
    else { sr_session_destroy(*out); *out = NULL; }
  }
  free(rab); free(rcd); free(rcv);
  free(specs);
  fclose(f);
  return rc;
}

SR_API int sr_session_state(sr_session *s, int32_t chain, int32_t *a, int32_t *b, int32_t *pi,
                            double *cdl3, int32_t *counts)
{
  if (!s || chain < 0 || chain >= s->nchains) return SR_EINVAL;
  sr_state_host st;
  int rc = download(s, &st);
  if (rc) return rc;
  const int N = s->ds.N, M = s->ds.M;
  if (a) memcpy(a, st.ab + (size_t)chain * 2 * M, M * 4);
  if (b) memcpy(b, st.ab + (size_t)chain * 2 * M + M, M * 4);
  if (pi) for (int n = 0; n < N; n++) pi[st.rpi[(size_t)chain * N + n]] = n;
  if (cdl3) memcpy(cdl3, st.cdl + (size_t)chain * 4, 3 * 8);
  if (counts) memcpy(counts, st.cnt + (size_t)chain * 4 * M, 4 * M * 4);
  state_free(&st);
  return SR_OK;
}

SR_API int sr_session_state_cd(sr_session *s, int32_t chain, double *c, double *d)
{
  if (!s || chain < 0 || chain >= s->nchains || !s->opts.manycd) return SR_EINVAL;
  sr_state_host st;
  int rc = download(s, &st);
  if (rc) return rc;
  const int M = s->ds.M;
  if (c) memcpy(c, st.cdv + (size_t)chain * 2 * M, (size_t)M * 8);
  if (d) memcpy(d, st.cdv + (size_t)chain * 2 * M + M, (size_t)M * 8);
  state_free(&st);
  return SR_OK;
}

SR_API int sr_session_accept_counts(sr_session *s, int32_t chain, int64_t *acc7)
{
  if (!s || chain < 0 || chain >= s->nchains || !acc7) return SR_EINVAL;
  sr_state_host st;
  int rc = download(s, &st);
  if (rc) return rc;
  for (int k = 0; k < 7; k++) acc7[k] = (int64_t)st.acc[(size_t)chain * SR_NACC + k];
  state_free(&st);
  return SR_OK;
}

SR_API int sr_session_fallback_counts(sr_session *s, int32_t chain, int64_t *fb3)
{
  if (!s || chain < 0 || chain >= s->nchains || !fb3) return SR_EINVAL;
  sr_state_host st;
  int rc = download(s, &st);
  if (rc) return rc;
  for (int k = 0; k < 3; k++) fb3[k] = (int64_t)st.acc[(size_t)chain * SR_NACC + 7 + k];
  state_free(&st);
  return SR_OK;
}

/* ---- posterior summaries on the GPU (script.py:155-189, 230-275, 306-417) ---- */
static const int post_kinds[6] = {SRP_PAIR_ORDER, SRP_ALIVE, SRP_FALSE_ALIVE, SRP_FALSE_ONES, SRP_EXP_PI, SRP_EXP_A};

static double *post_slot(sr_posterior_out *o, int k)
{
  switch (k) {
    case 0: return o->pair_order;
    case 1: return o->alive;
    case 2: return o->false_alive;
    case 3: return o->false_ones;
    case 4: return o->exp_pi;
    default: return o->exp_a;
  }
}

static int post_rc(int rc) { return rc == 0 ? SR_OK : (rc == -1 ? SR_EINVAL : (rc == -4 ? SR_ENOMEM : SR_EDEVICE)); }

SR_API int sr_posterior(const sr_dataset *ds, const int16_t *ab_pi, int32_t n_sel, int32_t count,
                        int32_t chains_selected, int32_t device, sr_posterior_out *out)
{
  if (!ds || !ab_pi || !out || n_sel <= 0 || count < 0 || chains_selected == 0) return SR_EINVAL;
  for (int k = 0; k < 6; k++) {
    double *dst = post_slot(out, k);
    if (!dst) continue;
    float ms = 0.0f;
    int rc = srp_posterior_host(device, post_kinds[k], ab_pi, n_sel, count, ds->N, ds->M, ds->X, chains_selected, dst, &ms);
    if (rc) return post_rc(rc);
    out->kernel_ms += ms;
  }
  return SR_OK;
}

SR_API int sr_session_posterior(sr_session *s, const int32_t *chains, int32_t n_sel, int32_t first, int32_t count,
                                int32_t chains_selected, sr_posterior_out *out)
{
  if (!s || !chains || !out || n_sel <= 0 || first < 0 || count < 0 || first + count > s->nrec || chains_selected == 0)
    return SR_EINVAL;
  for (int k = 0; k < n_sel; k++)
    if (chains[k] < 0 || chains[k] >= s->nchains) return SR_EINVAL;
  const int16_t *rec;
  int cap, dev;
  void *stream;
  if (srk_records_device(s->dev, &rec, &cap, &dev, &stream)) return SR_EDEVICE;
  const long long W = 2LL * s->ds.M + s->ds.N;
  long long *off = (long long *)malloc(sizeof(long long) * n_sel);
  if (!off) return SR_ENOMEM;
  for (int k = 0; k < n_sel; k++) off[k] = ((long long)chains[k] * cap + first) * W;
  int rc = 0;
  for (int k = 0; k < 6 && !rc; k++) {
    double *dst = post_slot(out, k);
    if (!dst) continue;
    float ms = 0.0f;
    rc = srp_posterior_dev(dev, stream, post_kinds[k], rec, off, n_sel, count, W, s->ds.N, s->ds.M, s->ds.X,
                           chains_selected, dst, &ms);
    out->kernel_ms += ms;
  }
  free(off);
  return post_rc(rc);
}

SR_API void sr_session_destroy(sr_session *s)
{
  if (!s) return;
  if (s->dev) srk_destroy(s->dev);
  sr_free_dataset(&s->ds);
  free(s->specs);
  free(s->acc0);
  free(s->dbg_bad);
  free(s);
}

/* mcmc_consistent (mcmc.c:999-1094) on a downloaded chain state; 0 = consistent */
static int check_chain(const sr_dataset *ds, const sr_state_host *st, int c)
{
  const int N = ds->N, M = ds->M;
  hmodel x;
  if (hmodel_alloc(&x, ds)) return 1;
  int flag = 0;
  memcpy(x.rpi, st->rpi + (size_t)c * N, N * 4);
  memcpy(x.a, st->ab + (size_t)c * 2 * M, M * 4);
  memcpy(x.b, st->ab + (size_t)c * 2 * M + M, M * 4);
  for (int m = 0; m < M; m++)
    if (!(0 <= x.a[m] && x.a[m] <= x.b[m] && x.b[m] <= N)) flag = 1;
  char *seen = (char *)calloc(N, 1);
  for (int n = 0; n < N; n++) {
    int v = x.rpi[n];
    if (v < 0 || v >= N || seen[v]) { flag = 1; break; }
    seen[v] = 1;
  }
  free(seen);
  if (flag) { hmodel_free(&x); return 1; }
  for (int n = 0; n < N; n++) x.pi[x.rpi[n]] = n;
  int last = -1, nh = 0;
  for (int n = 0; n < N; n++)
    if (ds->hard[n]) { nh++; if (last >= 0 && x.pi[n] < last) flag = 1; last = x.pi[n]; }
  if (nh != ds->nh) flag = 1;
  x.c = st->cdl[(size_t)c * 4 + 0];
  x.d = st->cdl[(size_t)c * 4 + 1];
  x.cv = st->manycd ? st->cdv + (size_t)c * 2 * M : NULL;
  h_count01(&x);
  const int32_t *cnt = st->cnt + (size_t)c * 4 * M;
  for (int m = 0; m < M; m++)
    if (x.t0[m] != cnt[m] || x.f0[m] != cnt[M + m] || x.t1[m] != cnt[2 * M + m] || x.f1[m] != cnt[3 * M + m]) flag = 1;
  double dl = st->cdl[(size_t)c * 4 + 2] - h_logl(&x);
  if (dl < 0) dl = -dl;
  if (!(dl <= 1e-8)) flag = 1;
  /* P must still be X in position order */
  const uint32_t *P = st->P + (size_t)c * st->NW * M;
  for (int p = 0; p < N && !flag; p++)
    for (int m = 0; m < M; m++)
      if ((int)((P[(size_t)(p >> 5) * M + m] >> (p & 31)) & 1u) != ds->X[(size_t)x.rpi[p] * M + m]) { flag = 1; break; }
  hmodel_free(&x);
  return flag;
}

/* ------------------------------------------------------------- run loops */
typedef struct {
  double ls, cs, ds;
} sr_sums;

typedef struct {
  FILE **f;     /* chain_data.csv per chain */
  int M;
} dir_ctx;

/* one mcmc_save_chain line (mcmc.c:69-92) into *buf; c and d are shared by all taxa
 * (manycd=0), so their "%.14f " text is formatted once and replicated; cdv (manycd=1): each
 * taxon's own c[M], d[M].  Returns the length. */
static char *put_int(char *p, int v);
static long format_line(char **buf, size_t *cap, int N, int M, const int16_t *ab_pi, const double *cdl, const double *cdv)
{
  char cbuf[64], dbuf[64];
  const int cl = snprintf(cbuf, sizeof cbuf, "%.14f ", exp(cdl[0]));
  const int dl = snprintf(dbuf, sizeof dbuf, "%.14f ", exp(cdl[1]));
  const size_t need = (size_t)(2 * M + N) * 12 + (size_t)M * (cdv ? 2 * 40 : (cl + dl)) + 128;
  if (need > *cap) {
    char *nl = (char *)realloc(*buf, need);
    if (!nl) return -1;
    *buf = nl; *cap = need;
  }
  char *p = *buf;
  for (int i = 0; i < M; i++) { p = put_int(p, ab_pi[i]); *p++ = ' '; }
  *p++ = ',';
  for (int i = 0; i < M; i++) { p = put_int(p, ab_pi[M + i]); *p++ = ' '; }
  *p++ = ',';
  for (int i = 0; i < N; i++) { p = put_int(p, ab_pi[2 * M + i]); *p++ = ' '; }
  *p++ = ',';
  if (cdv) {
    for (int i = 0; i < M; i++) p += sprintf(p, "%.14f ", exp(cdv[i]));
    *p++ = ',';
    for (int i = 0; i < M; i++) p += sprintf(p, "%.14f ", exp(cdv[M + i]));
  } else {
    for (int i = 0; i < M; i++) { memcpy(p, cbuf, cl); p += cl; }
    *p++ = ',';
    for (int i = 0; i < M; i++) { memcpy(p, dbuf, dl); p += dl; }
  }
  p += sprintf(p, ",%.14f\n", cdl[2]);
  return (long)(p - *buf);
}

/* per-launch consumer of the pipelined sampler (srk_run_pipelined): running sums of
 * compute_exp_data (mcmc.c:53-58) and either the caller's sink (sequential, per chain in sample
 * order) or the chain_data.csv writers (chains formatted in parallel by nthr threads, each chain
 * by one thread in sample order; the GPU runs the next launch meanwhile). */
typedef struct {
  int n, N, M;
  sr_sums *sums;
  sr_sample_sink_fn sink;
  void *ctx;
  int32_t *ra;
  dir_ctx *dir;
  int nthr;
  /* current batch (for the writer threads) */
  int first, count;
  const int16_t *ab;
  const double *cd;
  const double *cdv;   /* manycd: [n][count][2M] per-taxon c, d, else NULL */
  int err;
} run_ctx;

typedef struct { run_ctx *r; int t; char *line; size_t cap; } writer_arg;

static void chain_sums(run_ctx *r, int c)
{
  for (int t = 0; t < r->count; t++) {
    const double *cd = r->cd + ((size_t)c * r->count + t) * 3;
    r->sums[c].ls += -(cd[2]);
    r->sums[c].cs += exp(cd[0]);
    r->sums[c].ds += exp(cd[1]);
  }
}

static void *writer_main(void *va)
{
  writer_arg *w = (writer_arg *)va;
  run_ctx *r = w->r;
  const size_t W = 2 * (size_t)r->M + r->N;
  for (int c = w->t; c < r->n; c += r->nthr) {
    chain_sums(r, c);
    for (int t = 0; t < r->count; t++) {
      const long len = format_line(&w->line, &w->cap, r->N, r->M, r->ab + ((size_t)c * r->count + t) * W,
                                   r->cd + ((size_t)c * r->count + t) * 3,
                                   r->cdv ? r->cdv + ((size_t)c * r->count + t) * 2 * r->M : NULL);
      if (len < 0 || fwrite(w->line, 1, (size_t)len, r->dir->f[c]) != (size_t)len) { r->err = 1; return NULL; }
    }
  }
  return NULL;
}

static int consume_batch(void *vctx, int first, int count, const int16_t *ab, const double *cd, const double *cdv)
{
  run_ctx *r = (run_ctx *)vctx;
  r->first = first; r->count = count; r->ab = ab; r->cd = cd; r->cdv = cdv;
  const int N = r->N, M = r->M, W = 2 * M + N;
  if (r->dir) {
    writer_arg wa[SR_MAX_WRITERS];
    pthread_t th[SR_MAX_WRITERS];
    int started = 0;
    for (int t = 0; t < r->nthr; t++) { wa[t].r = r; wa[t].t = t; wa[t].line = NULL; wa[t].cap = 0; }
    for (int t = 1; t < r->nthr; t++) {
      if (pthread_create(&th[t], NULL, writer_main, &wa[t]) != 0) { r->err = 1; break; }
      started = t;
    }
    writer_main(&wa[0]);
    for (int t = 1; t <= started; t++) pthread_join(th[t], NULL);
    for (int t = 0; t < r->nthr; t++) free(wa[t].line);
    return r->err;
  }
  for (int c = 0; c < r->n; c++) {
    chain_sums(r, c);
    if (!r->sink) continue;
    for (int t = 0; t < count; t++) {
      const int16_t *src = ab + ((size_t)c * count + t) * W;
      const double *cdl = cd + ((size_t)c * count + t) * 3;
      for (int q = 0; q < W; q++) r->ra[q] = src[q];
      const double *cv = cdv ? cdv + ((size_t)c * count + t) * 2 * M : NULL;
      sr_record rec = {N, M, r->ra, r->ra + M, r->ra + 2 * M, cdl[0], cdl[1], cdl[2], cv, cv ? cv + M : NULL};
      if (r->sink(r->ctx, c, first + t, &rec)) return 1;
    }
  }
  return 0;
}

static int writer_threads(int n)
{
  const char *e = getenv("SR_WRITER_THREADS");
  long t = e ? strtol(e, NULL, 10) : sysconf(_SC_NPROCESSORS_ONLN);
  if (t < 1) t = 1;
  if (t > SR_MAX_WRITERS) t = SR_MAX_WRITERS;
  if (t > n) t = n;
  return (int)t;
}

static int run_common(const sr_dataset *ds, const sr_chain_spec *specs, int32_t n, const sr_run_opts *opts,
                      sr_sample_sink_fn sink, void *ctx, dir_ctx *dir, int wthr, sr_chain_summary *out,
                      sr_state_host *final_state)
{
  sr_run_opts o;
  if (opts) o = *opts; else sr_default_opts(&o);
  if (o.burnin_calls < 0 || o.sample_calls < 0) return SR_EINVAL;
  const int cpl = auto_calls_per_launch(&o);
  sr_run_opts o2 = o;
  o2.calls_per_launch = 2 * cpl;   /* two record halves: one being written, one being consumed */
  sr_session *s = NULL;
  int rc = sr_session_create(ds, specs, n, &o2, &s);
  if (rc) return rc;
  /* SR_F_DEBUG_CHECK: a chain failing the per-call check is flagged in the session (dbg_bad) and
     the run goes on (mcmc.c:254); its summary reports it at the end */
  for (int done = 0; done < o.burnin_calls;) {
    int k = o.burnin_calls - done < cpl ? o.burnin_calls - done : cpl;
    if ((rc = sr_session_run(s, k, 0)) && rc != SR_EINCONSISTENT) goto fail;
    done += k;
  }
  const int N = ds->N, M = ds->M, W = 2 * M + N;
  run_ctx r;
  memset(&r, 0, sizeof r);
  r.n = n; r.N = N; r.M = M; r.sink = sink; r.ctx = ctx; r.dir = dir;
  r.nthr = dir ? writer_threads(n) : 1;
  if (wthr > 0 && r.nthr > wthr) r.nthr = wthr;   /* a shard's share of the writer threads */
  r.sums = (sr_sums *)calloc(n, sizeof(sr_sums));
  r.ra = (int32_t *)malloc((size_t)W * 4);
  if (!r.sums || !r.ra) { free(r.sums); free(r.ra); rc = SR_ENOMEM; goto fail; }
  if (o.flags & SR_F_DEBUG_CHECK) {   /* checked call by call (sr_session_run), records consumed per call */
    const size_t W2 = (size_t)W;
    int16_t *ab = (int16_t *)malloc(W2 * n * sizeof(int16_t));
    double *cd = (double *)malloc((size_t)3 * n * sizeof(double));
    double *cv = o.manycd ? (double *)malloc((size_t)2 * M * n * sizeof(double)) : NULL;
    rc = (ab && cd && (cv || !o.manycd)) ? SR_OK : SR_ENOMEM;
    for (int t = 0; t < o.sample_calls && rc == SR_OK; t++) {
      sr_session_reset_records(s);
      if ((rc = sr_session_run(s, 1, 1)) && rc != SR_EINCONSISTENT) break;
      rc = SR_OK;   /* a flagged chain (dbg_bad) keeps sampling */
      if ((rc = sr_session_fetch_records(s, 0, 1, ab, cd))) break;
      if (cv && (rc = sr_session_fetch_cd_vectors(s, 0, 1, cv))) break;
      if (consume_batch(&r, t, 1, ab, cd, cv)) rc = dir ? SR_EIO : SR_EINVAL;
    }
    free(ab); free(cd); free(cv); free(r.ra);
    if (rc) { free(r.sums); goto fail; }
  } else {
  rc = srk_run_pipelined(s->dev, o.sample_calls, cpl, o.sweeps_per_call, consume_batch, &r);
  free(r.ra);
  if (rc) { free(r.sums); rc = (rc == -1) ? (dir ? SR_EIO : SR_EINVAL) : SR_EDEVICE; goto fail; }
  }
  sr_state_host st;
  rc = download(s, &st);
  if (rc) { free(r.sums); goto fail; }
  for (int c = 0; c < n; c++) {
    if (out) {
      out[c].chain_id = specs[c].chain_id;
      out[c].exp_loglik = r.sums[c].ls / 1000;      /* print_exp_data divides by 1000 (mcmc.c:62-64) */
      out[c].exp_c = r.sums[c].cs / 1000;
      out[c].exp_d = r.sums[c].ds / 1000;
      out[c].consistent = ((o.flags & SR_F_NO_CHECK) ? 0 : check_chain(ds, &st, c)) | (s->dbg_bad ? s->dbg_bad[c] : 0);
    }
  }
  free(r.sums);
  int bad = 0;
  for (int c = 0; c < n && s->dbg_bad; c++) bad |= s->dbg_bad[c];
  if (final_state) *final_state = st; else state_free(&st);
  sr_session_destroy(s);
  if (out && !(o.flags & SR_F_NO_CHECK))
    for (int c = 0; c < n; c++) if (out[c].consistent) return SR_EINCONSISTENT;
  return bad ? SR_EINCONSISTENT : SR_OK;
fail:
  sr_session_destroy(s);
  return rc;
}

/* ---- several devices from one call: chains sharded contiguously, one host thread per shard ----
 * Shard k (of nd) owns chains [k n / nd, (k + 1) n / nd) and runs run_common on devices[k]; a chain's
 * trajectory depends only on (dataset, seed), so every output equals the single-device run.  The
 * caller's sink is called under a mutex with the global chain index; final states are merged. */
typedef struct {
  const sr_dataset *ds;
  const sr_chain_spec *specs;
  int n, off, rc;
  sr_run_opts o;
  sr_sample_sink_fn sink;
  void *ctx;
  pthread_mutex_t *mu;
  dir_ctx dir;
  int have_dir;
  sr_chain_summary *out;
  sr_state_host st;
  int want_state;
  int wthr;                 /* this shard's share of the chain_data.csv writer threads */
} shard_arg;

static int shard_sink(void *ctx, int32_t ci, int32_t si, const sr_record *rec)
{
  shard_arg *a = (shard_arg *)ctx;
  pthread_mutex_lock(a->mu);
  const int rc = a->sink(a->ctx, a->off + ci, si, rec);
  pthread_mutex_unlock(a->mu);
  return rc;
}

static void *shard_main(void *va)
{
  shard_arg *a = (shard_arg *)va;
  a->rc = run_common(a->ds, a->specs, a->n, &a->o, a->sink ? shard_sink : NULL, a, a->have_dir ? &a->dir : NULL,
                     a->wthr, a->out, a->want_state ? &a->st : NULL);
  return NULL;
}

static int run_multi(const sr_dataset *ds, const sr_chain_spec *specs, int32_t n, const sr_run_opts *opts,
                     const int32_t *devices, int32_t nd, sr_sample_sink_fn sink, void *ctx, dir_ctx *dir,
                     sr_chain_summary *out, sr_state_host *final_state)
{
  if (nd <= 0 || nd > n || !devices) return SR_EINVAL;
  sr_run_opts o;
  if (opts) o = *opts; else sr_default_opts(&o);
  if (nd == 1) { o.device = devices[0]; return run_common(ds, specs, n, &o, sink, ctx, dir, 0, out, final_state); }
  shard_arg *sa = (shard_arg *)calloc(nd, sizeof(shard_arg));
  pthread_t *th = (pthread_t *)calloc(nd, sizeof(pthread_t));
  int *started = (int *)calloc(nd, sizeof(int));
  if (!sa || !th || !started) { free(sa); free(th); free(started); return SR_ENOMEM; }
  pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
  int rc = SR_OK;
  /* the host's writer threads are shared by the shards, not started per shard */
  const int wtot = dir ? writer_threads(n) : 1, wshare = wtot / nd > 0 ? wtot / nd : 1;
  for (int k = 0; k < nd; k++) {
    shard_arg *a = &sa[k];
    a->off = (int)((long)k * n / nd);
    a->n = (int)((long)(k + 1) * n / nd) - a->off;
    a->ds = ds; a->specs = specs + a->off; a->o = o; a->o.device = devices[k];
    a->sink = sink; a->ctx = ctx; a->mu = &mu;
    if (dir) { a->dir.f = dir->f + a->off; a->dir.M = dir->M; a->have_dir = 1; }
    a->out = out ? out + a->off : NULL;
    a->want_state = final_state != NULL;
    a->wthr = wshare;
    a->rc = SR_EDEVICE;
    if (pthread_create(&th[k], NULL, shard_main, a) != 0) { rc = SR_ENOMEM; break; }
    started[k] = 1;
  }
  for (int k = 0; k < nd; k++) if (started[k]) pthread_join(th[k], NULL);
  /* the first hard error wins; SR_EINCONSISTENT (every shard finished its run) only if none */
  for (int k = 0; k < nd && rc == SR_OK; k++) if (sa[k].rc && sa[k].rc != SR_EINCONSISTENT) rc = sa[k].rc;
  for (int k = 0; k < nd && rc == SR_OK; k++) if (sa[k].rc) rc = sa[k].rc;
  /* a shard that returned SR_EINCONSISTENT finished its run and left its final state; any shard
     without one (it failed before) makes the merge impossible */
  for (int k = 0; k < nd && final_state && (rc == SR_OK || rc == SR_EINCONSISTENT); k++)
    if (!sa[k].st.ab) rc = SR_EDEVICE;
  if (final_state && (rc == SR_OK || rc == SR_EINCONSISTENT)) {
    int r2 = state_alloc(final_state, ds->N, ds->M, ds->nh, n, o.manycd != 0);
    if (r2) rc = r2;
    else {
      ck_part dst[SR_CK_PARTS], src[SR_CK_PARTS];
      const int np = ck_parts(final_state, dst);
      for (int k = 0; k < nd; k++) {
        ck_parts(&sa[k].st, src);
        for (int q = 0; q < np; q++) {
          const size_t per = dst[q].bytes / (size_t)n;
          memcpy((char *)dst[q].p + per * sa[k].off, src[q].p, per * sa[k].n);
        }
      }
    }
  }
  for (int k = 0; k < nd; k++) if (sa[k].want_state) state_free(&sa[k].st);
  free(sa); free(th); free(started);
  return rc;
}

SR_API int sr_run_chains(const sr_dataset *ds, const sr_chain_spec *specs, int32_t n_chains, const sr_run_opts *opts,
                         sr_sample_sink_fn sink, void *sink_ctx, sr_chain_summary *out)
{
  if (!ds || !specs || n_chains <= 0) return SR_EINVAL;
  return run_common(ds, specs, n_chains, opts, sink, sink_ctx, NULL, 0, out, NULL);
}

SR_API int sr_run_chains_multi(const sr_dataset *ds, const sr_chain_spec *specs, int32_t n_chains, const sr_run_opts *opts,
                               const int32_t *devices, int32_t n_devices, sr_sample_sink_fn sink, void *sink_ctx,
                               sr_chain_summary *out)
{
  if (!ds || !specs || n_chains <= 0) return SR_EINVAL;
  return run_multi(ds, specs, n_chains, opts, devices, n_devices, sink, sink_ctx, NULL, out, NULL);
}

/* ------------------------------------------------------------ file output */
static char *put_int(char *p, int v)
{
  char tmp[16];
  int n = 0;
  unsigned u = v < 0 ? (unsigned)(-(long)v) : (unsigned)v;
  if (v < 0) *p++ = '-';
  do { tmp[n++] = (char)('0' + u % 10); u /= 10; } while (u);
  while (n) *p++ = tmp[--n];
  return p;
}

static void chain_dir(char *buf, size_t n, const char *root, int id)
{
  if (id >= 0 && id < 100) snprintf(buf, n, "%s/Chains/chain_%02d", root, id);
  else snprintf(buf, n, "%s/Chains/chain_%d", root, id);
}

SR_API int sr_run_to_dirs_multi(const sr_dataset *ds, const sr_chain_spec *specs, int32_t n, const sr_run_opts *opts,
                                const int32_t *devices, int32_t n_devices, const char *root, sr_chain_summary *out)
{
  if (!ds || !specs || n <= 0 || !root || !devices || n_devices <= 0 || n_devices > n) return SR_EINVAL;
  char path[4096], dir[4000];
  snprintf(path, sizeof path, "%s/mcmc_c.log", root);     /* mcmc.c:104 (never written) */
  FILE *lf = fopen(path, "a");
  if (lf) fclose(lf);
  snprintf(dir, sizeof dir, "%s/Chains", root);
  mkdir(dir, 0777);
  dir_ctx x;
  x.M = ds->M;
  x.f = (FILE **)calloc(n, sizeof(FILE *));
  sr_chain_summary *sum = out ? out : (sr_chain_summary *)calloc(n, sizeof(sr_chain_summary));
  if (!x.f || !sum) { free(x.f); if (!out) free(sum); return SR_ENOMEM; }
  int rc = SR_OK;
  for (int c = 0; c < n && !rc; c++) {
    chain_dir(dir, sizeof dir, root, specs[c].chain_id);
    mkdir(dir, 0777);
    snprintf(path, sizeof path, "%s/chain_data.csv", dir);
    x.f[c] = fopen(path, "w");
    if (!x.f[c]) rc = SR_EIO;
  }
  sr_state_host st;
  memset(&st, 0, sizeof st);
  if (!rc) rc = run_multi(ds, specs, n, opts, devices, n_devices, NULL, NULL, &x, sum, &st);
  for (int c = 0; c < n; c++) if (x.f[c]) fclose(x.f[c]);
  free(x.f);
  if (rc && rc != SR_EINCONSISTENT) { if (!out) free(sum); state_free(&st); return rc; }
  const int N = ds->N, M = ds->M;
  for (int c = 0; c < n && st.ab; c++) {
    chain_dir(dir, sizeof dir, root, specs[c].chain_id);
    FILE *f1, *f2, *f3, *f4;
    snprintf(path, sizeof path, "%s/taxa.csv", dir); f1 = fopen(path, "w");
    snprintf(path, sizeof path, "%s/sites.csv", dir); f2 = fopen(path, "w");
    snprintf(path, sizeof path, "%s/hard_sites.csv", dir); f3 = fopen(path, "w");
    snprintf(path, sizeof path, "%s/exp_data.csv", dir); f4 = fopen(path, "w");
    if (!f1 || !f2 || !f3 || !f4) {
      if (f1) fclose(f1);
      if (f2) fclose(f2);
      if (f3) fclose(f3);
      if (f4) fclose(f4);
      rc = SR_EIO;
      break;
    }
    fprintf(f4, "exp_loglik,exp_c,exp_d\n");                   /* print_exp_data, mcmc.c:60-67 */
    fprintf(f4, "%.14f,%.14f,%.14f", sum[c].exp_loglik, sum[c].exp_c, sum[c].exp_d);
    const int32_t *a = st.ab + (size_t)c * 2 * M, *b = a + M;
    const double cc = exp(st.cdl[(size_t)c * 4 + 0]), dd = exp(st.cdl[(size_t)c * 4 + 1]);
    const double *cv = st.manycd ? st.cdv + (size_t)c * 2 * M : NULL;   /* manycd: each taxon's own */
    fprintf(f1, "a,b,c,d\n");                                   /* mcmc_save, mcmc.c:261-293 */
    for (int i = 0; i < M; i++)
      fprintf(f1, "%d,%d,%.14f,%.14f\n", a[i], b[i], cv ? exp(cv[i]) : cc, cv ? exp(cv[M + i]) : dd);
    int *pi = (int *)malloc(N * sizeof(int));
    for (int p = 0; p < N; p++) pi[st.rpi[(size_t)c * N + p]] = p;
    fprintf(f2, "sites\n");
    for (int i = 0; i < N; i++) fprintf(f2, "%d\n", pi[i]);
    fprintf(f3, "i,pi_i\n");
    for (int i = 0; i < N; i++) if (ds->hard[i]) fprintf(f3, "%d,%d\n", i, pi[i]);
    free(pi);
    fclose(f1); fclose(f2); fclose(f3); fclose(f4);
  }
  state_free(&st);
  if (!out) free(sum);
  return rc;
}

SR_API int sr_run_to_dirs(const sr_dataset *ds, const sr_chain_spec *specs, int32_t n, const sr_run_opts *opts,
                          const char *root, sr_chain_summary *out)
{
  const int32_t dev = opts ? opts->device : 0;
  return sr_run_to_dirs_multi(ds, specs, n, opts, &dev, 1, root, out);
}

/* ------------------------------------------------------ test / diagnostic hooks */
/* per-chain phase cycle counters of an SR_STAMPS build ([n_chains][16]); zeros otherwise */
SR_API int sr_session_debug_counters(sr_session *s, unsigned long long *out)
{
  if (!s || !out) return SR_EINVAL;
  return srk_fetch_dbg(s->dev, out) ? SR_EDEVICE : SR_OK;
}

SR_API void sr_host_exp_log(const double *in, long n, double *out_exp, double *out_log)
{
  for (long k = 0; k < n; k++) {
    if (out_exp) out_exp[k] = h_exp(in[k]);
    if (out_log) out_log[k] = h_log(in[k]);
  }
}

SR_API double sr_host_run_add(double x, double e, long L) { return sr_run_add(x, e, L); }

/* the Philox mode's building blocks as the device uses them (sr_rng.h) */
SR_API void sr_host_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) { sr_philox4x32_10(ctr, key, out); }
SR_API void sr_host_mt_untemper(const uint32_t *in, long n, uint32_t *untempered, uint32_t *roundtrip)
{
  for (long k = 0; k < n; k++) { untempered[k] = sr_mt_untemper(in[k]); roundtrip[k] = sr_mt_temper(untempered[k]); }
}
SR_API long sr_host_run_sub(double *r, double p, long L) { return sr_run_sub(r, p, L); }

/* initial chain state as the host builds it (a, b, pi after mcmc_randomize; c, d, loglik) */
SR_API int sr_host_init_chain(const sr_dataset *ds, uint64_t seed, int32_t *a, int32_t *b, int32_t *pi,
                              double *cdl3, uint64_t *rng_pos)
{
  sr_state_host st;
  int rc = state_alloc(&st, ds->N, ds->M, ds->nh, 1, 0);
  if (rc) return rc;
  rc = init_chain(ds, seed, &st, 0, 0);
  if (!rc) {
    if (a) memcpy(a, st.ab, ds->M * 4);
    if (b) memcpy(b, st.ab + ds->M, ds->M * 4);
    if (pi) for (int n = 0; n < ds->N; n++) pi[st.rpi[n]] = n;
    if (cdl3) memcpy(cdl3, st.cdl, 24);
    if (rng_pos) *rng_pos = st.rng[0];
  }
  state_free(&st);
  return rc;
}
