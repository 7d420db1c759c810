/* tests/asan/srk_fake.c -- TEST INFRASTRUCTURE: a host-memory stand-in for the device layer of
 * libseriation.so, so that the host run loops (csrc/sr_host.c: run_common, run_multi, the debug
 * check, the pipelined writer, the file tree) run on a CPU-only machine under ASan/UBSan.
 *
 * It does NOT sample: a "sweep" leaves the uploaded chain state unchanged (so every chain stays
 * exactly as consistent as mcmc_randomize left it), records are the current state, and two
 * "devices" are reported; manycd sessions keep their per-taxon c, d (unchanged, recorded per call).
 * Fault injection: SR_FAKE_DAMAGE="chain:call" adds 1 to chain's t0 of
 * taxon 0 when that chain's session has completed `call` mcmc_sample calls (a count that no longer
 * matches count01: mcmc_consistent must flag it).  Never linked by the product. */
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>
#include "sr_internal.h"

struct srk_dev {
  sr_state_host st;
  int rec_cap;
  int16_t *rec;
  double *rcd;
  double *rcv;   /* manycd: [chain][rec_cap][2M] */
  long calls;
  int dmg_chain;
  long dmg_call;
};

int srk_device_count(void) { return 2; }

static void *dup(const void *p, size_t n)
{
  void *q = malloc(n ? n : 1);
  if (q && n) memcpy(q, p, n);
  return q;
}

int srk_create(const sr_state_host *st, int device, int block_threads, int rec_cap_calls, int gm_force,
               const uint32_t *pkey, int spec, srk_dev **out)
{
  (void)block_threads; (void)gm_force; (void)pkey; (void)spec;
  if (device < 0 || device >= 2) return -5;
  srk_dev *d = (srk_dev *)calloc(1, sizeof(*d));
  if (!d) return -5;
  const size_t C = (size_t)st->nchains;
  d->st = *st;
  d->st.P = (uint32_t *)dup(st->P, C * st->NW * st->M * 4);
  d->st.rpi = (int32_t *)dup(st->rpi, C * st->N * 4);
  d->st.hp = (int32_t *)dup(st->hp, C * SR_NHCAP(st->nh) * 4);
  d->st.ab = (int32_t *)dup(st->ab, C * 2 * st->M * 4);
  d->st.cnt = (int32_t *)dup(st->cnt, C * 4 * st->M * 4);
  d->st.cdl = (double *)dup(st->cdl, C * 4 * 8);
  d->st.mt = (uint32_t *)dup(st->mt, C * SR_RING * 624 * 4);
  d->st.rng = (uint64_t *)dup(st->rng, C * 2 * 8);
  d->st.acc = (uint64_t *)dup(st->acc, C * SR_NACC * 8);
  d->st.cdv = st->manycd ? (double *)dup(st->cdv, C * 2 * st->M * 8) : NULL;
  d->rec_cap = rec_cap_calls > 0 ? rec_cap_calls : 1;
  d->rec = (int16_t *)calloc(C * d->rec_cap * (2 * (size_t)st->M + st->N), 2);
  d->rcd = (double *)calloc(C * d->rec_cap * 3, 8);
  d->rcv = st->manycd ? (double *)calloc(C * d->rec_cap * 2 * st->M, 8) : NULL;
  d->dmg_chain = -1;
  const char *e = getenv("SR_FAKE_DAMAGE");
  if (e) sscanf(e, "%d:%ld", &d->dmg_chain, &d->dmg_call);
  *out = d;
  return 0;
}

int srk_set_stream(srk_dev *d, void *s) { (void)d; (void)s; return 0; }

static void put_record(srk_dev *d, int c, int slot)
{
  const int N = d->st.N, M = d->st.M, W = 2 * M + N;
  int16_t *r = d->rec + ((size_t)c * d->rec_cap + slot) * W;
  for (int k = 0; k < 2 * M; k++) r[k] = (int16_t)d->st.ab[(size_t)c * 2 * M + k];
  for (int p = 0; p < N; p++) r[2 * M + d->st.rpi[(size_t)c * N + p]] = (int16_t)p;
  memcpy(d->rcd + ((size_t)c * d->rec_cap + slot) * 3, d->st.cdl + (size_t)c * 4, 3 * 8);
  if (d->rcv)
    memcpy(d->rcv + ((size_t)c * d->rec_cap + slot) * 2 * M, d->st.cdv + (size_t)c * 2 * M, (size_t)2 * M * 8);
}

int srk_run(srk_dev *d, int calls, int spc, int save, int rec_base)
{
  (void)spc;
  if (save && rec_base + calls > d->rec_cap) return -1;
  for (int k = 0; k < calls; k++) {
    d->calls++;
    if (d->dmg_chain >= 0 && d->dmg_chain < d->st.nchains && d->calls == d->dmg_call)
      d->st.cnt[(size_t)d->dmg_chain * 4 * d->st.M] += 1;
    for (int c = 0; save && c < d->st.nchains; c++) put_record(d, c, rec_base + k);
  }
  return 0;
}

int srk_sync(srk_dev *d) { (void)d; return 0; }
double srk_last_ms(srk_dev *d) { (void)d; return 0.0; }
int srk_block_threads(const srk_dev *d) { (void)d; return 64; }
int srk_variant(const srk_dev *d) { (void)d; return 0; }
int srk_specialized(const srk_dev *d) { (void)d; return 0; }
int srk_fetch_dbg(srk_dev *d, unsigned long long *o) { memset(o, 0, (size_t)d->st.nchains * 17 * 8 * 8); return 0; }

int srk_fetch_records(srk_dev *d, int first, int count, int16_t *ab_pi, double *cdl)
{
  if (first < 0 || count < 0 || first + count > d->rec_cap) return -1;
  const size_t W = 2 * (size_t)d->st.M + d->st.N;
  for (int c = 0; c < d->st.nchains; c++) {
    if (ab_pi) memcpy(ab_pi + (size_t)c * count * W, d->rec + ((size_t)c * d->rec_cap + first) * W, (size_t)count * W * 2);
    if (cdl) memcpy(cdl + (size_t)c * count * 3, d->rcd + ((size_t)c * d->rec_cap + first) * 3, (size_t)count * 24);
  }
  return 0;
}

int srk_exp_data(srk_dev *d, int first, int count, double *sums)
{
  if (first < 0 || count < 0 || first + count > d->rec_cap) return -1;
  for (int c = 0; c < d->st.nchains; c++) {
    double ls = 0., cs = 0., ds = 0.;
    for (int t = 0; t < count; t++) {
      const double *r = d->rcd + ((size_t)c * d->rec_cap + first + t) * 3;
      ls += -(r[2]); cs += exp(r[0]); ds += exp(r[1]);
    }
    sums[3 * c] = ls; sums[3 * c + 1] = cs; sums[3 * c + 2] = ds;
  }
  return 0;
}

int srk_fetch_chain_records(srk_dev *d, int chain, int first, int count, int16_t *ab_pi, double *cdl)
{
  if (chain < 0 || chain >= d->st.nchains || first < 0 || count < 0 || first + count > d->rec_cap) return -1;
  const size_t W = 2 * (size_t)d->st.M + d->st.N, row = (size_t)chain * d->rec_cap + first;
  if (ab_pi) memcpy(ab_pi, d->rec + row * W, (size_t)count * W * 2);
  if (cdl) memcpy(cdl, d->rcd + row * 3, (size_t)count * 24);
  return 0;
}

int srk_download_state(srk_dev *d, sr_state_host *st)
{
  const size_t C = (size_t)d->st.nchains;
  if (st->P) memcpy(st->P, d->st.P, C * d->st.NW * d->st.M * 4);
  if (st->rpi) memcpy(st->rpi, d->st.rpi, C * d->st.N * 4);
  if (st->hp) memcpy(st->hp, d->st.hp, C * SR_NHCAP(st->nh) * 4);
  if (st->ab) memcpy(st->ab, d->st.ab, C * 2 * d->st.M * 4);
  if (st->cnt) memcpy(st->cnt, d->st.cnt, C * 4 * d->st.M * 4);
  if (st->cdl) memcpy(st->cdl, d->st.cdl, C * 4 * 8);
  if (st->mt) memcpy(st->mt, d->st.mt, C * SR_RING * 624 * 4);
  if (st->rng) memcpy(st->rng, d->st.rng, C * 2 * 8);
  if (st->acc) memcpy(st->acc, d->st.acc, C * SR_NACC * 8);
  if (st->cdv && d->st.cdv) memcpy(st->cdv, d->st.cdv, C * 2 * d->st.M * 8);
  return 0;
}

int srk_run_pipelined(srk_dev *d, int total, int cpl, int spc, int (*consume)(void *, int, int, const int16_t *, const double *, const double *),
                      void *ctx)
{
  if (cpl <= 0 || 2 * cpl > d->rec_cap) return -1;
  const size_t W = 2 * (size_t)d->st.M + d->st.N, C = (size_t)d->st.nchains;
  int16_t *ab = (int16_t *)malloc(C * cpl * W * 2);
  double *cd = (double *)malloc(C * cpl * 24);
  double *cv = d->rcv ? (double *)malloc(C * cpl * 2 * d->st.M * 8) : NULL;
  int rc = (ab && cd && (cv || !d->rcv)) ? 0 : -5;
  for (int done = 0; !rc && done < total;) {
    const int k = total - done < cpl ? total - done : cpl;
    rc = srk_run(d, k, spc, 1, 0);
    if (!rc) rc = srk_fetch_records(d, 0, k, ab, cd);
    if (!rc && cv) rc = srk_fetch_cdv(d, 0, k, cv);
    if (!rc && consume(ctx, done, k, ab, cd, cv)) rc = -1;
    done += k;
  }
  free(ab); free(cd); free(cv);
  return rc;
}

int srk_records_device(srk_dev *d, const int16_t **rec, int *cap, int *dev, void **stream)
{
  *rec = d->rec; *cap = d->rec_cap; *dev = 0; *stream = NULL;
  return 0;
}

int srp_posterior_dev(int device, void *stream, int kind, const int16_t *d_rec, const long long *off, int n_sel, int count,
                      long long row_stride, int N, int M, const uint8_t *X, int cs, double *out, float *ms)
{
  (void)device; (void)stream; (void)kind; (void)d_rec; (void)off; (void)n_sel; (void)count; (void)row_stride;
  (void)N; (void)M; (void)X; (void)cs; (void)out; (void)ms;
  return -5;
}
int srp_posterior_host(int device, int kind, const int16_t *ab, int n_sel, int count, int N, int M, const uint8_t *X,
                       int cs, double *out, float *ms)
{
  (void)device; (void)kind; (void)ab; (void)n_sel; (void)count; (void)N; (void)M; (void)X; (void)cs; (void)out; (void)ms;
  return -5;
}

void srk_destroy(srk_dev *d)
{
  if (!d) return;
  free(d->st.P); free(d->st.rpi); free(d->st.hp); free(d->st.ab); free(d->st.cnt);
  free(d->st.cdl); free(d->st.mt); free(d->st.rng); free(d->st.acc); free(d->st.cdv);
  free(d->rec); free(d->rcd); free(d->rcv);
  free(d);
}
int srk_fetch_cdv(srk_dev *d, int first, int count, double *cdv)
{
  if (!d->rcv || first < 0 || count < 0 || first + count > d->rec_cap) return -1;
  const size_t R2 = 2 * (size_t)d->st.M;
  for (int c = 0; c < d->st.nchains; c++)
    memcpy(cdv + (size_t)c * count * R2, d->rcv + ((size_t)c * d->rec_cap + first) * R2, (size_t)count * R2 * 8);
  return 0;
}
/* "device" memory of the fake is host memory: the device-to-device copy is a memcpy */
int srk_copy_chain_records(srk_dev *d, int chain, int first, int count, int16_t *ab_pi, double *cdl)
{
  return srk_fetch_chain_records(d, chain, first, count, ab_pi, cdl);
}
/* no specialised kernels on the fake device */
int srk_plan(int N, int M, int nh, int block_threads, int gm_force, int manycd, sr_spec_shape *shape)
{
  (void)N; (void)M; (void)nh; (void)block_threads; (void)gm_force; (void)manycd; (void)shape;
  return 0;
}
const void *sr_spec_embedded(const sr_spec_shape *s, size_t *bytes) { (void)s; *bytes = 0; return NULL; }
int srk_upload_records(srk_dev *d, int count, const int16_t *ab_pi, const double *cdl, const double *cdv)
{
  if (count < 0 || count > d->rec_cap) return -1;
  const size_t W = 2 * (size_t)d->st.M + d->st.N, R2 = 2 * (size_t)d->st.M;
  for (int c = 0; c < d->st.nchains; c++) {
    memcpy(d->rec + (size_t)c * d->rec_cap * W, ab_pi + (size_t)c * count * W, (size_t)count * W * 2);
    memcpy(d->rcd + (size_t)c * d->rec_cap * 3, cdl + (size_t)c * count * 3, (size_t)count * 24);
    if (cdv && d->rcv) memcpy(d->rcv + (size_t)c * d->rec_cap * R2, cdv + (size_t)c * count * R2, (size_t)count * R2 * 8);
  }
  return 0;
}
