/* tests/asan/srk_stub.c -- TEST INFRASTRUCTURE: the device layer of libseriation.so replaced by
 * "no device" stubs, so that the C host layer (csrc/sr_host.c) can be built and exercised under
 * AddressSanitizer / UndefinedBehaviorSanitizer on a CPU-only machine (SURVEY §5 "race/sanitizer").
 * Every entry reports the same error the real layer reports without a gfx950 device. */
#include <stddef.h>
#include <stdint.h>
#include "sr_internal.h"

int srk_device_count(void) { return 0; }
int srk_create(const sr_state_host *st, int device, int block_threads, int rec_cap_calls, int gm_force,
               const uint32_t *pkey, int spec, srk_dev **out)
{
  (void)st; (void)device; (void)block_threads; (void)rec_cap_calls; (void)gm_force; (void)pkey; (void)spec; (void)out;
  return -5;
}
int srk_set_stream(srk_dev *d, void *s) { (void)d; (void)s; return -5; }
int srk_run(srk_dev *d, int calls, int spc, int save, int rec_base) { (void)d; (void)calls; (void)spc; (void)save; (void)rec_base; return -5; }
int srk_sync(srk_dev *d) { (void)d; return -5; }
double srk_last_ms(srk_dev *d) { (void)d; return -1.0; }
int srk_block_threads(const srk_dev *d) { (void)d; return 0; }
int srk_variant(const srk_dev *d) { (void)d; return -1; }
int srk_specialized(const srk_dev *d) { (void)d; return 0; }
int srk_fetch_dbg(srk_dev *d, unsigned long long *o) { (void)d; (void)o; return -5; }
int srk_fetch_records(srk_dev *d, int f, int c, int16_t *a, double *b) { (void)d; (void)f; (void)c; (void)a; (void)b; return -5; }
int srk_exp_data(srk_dev *d, int f, int c, double *s) { (void)d; (void)f; (void)c; (void)s; return -5; }
int srk_download_state(srk_dev *d, sr_state_host *st) { (void)d; (void)st; return -5; }
int srk_fetch_chain_records(srk_dev *d, int ch, int f, int c, int16_t *a, double *b)
{
  (void)d; (void)ch; (void)f; (void)c; (void)a; (void)b;
  return -5;
}
int srk_run_pipelined(srk_dev *d, int total, int cpl, int spc, int (*consume)(void *, int, int, const int16_t *, const double *, const double *),
                      void *ctx)
{
  (void)d; (void)total; (void)cpl; (void)spc; (void)consume; (void)ctx;
  return -5;
}
int srk_records_device(srk_dev *d, const int16_t **rec, int *cap, int *dev, void **stream)
{
  (void)d; (void)rec; (void)cap; (void)dev; (void)stream;
  return -5;
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
void srk_destroy(srk_dev *d) { (void)d; }
int srk_fetch_cdv(srk_dev *d, int f, int c, double *v) { (void)d; (void)f; (void)c; (void)v; return -5; }
int srk_copy_chain_records(srk_dev *d, int ch, int f, int c, int16_t *a, double *x)
{
  (void)d; (void)ch; (void)f; (void)c; (void)a; (void)x;
  return -5;
}
int srk_plan(int N, int M, int nh, int bt, int gm, int mcd, sr_spec_shape *s)
{
  (void)N; (void)M; (void)nh; (void)bt; (void)gm; (void)mcd; (void)s;
  return 0;
}
const void *sr_spec_embedded(const sr_spec_shape *s, size_t *bytes) { (void)s; *bytes = 0; return NULL; }
int srk_upload_records(srk_dev *d, int count, const int16_t *a, const double *c, const double *v)
{
  (void)d; (void)count; (void)a; (void)c; (void)v;
  return -5;
}
