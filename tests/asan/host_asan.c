/* tests/asan/host_asan.c -- TEST INFRASTRUCTURE: drives the C host layer (csrc/sr_host.c) built with
 * -fsanitize=address,undefined against the no-device stubs (srk_stub.c): dataset parsing (text with
 * and without the MAXS line limit, malformed inputs), the binary format round trip, chain
 * initialisation (mcmc_init / randomize), checkpoint writing, restore validation of intact and
 * damaged files, the multi-device argument checks, and the error paths of every run entry point.
 * usage: host_asan DATASET TMPDIR   (exit 0 = every check held; sanitizer reports abort) */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "seriation.h"

int sr_host_init_chain(const sr_dataset *ds, uint64_t seed, int32_t *a, int32_t *b, int32_t *pi, double *cdl3,
                       uint64_t *rng_pos);
int sr_host_initial_checkpoint(const sr_dataset *ds, const sr_chain_spec *specs, int32_t n, const char *path);

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "host_asan: check failed at line %d: %s\n", __LINE__, #c); return 1; } } while (0)

static char *slurp(const char *path, size_t *len)
{
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  char *b = (char *)malloc((size_t)n + 1);
  if (b && fread(b, 1, (size_t)n, f) != (size_t)n) { free(b); b = NULL; }
  fclose(f);
  if (b) { b[n] = 0; *len = (size_t)n; }
  return b;
}

int main(int argc, char **argv)
{
  if (argc != 3) return 2;
  char path[4096];
  size_t len = 0;
  char *text = slurp(argv[1], &len);
  CHECK(text);
  sr_dataset ds, ds2;
  CHECK(sr_parse_dataset(text, len, SR_MAXS, &ds) == SR_OK);
  CHECK(sr_parse_dataset(text, len, 0, &ds2) == SR_OK && ds2.N == ds.N && ds2.M == ds.M);
  sr_free_dataset(&ds2);
  /* malformed inputs: empty, bad header, short rows, garbage */
  const char *bad[] = {"", "x y\n", "3 2\n1 0\n", "2 2\n1 1\n1 q\n", "-1 4\n", "2 2\n1 1 1 1 1\n0 0\n"};
  for (size_t k = 0; k < sizeof bad / sizeof bad[0]; k++) {
    sr_dataset t;
    int rc = sr_parse_dataset(bad[k], strlen(bad[k]), SR_MAXS, &t);
    if (rc == SR_OK) sr_free_dataset(&t);
  }
  /* binary round trip */
  snprintf(path, sizeof path, "%s/ds.srbx", argv[2]);
  CHECK(sr_save_dataset_bin(&ds, path) == SR_OK);
  CHECK(sr_load_dataset(path, 0, &ds2) == SR_OK);
  CHECK(ds2.N == ds.N && ds2.M == ds.M && memcmp(ds2.X, ds.X, (size_t)ds.N * ds.M) == 0 &&
        memcmp(ds2.hard, ds.hard, (size_t)ds.N) == 0);
  sr_free_dataset(&ds2);
  /* chain initialisation for several seeds */
  int32_t *a = (int32_t *)malloc(sizeof(int32_t) * ds.M), *b = (int32_t *)malloc(sizeof(int32_t) * ds.M);
  int32_t *pi = (int32_t *)malloc(sizeof(int32_t) * ds.N);
  double cdl[3];
  uint64_t pos;
  for (uint64_t s = 0; s < 6; s++) {
    CHECK(sr_host_init_chain(&ds, s, a, b, pi, cdl, &pos) == SR_OK);
    for (int m = 0; m < ds.M; m++) CHECK(a[m] >= 0 && a[m] < b[m] && b[m] <= ds.N);
  }
  /* checkpoints: intact file passes validation (then no device), damaged ones are refused */
  sr_chain_spec specs[3] = {{0, 1}, {1, 2}, {2, 3}};
  snprintf(path, sizeof path, "%s/init.srck", argv[2]);
  CHECK(sr_host_initial_checkpoint(&ds, specs, 3, path) == SR_OK);
  sr_run_opts o;
  sr_default_opts(&o);
  sr_session *s = NULL;
  CHECK(sr_session_restore(&ds, path, &o, &s) == SR_EDEVICE);
  size_t clen = 0;
  char *ck = slurp(path, &clen);
  CHECK(ck);
  char dpath[4096];
  snprintf(dpath, sizeof dpath, "%s/damaged.srck", argv[2]);
  const size_t hdr = 4 + 4 + 16 + 8 + 3 * sizeof(sr_chain_spec);
  for (size_t off = hdr; off < clen; off += (clen - hdr) / 97 + 1) {
    char save = ck[off];
    ck[off] = (char)(save ^ 0x5a);
    FILE *f = fopen(dpath, "wb");
    CHECK(f && fwrite(ck, 1, clen, f) == clen);
    fclose(f);
    const int rc = sr_session_restore(&ds, dpath, &o, &s);
    CHECK(rc == SR_EPARSE || rc == SR_EDEVICE);   /* refused, or an unused byte: accepted, then no device */
    ck[off] = save;
  }
  FILE *f = fopen(dpath, "wb");
  CHECK(f && fwrite(ck, 1, clen / 2, f) == clen / 2);   /* truncated */
  fclose(f);
  CHECK(sr_session_restore(&ds, dpath, &o, &s) == SR_EPARSE);
  free(ck);
  /* run entry points without a device; multi-device argument checks */
  sr_chain_summary out[3];
  CHECK(sr_run_chains(&ds, specs, 3, &o, NULL, NULL, out) == SR_EDEVICE);
  const int32_t devs[3] = {0, 0, 0};
  CHECK(sr_run_chains_multi(&ds, specs, 3, &o, devs, 3, NULL, NULL, out) == SR_EDEVICE);
  CHECK(sr_run_chains_multi(&ds, specs, 2, &o, devs, 3, NULL, NULL, out) == SR_EINVAL);
  CHECK(sr_run_to_dirs_multi(&ds, specs, 3, &o, devs, 2, argv[2], out) == SR_EDEVICE);
  o.flags = SR_F_RNG_PHILOX | SR_F_DEBUG_CHECK;
  CHECK(sr_session_create(&ds, specs, 3, &o, &s) == SR_EDEVICE);
  CHECK(sr_strerror(SR_EDEVICE) && sr_version());
  free(a); free(b); free(pi); free(text);
  sr_free_dataset(&ds);
  printf("host_asan: ok\n");
  return 0;
}
