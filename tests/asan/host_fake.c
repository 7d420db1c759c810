/* tests/asan/host_fake.c -- TEST INFRASTRUCTURE: the host run loops of csrc/sr_host.c (run_common,
 * run_multi, the SR_F_DEBUG_CHECK path, the chain file tree) driven against the host-memory fake
 * device (srk_fake.c: sweeps leave the state unchanged; SR_FAKE_DAMAGE="chain:call" corrupts a count)
 * under ASan + UBSan.  Checks that a chain failing mcmc_consistent after some call is reported in
 * its summary and by SR_EINCONSISTENT -- single device, two shards, the session API -- and that no
 * path crashes on it; and manycd = 1 through the same paths (records, writers, checkpoint v4).   usage: host_fake DATASET TMPDIR   (exit 0 = every check held) */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include "seriation.h"

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "host_fake: check failed at line %d: %s\n", __LINE__, #c); return 1; } } while (0)

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

static int exists(const char *p) { struct stat sb; return stat(p, &sb) == 0; }

int main(int argc, char **argv)
{
  if (argc != 3) return 2;
  size_t len = 0;
  char *text = slurp(argv[1], &len), path[4096];
  CHECK(text);
  sr_dataset ds;
  CHECK(sr_parse_dataset(text, len, 0, &ds) == SR_OK);
  free(text);
  sr_chain_spec specs[4] = {{0, 11}, {1, 12}, {2, 13}, {3, 14}};
  sr_chain_summary out[4];
  sr_run_opts o;
  sr_default_opts(&o);
  o.burnin_calls = 3;
  o.sample_calls = 5;
  o.calls_per_launch = 2;
  o.flags = SR_F_DEBUG_CHECK;
  const int32_t devs[2] = {0, 1};

  /* 1. intact chains: every per-call check and the closing check pass, two shards */
  unsetenv("SR_FAKE_DAMAGE");
  memset(out, 0xff, sizeof out);
  CHECK(sr_run_to_dirs_multi(&ds, specs, 4, &o, devs, 2, argv[2], out) == SR_OK);
  for (int c = 0; c < 4; c++) CHECK(out[c].consistent == 0 && out[c].chain_id == c && out[c].exp_loglik > 0.0);
  snprintf(path, sizeof path, "%s/Chains/chain_03/taxa.csv", argv[2]);
  CHECK(exists(path));

  /* 2. chain 1 of every shard (global 1 and 3) damaged after its 4th call (a burn-in call): the run
        completes, both are flagged, the others are not, the final state is merged and written */
  setenv("SR_FAKE_DAMAGE", "1:4", 1);
  memset(out, 0, sizeof out);
  CHECK(sr_run_to_dirs_multi(&ds, specs, 4, &o, devs, 2, argv[2], out) == SR_EINCONSISTENT);
  CHECK(out[0].consistent == 0 && out[1].consistent != 0 && out[2].consistent == 0 && out[3].consistent != 0);
  for (int c = 0; c < 4; c++) CHECK(out[c].chain_id == c && out[c].exp_loglik > 0.0);

  /* 3. the same with the closing check off: the per-call check alone must still report it */
  o.flags = SR_F_DEBUG_CHECK | SR_F_NO_CHECK;
  memset(out, 0, sizeof out);
  CHECK(sr_run_to_dirs_multi(&ds, specs, 4, &o, devs, 2, argv[2], out) == SR_EINCONSISTENT);
  CHECK(out[0].consistent == 0 && out[1].consistent != 0 && out[2].consistent == 0 && out[3].consistent != 0);

  /* 4. single device, damage during the sampling phase (call 6 of 8) */
  o.flags = SR_F_DEBUG_CHECK;
  setenv("SR_FAKE_DAMAGE", "2:6", 1);
  memset(out, 0, sizeof out);
  CHECK(sr_run_chains(&ds, specs, 4, &o, NULL, NULL, out) == SR_EINCONSISTENT);
  for (int c = 0; c < 4; c++) CHECK((out[c].consistent != 0) == (c == 2) && out[c].exp_loglik > 0.0);

  /* 5. the session API: the failing call returns SR_EINCONSISTENT, later calls still run and the
        flag stays set for that chain only */
  sr_session *s = NULL;
  setenv("SR_FAKE_DAMAGE", "0:2", 1);
  o.calls_per_launch = 8;   /* record capacity */
  CHECK(sr_session_create(&ds, specs, 4, &o, &s) == SR_OK);
  CHECK(sr_session_run(s, 1, 0) == SR_OK);
  CHECK(sr_session_debug_flagged(s, 0) == 0);
  CHECK(sr_session_run(s, 3, 1) == SR_EINCONSISTENT);
  CHECK(sr_session_records(s) == 3);
  CHECK(sr_session_debug_flagged(s, 0) == 1 && sr_session_debug_flagged(s, 1) == 0);
  CHECK(sr_session_run(s, 1, 0) == SR_EINCONSISTENT);
  CHECK(sr_session_debug_flagged(s, 4) == SR_EINVAL);
  sr_session_destroy(s);

  /* 6. without the flag nothing is checked per call; the closing check alone flags the damage */
  o.flags = 0;
  setenv("SR_FAKE_DAMAGE", "3:1", 1);
  memset(out, 0, sizeof out);
  CHECK(sr_run_chains(&ds, specs, 4, &o, NULL, NULL, out) == SR_EINCONSISTENT);
  for (int c = 0; c < 4; c++) CHECK((out[c].consistent != 0) == (c == 3));

  /* 7. manycd = 1 through the writers, the debug check, a checkpoint (v4) and its restore: every taxon's
        c, d travels with the records (the fake device keeps them unchanged: log .01 / log .3) */
  unsetenv("SR_FAKE_DAMAGE");
  o.flags = SR_F_DEBUG_CHECK;
  o.manycd = 1;
  o.calls_per_launch = 2;
  memset(out, 0, sizeof out);
  char root[4096];
  snprintf(root, sizeof root, "%s/manycd", argv[2]);
  mkdir(root, 0777);
  CHECK(sr_run_to_dirs_multi(&ds, specs, 4, &o, devs, 2, root, out) == SR_OK);
  for (int c = 0; c < 4; c++) CHECK(out[c].consistent == 0);
  snprintf(path, sizeof path, "%s/Chains/chain_02/chain_data.csv", root);
  size_t clen = 0;
  char *cd = slurp(path, &clen);
  CHECK(cd && strstr(cd, "0.01000000000000 ") && strstr(cd, "0.30000000000000 "));
  free(cd);
  o.flags = 0;
  CHECK(sr_run_chains(&ds, specs, 4, &o, NULL, NULL, out) == SR_OK);
  o.calls_per_launch = 8;
  CHECK(sr_session_create(&ds, specs, 4, &o, &s) == SR_OK && sr_session_manycd(s) == 1);
  CHECK(sr_session_run(s, 2, 1) == SR_OK);
  double *cv = (double *)malloc(sizeof(double) * 4 * 2 * 2 * ds.M);
  CHECK(cv && sr_session_fetch_cd_vectors(s, 0, 2, cv) == SR_OK);
  CHECK(cv[0] < -4.6 && cv[0] > -4.61 && cv[ds.M] < -1.2 && cv[ds.M] > -1.21);   /* log .01, log .3 */
  free(cv);
  snprintf(path, sizeof path, "%s/m.ck", argv[2]);
  CHECK(sr_session_checkpoint(s, path) == SR_OK);
  sr_session_destroy(s);
  s = NULL;
  CHECK(sr_session_restore(&ds, path, &o, &s) == SR_OK && sr_session_manycd(s) == 1);
  sr_session_destroy(s);
  o.manycd = 0;
  CHECK(sr_session_restore(&ds, path, &o, &s) == SR_EINVAL);   /* a manycd checkpoint, opts say 0 */

  sr_free_dataset(&ds);
  printf("host_fake: ok\n");
  return 0;
}
