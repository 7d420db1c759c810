/*
 * mcmc_cli.c -- the drop-in `mcmc` executable (reference CLI, mcmc.c:102-210):
 *
 *   env GSL_RNG_SEED=42 ./mcmc <chain_index> < dataset.txt
 *   ./mcmc manycd Tburnin T < dataset.txt      (chain index 0: Chains/chain_00; the reference's own binary
 *                                             reads its unset chain index there and crashes, mcmc.c:153)
 *
 * Reads the dataset on stdin (fgets(MAXS) semantics), seeds MT19937 from GSL_RNG_SEED
 * (strtoul base 0, unset -> GSL default; GSL_RNG_TYPE as gsl_rng_env_setup reads it: mt19937 runs,
 * another generator is refused with exit 1), runs the chain on the GPU and writes
 * Chains/chain_NN/{chain_data,exp_data,taxa,sites,hard_sites}.csv in the cwd.
 * Extension (not in the reference): SR_DEVICE=<ordinal> picks the GPU.
 * Exit 1 with the reference's messages on parse / consistency errors.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "seriation.h"

int main(int argc, char *argv[])
{
  int tb = 1000, ts = 1000, manycd = 0;
  const char *chain_index = "0";
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
  uint64_t seed = 0;
  /* mcmc_init (mcmc.c:591-592): GSL_RNG_TYPE (mt19937 only; another generator exits 1) and GSL_RNG_SEED */
  if (sr_rng_env_setup(&seed, 1)) return 1;
  size_t cap = 1 << 16, len = 0, got;
  char *text = malloc(cap);
  while (text && (got = fread(text + len, 1, cap - len, stdin)) > 0) {
    len += got;
    if (len == cap) { cap *= 2; text = realloc(text, cap); }
  }
  if (!text) { fprintf(stderr, "mcmc: out of memory.\n"); return 1; }
  sr_dataset ds;
  int rc = sr_parse_dataset(text, len, SR_MAXS, &ds);
  free(text);
  if (rc) { fprintf(stderr, "%s\n", sr_strerror(rc)); return 1; }
  sr_run_opts o;
  sr_default_opts(&o);
  o.burnin_calls = tb;
  o.sample_calls = ts;
  o.manycd = manycd;
  o.flags |= SR_F_DIAG;   /* mcmc_initab's "zero column" lines on stderr, as the reference */
  const char *dev = getenv("SR_DEVICE");
  if (dev) o.device = atoi(dev);
  /* reference naming: index > 9 uses its first two characters, else "0" + first char */
  int idx = atoi(chain_index);
  int id = idx > 9 ? (chain_index[0] - '0') * 10 + (chain_index[1] - '0') : (chain_index[0] - '0');
  if (idx >= 100) id = idx;  /* extension: chain_NNN for >= 100 chains */
  sr_chain_spec spec = {id, (uint64_t)seed};
  sr_chain_summary sum;
  rc = sr_run_to_dirs(&ds, &spec, 1, &o, ".", &sum);
  sr_free_dataset(&ds);
  if (rc == SR_EINCONSISTENT) { fprintf(stderr, "main: error.\n"); return 1; }
  if (rc) { fprintf(stderr, "mcmc: %s\n", sr_strerror(rc)); return 1; }
  return 0;
}
