/*
 * seriation.h -- C ABI of libseriation.so, the MI355X-native drop-in for the reference's
 * per-chain MCMC sweep (PrayagS/Seriation-in-Paleontological-Data-using-MCMC,
 * C_Implementation/mcmc.c).  Plain C types only; caller-owned buffers; every function
 * returns SR_OK (0) or a negative SR_E* code -- the library never calls exit().
 *
 * Reference interfaces replaced (file:line in the reference tree):
 *   sr_parse_dataset / sr_load_dataset   mcmc_readmodel            mcmc.c:339-437, mcmc.h:47
 *   sr_run_chains / sr_session_*         mcmc_init + mcmc_randomize + mcmc_sample loop
 *                                         mcmc.c:127-185, 214-258, 477-593, mcmc.h:48,51,55
 *   sr_chain_summary.exp_*               compute_exp_data / print_exp_data  mcmc.c:53-67
 *   sr_record / sink                     mcmc_save_chain           mcmc.c:69-92
 *   sr_run_to_dirs                       main()'s Chains/chain_XX/<name>.csv output  mcmc.c:148-197, 261-293
 *   sr_chain_summary.consistent          mcmc_consistent           mcmc.c:999-1094, 199-204
 *   sr_chain_spec.seed                   GSL_RNG_SEED via gsl_rng_env_setup  mcmc.c:591 / script.py:42
 * A chain's trajectory depends only on (dataset, seed): sharding chains over devices or
 * sessions never changes any chain's output.
 */
#ifndef SERIATION_H
#define SERIATION_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define SR_OK 0
#define SR_EINVAL (-1)         /* bad argument */
#define SR_EPARSE (-2)         /* "mcmc_readmodel: read error." (mcmc.c:349, 371) */
#define SR_EHEADER (-3)        /* "mcmc_readmodel: read error at header." (mcmc.c:355) */
#define SR_ENOMEM (-4)
#define SR_EDEVICE (-5)        /* HIP runtime error or no gfx950 device */
#define SR_EUNSUPPORTED (-6)   /* configuration outside the kernel's limits */
#define SR_EIO (-7)            /* cannot open/write an output file */
#define SR_EINCONSISTENT (-8)  /* mcmc_consistent failed after the run (mcmc.c:199-204) */

#define SR_MAXS 2000           /* mcmc.h:25 line limit of the reference parser */

typedef struct {
  int32_t N, M, nh;   /* sites, taxa, hard sites */
  uint8_t *X;         /* N*M, row-major (row = site), 0/1 */
  uint8_t *hard;      /* N, 1 if the row ended with '*' */
} sr_dataset;

/* maxs = SR_MAXS reproduces the reference's fgets(MAXS) semantics exactly (a longer line
 * is split and its tail read as the next row); maxs = 0 reads lines of any length. */
int sr_parse_dataset(const char *text, size_t len, int32_t maxs, sr_dataset *out);
int sr_load_dataset(const char *path, int32_t maxs, sr_dataset *out);
void sr_free_dataset(sr_dataset *ds);
/* Binary bit-packed form ("SRBX" header, N hard bytes, N rows of ceil(M/8) bytes; SURVEY §8f-4,
 * an extension: the reference reads text only).  sr_load_dataset also accepts it (by magic). */
int sr_save_dataset_bin(const sr_dataset *ds, const char *path);
int sr_load_dataset_bin(const char *path, sr_dataset *out);

typedef struct {
  int32_t chain_id;   /* names the output directory Chains/chain_NN */
  uint64_t seed;      /* GSL_RNG_SEED value (0 -> GSL default 4357) */
} sr_chain_spec;

typedef struct {
  int32_t burnin_calls;      /* tb: mcmc_sample calls before saving (mcmc.c:107, default 1000) */
  int32_t sample_calls;      /* ts: saved mcmc_sample calls (default 1000) */
  int32_t sweeps_per_call;   /* sweeps per mcmc_sample (mcmc.c:225, default 10) */
  int32_t manycd;            /* mcmc_readmodel's manycd (mcmc.h:40, mcmc.c:118): 0 = c, d shared by all taxa (the
                                reference CLI's default and script.py's); nonzero = per-taxon c[m], d[m] drawn one
                                after another each sweep (mcmc.c:777-786, 807-816) -- the exact (slower) kernel
                                paths, block_threads 0 or 1024 */
  int32_t device;            /* HIP device ordinal */
  int32_t block_threads;     /* threads per chain workgroup, 0 = auto */
  int32_t calls_per_launch;  /* mcmc_sample calls per kernel launch, 0 = auto */
  int32_t flags;             /* SR_F_* */
} sr_run_opts;
#define SR_F_NO_CHECK 1      /* skip the closing mcmc_consistent check */
#define SR_F_HBM_COLUMNS 2   /* force the HBM-column kernel variant (default: only when LDS is too small) */
#define SR_F_LDS_COLUMNS 4   /* force the LDS-column variant (SR_EUNSUPPORTED if it does not fit) */
#define SR_F_DEBUG_CHECK 8   /* the reference's MCMCDEBUG (mcmc.c:249-255): mcmc_consistent on every chain after
                                every mcmc_sample call (one call per launch); SR_EINCONSISTENT on the first failure */
#define SR_F_DEBUG_PRINT 16  /* with SR_F_DEBUG_CHECK: MCMCDEBUG's acceptance-rate line on stderr per chain and call */
#define SR_F_RNG_PHILOX 32   /* opt-in: the sampling phase draws every word from a counter-based Philox4x32-10 stream
                                keyed by the chain's seed instead of GSL's MT19937 (initialisation unchanged).  Not
                                the reference's stream: statistically equivalent, not bit-equal.  A checkpoint
                                keeps its stream kind; restoring it needs the same flag (else SR_EINVAL). */
#define SR_F_DIAG 64         /* the reference's stderr diagnostics during initialisation: "mcmc_initab: zero column
                                at %d, continuing." per all-zero column, from mcmc_readmodel's and mcmc_randomize's
                                mcmc_initab (mcmc.c:457); the drop-in CLI sets it */
#define SR_F_GENERIC_KERNEL 128  /* run the generic sweep kernel (shape from the launch arguments) instead of the
                                    default shape-specialised one (sr_session_specialized); SR_JIT=0 in the
                                    environment does the same.  Results are identical either way. */

typedef struct {
  int32_t chain_id;
  int32_t consistent;        /* 0 = mcmc_consistent passed (as the reference's exit 0) */
  double exp_loglik, exp_c, exp_d;   /* exactly print_exp_data's values (sums / 1000) */
} sr_chain_summary;

typedef struct {
  int32_t N, M;
  const int32_t *a, *b, *pi;  /* M, M, N: one mcmc_save_chain line */
  double c, d, loglik;        /* log P(false 1), log P(false 0) (manycd: taxon 0's), loglik */
  const double *cv, *dv;      /* manycd: every taxon's c[M], d[M]; NULL when all taxa share c, d */
} sr_record;

/* Called once per saved sample, per chain in sample order; return nonzero to abort. */
typedef int (*sr_sample_sink_fn)(void *ctx, int32_t chain_index, int32_t sample_index,
                                 const sr_record *rec);

void sr_default_opts(sr_run_opts *o);

/* gsl_rng_env_setup (mcmc_init, mcmc.c:591-592; GSL 2.6 rng/env.c) for callers that take the seed from the
 * environment as the reference CLI does: GSL_RNG_TYPE unset or "mt19937" -> SR_OK (verbose: the line
 * "GSL_RNG_TYPE=mt19937" when set), then GSL_RNG_SEED (strtoul base 0, unset -> 0 = GSL's default 4357;
 * verbose: "GSL_RNG_SEED=<value>") into *seed.  Another GSL generator -> SR_EUNSUPPORTED (the sampler
 * implements MT19937's stream only), a name GSL does not know -> SR_EINVAL (verbose: GSL's "not recognized"
 * message and list of generator types).  Every session / run entry point that samples MT19937's stream
 * applies the same GSL_RNG_TYPE check (silently) and refuses with the same codes, so no run samples MT19937
 * where the environment named another generator; SR_F_RNG_PHILOX sessions sample no GSL stream and ignore it.
 * Departure: for an unknown name GSL 2.6 prints the list, then its default error handler reports "unknown
 * generator" and aborts (SIGABRT); here the caller gets SR_EINVAL and the CLIs exit 1 (parity unpinned: no GSL
 * here to take the handler's exact line from). */
int sr_rng_env_setup(uint64_t *seed, int32_t verbose);

/* Run n_chains independent chains on one GPU (opts->device), burn-in then sampling;
 * per-sample records go to sink (may be NULL); out[n_chains] receives the summaries. */
int sr_run_chains(const sr_dataset *ds, const sr_chain_spec *specs, int32_t n_chains,
                  const sr_run_opts *opts, sr_sample_sink_fn sink, void *sink_ctx,
                  sr_chain_summary *out);

/* Same run, writing Chains/chain_NN/{chain_data,exp_data,taxa,sites,hard_sites}.csv
 * under chains_root byte-for-byte as the reference's main() does. */
int sr_run_to_dirs(const sr_dataset *ds, const sr_chain_spec *specs, int32_t n_chains,
                   const sr_run_opts *opts, const char *chains_root, sr_chain_summary *out);

/* Several GPUs from one call (the reference runs one process per chain, script.py:55-62):
 * chains sharded contiguously over n_devices shards, shard k on HIP device devices[k] (an ordinal may
 * repeat: those shards share the GPU), one host thread per shard.  Every output equals the
 * sr_run_chains / sr_run_to_dirs one; the sink is serialised and receives global chain indices
 * (samples in order per chain, chains of different shards interleaved).  opts->device is ignored. */
int sr_run_chains_multi(const sr_dataset *ds, const sr_chain_spec *specs, int32_t n_chains,
                        const sr_run_opts *opts, const int32_t *devices, int32_t n_devices,
                        sr_sample_sink_fn sink, void *sink_ctx, sr_chain_summary *out);
int sr_run_to_dirs_multi(const sr_dataset *ds, const sr_chain_spec *specs, int32_t n_chains,
                         const sr_run_opts *opts, const int32_t *devices, int32_t n_devices,
                         const char *chains_root, sr_chain_summary *out);

/* ---- sessions: chains resident in HBM on one GPU, asynchronous launches ---- */
typedef struct sr_session sr_session;
int sr_session_create(const sr_dataset *ds, const sr_chain_spec *specs, int32_t n_chains,
                      const sr_run_opts *opts, sr_session **out);
/* Launch on a caller-owned hipStream_t (e.g. torch.cuda.current_stream().cuda_stream). */
int sr_session_set_stream(sr_session *s, void *hip_stream);
/* Enqueue `calls` mcmc_sample calls for every chain; save != 0 appends one record per call. */
int sr_session_run(sr_session *s, int32_t calls, int32_t save);
int sr_session_sync(sr_session *s);
int32_t sr_session_records(const sr_session *s);
int32_t sr_session_record_capacity(const sr_session *s);
/* ab_pi: [n_chains][count][2M+N] int16 (a, b, pi); cdl: [n_chains][count][3] (c, d, loglik);
   either may be NULL (not fetched) */
int sr_session_fetch_records(sr_session *s, int32_t first, int32_t count, int16_t *ab_pi, double *cdl);
int sr_session_reset_records(sr_session *s);
/* One chain's buffered records [first, first + count): ab_pi [count][2M+N] int16, cdl [count][3]
   (either may be NULL). */
int sr_session_fetch_chain_records(sr_session *s, int32_t chain, int32_t first, int32_t count, int16_t *ab_pi,
                                   double *cdl);
/* The same rows copied device to device into caller-owned memory on the session's GPU (dev_ab_pi [count][2M+N]
   int16, dev_cdl [count][3]; either may be NULL), queued on the session stream without waiting: the records
   never leave HBM (e.g. straight into the buffer of an RCCL all-gather on that stream). */
int sr_session_copy_chain_records(sr_session *s, int32_t chain, int32_t first, int32_t count, int16_t *dev_ab_pi,
                                  double *dev_cdl);
/* manycd sessions: the per-taxon c, d of buffered records [first, first + count): cdv [n_chains][count][2M]
   (c[M] then d[M], log values as mcmc_save_chain exponentiates them); SR_EINVAL for manycd = 0 sessions. */
int sr_session_fetch_cd_vectors(sr_session *s, int32_t first, int32_t count, double *cdv);
int32_t sr_session_manycd(const sr_session *s);
/* compute_exp_data / print_exp_data (mcmc.c:53-67) of every chain over its buffered records [first,
   first + count): out[c] = {chain_id, 0, sum(-loglik) / 1000, sum(e^c) / 1000, sum(e^d) / 1000}, sums in
   sample order, the reference's hard-coded divisor (exact means when count = 1000). */
int sr_session_summaries(sr_session *s, int32_t first, int32_t count, sr_chain_summary *out);
/* Current state of one chain (any pointer may be NULL); counts = t0,f0,t1,f1 (4*M). */
int sr_session_state(sr_session *s, int32_t chain, int32_t *a, int32_t *b, int32_t *pi,
                     double *c_d_loglik, int32_t *counts);
/* manycd sessions: one chain's current per-taxon c[M], d[M] (log values; either may be NULL); SR_EINVAL for
   manycd = 0 sessions (their c, d are sr_session_state's). */
int sr_session_state_cd(sr_session *s, int32_t chain, double *c, double *d);
/* Acceptance counters cc, cd, cab, cpi1, cpi20, cpi21, cpi3 (mcmc.c:220). */
int sr_session_accept_counts(sr_session *s, int32_t chain, int64_t *acc7);
/* How often the fast paths fell back to the reference's own computation (no counterpart in
   mcmc.c; every fallback is bit-exact): fb3 = {proposals decided by the exact sequential delta,
   Gibbs draws by the exact three-pass walk, c/d draws by the sequential GSL path}. */
int sr_session_fallback_counts(sr_session *s, int32_t chain, int64_t *fb3);
/* SR_F_DEBUG_CHECK: 1 if the chain failed mcmc_consistent after some mcmc_sample call of this
   session (the check of mcmc.c:254; sticky), 0 if not or without the flag. */
int sr_session_debug_flagged(const sr_session *s, int32_t chain);
/* Device time of the last sr_session_run (ms, HIP events on the session stream; syncs). */
double sr_session_last_kernel_ms(sr_session *s);
int32_t sr_session_block_threads(const sr_session *s);
/* Kernel variant the session runs: 0 = occurrence columns in LDS, one thread per taxon; 1 = columns
 * in HBM (chosen when the LDS layout exceeds 160 KB, e.g. 1024 sites x 2048 taxa); 2 = columns in
 * LDS, two lanes per taxon (the pair kernel: walks of <= 9 words and 257..512 taxa; opt-in with
 * SR_KERNEL=pair in the environment and block_threads unset -- slower than variant 0);
 * 3 = columns in HBM, split chains: two co-resident workgroups per chain, each owning half of the
 * taxa (1024 threads, 1025..2048 taxa, grid co-resident; SR_SPLIT=0 in the environment disables it). */
int32_t sr_session_variant(const sr_session *s);
/* 1 when the session's launches use the sweep kernel compiled for its exact shape (sites, taxa, hard
 * sites fixed at compile time) -- the default for sessions with occurrence columns in LDS (variant 0) --
 * 0 for the generic kernel (HBM columns, the pair kernel, SR_F_GENERIC_KERNEL / SR_JIT=0, or the
 * specialised code object unavailable: one stderr line says why).  Results are identical either way. */
int32_t sr_session_specialized(const sr_session *s);
/* Prepare the shape-specialised kernel a session of this dataset and opts (block_threads, SR_F_*_COLUMNS,
 * SR_F_GENERIC_KERNEL) would run, without a GPU: compiled from the source snapshot the library was built
 * from (build/spec/) with hipcc into the cache ($SR_JIT_CACHE, else build/jit/ next to the library), so
 * that session creation finds it.  1 ready, 0 the session runs no specialised kernel, SR_EIO the code
 * object could not be produced (stderr says why), SR_EUNSUPPORTED / SR_EINVAL as sr_session_create.
 * (Session creation compiles a missing shape itself unless SR_JIT=cache: then only embedded or cached objects
 * are used and any other shape runs the generic kernel -- no compiler is spawned at run time.) */
int sr_specialize(const sr_dataset *ds, const sr_run_opts *opts);
/* Checkpoint / resume (the reference has none): the full chain state (columns, pi,
   limits, counts, c/d/loglik, MT19937 ring and cursor, acceptance counters) and the session's buffered
   records to a file; restoring it over the same dataset continues every chain exactly where it stopped,
   with the records in the new session's buffer (its capacity: the larger of opts->calls_per_launch and the
   record count), so summaries over a resumed sampling phase equal an uninterrupted run's.  Files without
   records (versions 3 / 4, before round 5) still restore, with an empty record buffer. */
int sr_session_checkpoint(sr_session *s, const char *path);
int sr_session_restore(const sr_dataset *ds, const char *path, const sr_run_opts *opts, sr_session **out);
void sr_session_destroy(sr_session *s);

/* ---- posterior summaries over saved samples, on the GPU ----
 * Replace the per-sample loops of the reference's analysis script (script.py):
 *   pair_order  [N][N]  compute_pair_order_matrix / generate_po_matrix   script.py:155-189
 *   alive       [N][M]  X_sum of plot_taxa_occurence_probability_matrix  script.py:306-333
 *   false_alive [N][M]  X_sum of plot_false_taxa_occurence_probability   script.py:350-377
 *   false_ones  [N][M]  X_sum of plot_false_ones_probability             script.py:392-417
 *   exp_pi      [N]     compute_exp_pi                                   script.py:230-251
 *   exp_a       [M]     compute_exp_a                                    script.py:254-275
 * bit for bit, quirks included (per-chain accumulators never reset, the fixed /1000, the
 * [site][taxon] loops comparing the site index with the limits); the argsort reorderings that
 * follow in the script are left to the caller.  NULL outputs are skipped; kernel_ms receives
 * the summed device time.  Samples are mcmc_save_chain rows (a, b, pi with pi[site] = position). */
typedef struct {
  double *pair_order, *alive, *false_alive, *false_ones, *exp_pi, *exp_a;
  double kernel_ms;
} sr_posterior_out;
/* ab_pi: [n_sel][count][2M+N] int16 host rows, chains in selection order; ds supplies N, M, X. */
int sr_posterior(const sr_dataset *ds, const int16_t *ab_pi, int32_t n_sel, int32_t count,
                 int32_t chains_selected, int32_t device, sr_posterior_out *out);
/* The session's own records in HBM (no host round trip): chains[n_sel] are session chain
 * indices in selection order, samples [first, first + count) of its record buffer. */
int sr_session_posterior(sr_session *s, const int32_t *chains, int32_t n_sel, int32_t first, int32_t count,
                         int32_t chains_selected, sr_posterior_out *out);

const char *sr_strerror(int code);
int sr_device_count(void);
const char *sr_version(void);

#ifdef __cplusplus
}
#endif
#endif
