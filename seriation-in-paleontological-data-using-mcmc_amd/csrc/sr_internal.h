/*
 * sr_internal.h -- interface between the C host layer (sr_host.c) and the HIP device
 * layer (sr_device.hip).  Plain C.
 */
#ifndef SR_INTERNAL_H
#define SR_INTERNAL_H
#include <stdint.h>
#include <stddef.h>

#define SR_NHMAX 64      /* hard sites of the mask paths (a 64-bit mask per taxon, one hard site per lane); more
                            hard sites take the bitmap paths (any number up to N) */
/* hard positions stored per chain: 64, or nh rounded up to whole waves */
#define SR_NHCAP(nh) ((nh) <= SR_NHMAX ? SR_NHMAX : (((nh) + 63) & ~63))
#define SR_RING 8        /* MT19937 blocks resident per chain */
#define SR_MMAX (1 << 20)   /* taxa per dataset (int32 indices; per-chain columns and records grow with M) */

/* Per-chain state in HBM, struct-of-arrays over chains.  Layout (per chain c):
 *   P   [NW][M] u32  position-ordered occurrence columns: bit (p&31) of P[p>>5][m]
 *                    = X[rpi[p]][m]  (the column of taxon m in current site order)
 *   rpi [N]     i32  site at each position (gsl_permutation rpi, mcmc.h:37)
 *   hp  [NHMAX] i32  positions of the hard sites, ascending (hard order is invariant)
 *   ab  [2][M]  i32  a, b (mcmc.h:36)
 *   cnt [4][M]  i32  t0, f0, t1, f1 (mcmc.h:42)
 *   cdl [4]     f64  c, d, loglik, unused
 *   mt  [RING][624] u32, rng [2] u64 (pos, gen), acc [8] u64                       */
/* per-chain counters: [0..6] acceptances cc, cd, cab, cpi1, cpi20, cpi21, cpi3 (mcmc.c:220),
 * [7] proposals decided by the exact sequential delta, [8] Gibbs draws taken by the exact
 * three-pass walk, [9] c/d draws taken by the sequential GSL path (the fast paths' fallbacks) */
#define SR_NACC 10

typedef struct {
  int N, M, NW, nh, nchains;
  uint32_t *P;
  int32_t *rpi, *hp, *ab, *cnt;
  double *cdl;
  uint32_t *mt;
  uint64_t *rng, *acc;
  int manycd;         /* 1: per-taxon c, d (mcmc.h:40 manycd) */
  double *cdv;        /* manycd: [nchains][2M] c[M], d[M] (NULL otherwise) */
} sr_state_host;

typedef struct srk_dev srk_dev;

#ifdef __cplusplus
extern "C" {
#endif

/* shape-specialised kernels (sr_spec.c): the code object of sr_sweep_kernel<TB, NWM, false> compiled with
 * SR_FN = N, SR_FM = M, SR_FH = NH (and SR_FORCE_EXACT when force) */
typedef struct { int TB, NWM, N, M, NH, force; } sr_spec_shape;
#define SR_SPEC_ENOSRC (-1)
#define SR_SPEC_ESTALE (-2)
#define SR_SPEC_ENOCC (-3)
#define SR_SPEC_ECC (-4)
#define SR_SPEC_EPROF (-5)
#define SR_SPEC_ELOAD (-6)
#define SR_SPEC_ECACHE (-7)
#define SR_SPEC_ENOJIT (-8)   /* not embedded, not cached, and run-time compiles are off (SR_JIT=cache) */
/* the cache path of the shape's code object (0), or a reason code */
int sr_spec_path(const sr_spec_shape *s, char *path, size_t len);
/* the path of the shape's code object, compiled into the cache first if it is missing (0), or a reason;
   announce: one stderr line when a compile starts (session creation: it can take seconds) */
int sr_spec_object(const sr_spec_shape *s, char *path, size_t len, int announce);
/* Code objects embedded in libseriation.so at build time (the shapes of csrc/sr_embed_shapes.txt, compiled by
   build/srembed; build/sr_emb.c holds the table).  Weak and hidden: builds without the table (test variants,
   the build tools) find none. */
typedef struct { int TB, NWM, N, M, NH, force; const unsigned char *begin, *end; } sr_spec_emb;
/* the embedded code object of this shape (*bytes its size), or NULL */
const void *sr_spec_embedded(const sr_spec_shape *s, size_t *bytes);
const char *sr_spec_reason(int code);
/* one stderr line per reason and process: the session falls back to the generic kernel */
void sr_spec_note(int code, const char *detail);

int srk_device_count(void);
/* gm_force: -1 auto (LDS columns when they fit, else HBM columns), 0 LDS, 1 HBM;
 * pkey: [nchains][2] Philox keys (the SR_F_RNG_PHILOX stream), NULL = MT19937 */
/* spec: 1 the shape-specialised kernel when the session runs LDS columns (sr_spec.c; the default),
 * 0 the generic kernel (SR_F_GENERIC_KERNEL, or SR_JIT=0 in the environment) */
int srk_create(const sr_state_host *st, int device, int block_threads, int rec_cap_calls, int gm_force,
               const uint32_t *pkey, int spec, srk_dev **out);
/* the kernel a session of this shape would run, without a GPU: *lds_cols 1 for LDS columns, *shape the
 * specialised kernel's shape (valid when the function returns 1); 0 no specialised kernel (HBM columns,
 * pair kernel), negative: unsupported */
int srk_plan(int N, int M, int nh, int block_threads, int gm_force, int manycd, sr_spec_shape *shape);
int srk_set_stream(srk_dev *d, void *stream);
/* calls*spc sweeps for all chains; save -> records appended at slot rec_base.. */
int srk_run(srk_dev *d, int calls, int spc, int save, int rec_base);
int srk_sync(srk_dev *d);
double srk_last_ms(srk_dev *d);
int srk_block_threads(const srk_dev *d);
int srk_variant(const srk_dev *d);   /* 0 LDS columns, 1 HBM columns */
int srk_specialized(const srk_dev *d);   /* 1: the run-time specialised kernel */
int srk_fetch_dbg(srk_dev *d, unsigned long long *out);
int srk_fetch_records(srk_dev *d, int first, int count, int16_t *ab_pi, double *cdl);
/* per chain {sum -loglik, sum exp(c), sum exp(d)} over record rows [first, first + count) (compute_exp_data) */
int srk_exp_data(srk_dev *d, int first, int count, double *sums);
int srk_fetch_chain_records(srk_dev *d, int chain, int first, int count, int16_t *ab_pi, double *cdl);
/* the same rows copied device to device into memory on the session's GPU, queued on the session stream */
int srk_copy_chain_records(srk_dev *d, int chain, int first, int count, int16_t *ab_pi, double *cdl);
int srk_download_state(srk_dev *d, sr_state_host *st);
/* consume's last argument: manycd sessions' per-taxon c, d rows [nchains][count][2M], else NULL */
int srk_run_pipelined(srk_dev *d, int total_calls, int cpl, int spc,
                      int (*consume)(void *, int, int, const int16_t *, const double *, const double *), void *ctx);
/* manycd: per-taxon c, d of record rows [first, first + count), [nchains][count][2M] */
int srk_fetch_cdv(srk_dev *d, int first, int count, double *cdv);
/* record rows [0, count) of every chain uploaded (checkpoint restore); cdv only for manycd sessions */
int srk_upload_records(srk_dev *d, int count, const int16_t *ab_pi, const double *cdl, const double *cdv);
/* the session's record buffer in HBM: [nchains][rec_cap][2M+N] int16 */
int srk_records_device(srk_dev *d, const int16_t **rec, int *rec_cap, int *device, void **stream);

/* posterior summaries (sr_post.hip); kinds = SR_POST_* bit positions */
#define SRP_PAIR_ORDER 0
#define SRP_ALIVE 1
#define SRP_FALSE_ALIVE 2
#define SRP_FALSE_ONES 3
#define SRP_EXP_PI 4
#define SRP_EXP_A 5
int srp_posterior_dev(int device, void *stream, int kind, const int16_t *d_rec, const long long *chain_off, int n_sel,
                      int count, long long row_stride, int N, int M, const uint8_t *X_host, int chains_selected,
                      double *out_host, float *ms);
int srp_posterior_host(int device, int kind, const int16_t *ab_pi, int n_sel, int count, int N, int M,
                       const uint8_t *X_host, int chains_selected, double *out_host, float *ms);
void srk_destroy(srk_dev *d);

#ifdef __cplusplus
}
#endif

#endif
