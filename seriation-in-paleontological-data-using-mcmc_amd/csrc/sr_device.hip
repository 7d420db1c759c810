/*
 * sr_device.hip -- the MI355X (gfx950) sweep kernel and the device session layer.
 *
 * One workgroup = one chain; one thread owns taxa m = tid + k*TB (k < TPT).  Everything a
 * sweep touches lives on chip for the whole launch:
 *   registers: per-taxon a, b, t0, f0, t1, f1 (owned taxa); the hard-site positions
 *              (uniform); c, d, log(1-e^c), log(1-e^d); RNG cursor (uniform)
 *   LDS:       P[w][m]  -- the occurrence matrix in CURRENT site order, one bit column per
 *                          taxon (column m is private to its owner thread, so the Gibbs
 *                          update and every proposal read it without synchronisation)
 *              rpi (double-buffered), the MT19937 ring (8 x 624 words), exp/log tables,
 *              per-taxon term buffers for the ordered sums.
 * HBM is touched only to load/store the chain state at launch boundaries and to append
 * the saved samples (records), so the kernel is latency/VALU-bound, not HBM-bound.
 *
 * Reference mapping (C_Implementation/mcmc.c):
 *   sweep()            mcmc_sample body            :225-244
 *   draw_c_d (wave 0)  mcmc_samplec/_sampled/_samplebeta :751-825 (+ GSL beta/gamma/zig)
 *   sampleab           mcmc_sampleab/_auxa/_logtop/_randompick :711-748, 828-996
 *   prop_pi1/2/3       mcmc_samplepi1/2/3          :1127-1682
 *   logl_wave0         mcmc_logl                   :625-648
 * Bit-exactness: every floating-point expression is evaluated in the reference's order
 * (-ffp-contract=off); sums that the reference does sequentially (logl, logtop, the
 * proposal deltas, randompick) are done sequentially (the ordered sums run on one wave;
 * runs of clamped logtop terms use the exact closed form in sr_math.h).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <type_traits>
#define SR_TABLES_NO_ARRAYS
#include "sr_tables.h"
#include "sr_math.h"
#include "sr_rng.h"
#include "sr_internal.h"
#include "seriation.h"

__constant__ double c_zig_y[128] = SR_ZIG_YTAB_INIT;
__constant__ unsigned int c_zig_k[128] = SR_ZIG_KTAB_INIT;
__constant__ double c_zig_w[128] = SR_ZIG_WTAB_INIT;
__constant__ uint64_t c_exp_tab[256] = SR_EXP_TAB_INIT;
__constant__ double c_log_tab[256] = SR_LOG_TAB_INIT;

#define SR_ZIGR 3.44428647676   /* GSL gaussian_ziggurat PARAM_R */

/* Shape specialisation (the session's kernel compiled for its shape, sr_spec.c): SR_FN / SR_FM / SR_FH fix the
 * dataset's sites, taxa and hard sites at compile time, so the layout offsets, strides, loop bounds and
 * the uniform_int divisors fold into immediates (the generic kernel holds them in ~600 spilled SGPRs).
 * 0 / 0 / -1 (the default): taken from the launch arguments. */
#ifndef SR_FN
#define SR_FN 0
#endif
#ifndef SR_FM
#define SR_FM 0
#endif
#ifndef SR_FH
#define SR_FH (-1)
#endif

struct KArgs {
  int N, M, NW, nh, nchains;
  int calls, spc, save, rec_base, rec_cap;
  uint32_t *P;
  int32_t *rpi, *hp, *ab, *cnt;
  double *cdl;
  uint32_t *mt;
  uint64_t *rng, *acc;
  int16_t *rec_abpi;
  double *rec_cdl;
  unsigned long long *dbg;   /* SR_STAMPS builds: [chain][16] cycles per phase */
  uint16_t *gpre;            /* gm variant scratch, per chain: column prefix tables */
  uint32_t *pkey;            /* [chain][2] Philox keys (SR_F_RNG_PHILOX), else null: MT19937 */
  void *gck;                     /* gm variant scratch: Gibbs checkpoints (SR_CK32: f32, half the bytes of the scratch stream;
                                    unused by the split kernels, whose checkpoints are in LDS: SR_SP_LCK) */
  double *glbuf, *gcbuf;         /* gm variant scratch: logl terms, exact-delta terms */
  int *xflag, *xbuf, *xerr;      /* split chains (SP kernels): [chain][2] progress flags, exchange slots, timeout flag */
  double *cdv, *cdx;   /* manycd (MCD kernels): [chain][2M] per-taxon c, d (state); [chain][2M] their cc, dd (scratch) */
  double *rec_cdv;     /* manycd: [chain][rec_cap][2M] per-taxon c, d of every saved sample */
};

/* The launch arguments re-read from the kernarg segment (constant for the launch; the kernel's only
 * argument is KArgs, at offset 0): the record and state pointers used after the sweeps come from here, so
 * they are not held live (in spilled SGPRs) across the sweep loop.  SR_KARG_RELOAD=0: the by-value copy. */
/* HBM-column kernels: Gibbs checkpoints stored as f32 (1) or f64 (0) in their HBM scratch (draw_fast).
   f32 halves the scratch stream but is rejected (r04c/r04d, same box): the certification's absolute slack
   must then grow to 2^-21 S, and an entry with less mass than twice the slack can never be certified, so
   u landing in the window's many small-mass entries sends ~1.3e-4 of the draws to the exact walk (0.52
   per chain-sweep against 0.0025 in f64): config 5 ran 2.3x slower (10.45 vs 4.56 ms per launch). */
#ifndef SR_CK32
#define SR_CK32 0
#endif
/* HBM-column kernels: window words per stored Gibbs checkpoint (pass 2 re-sums the chosen group's words in
   one round trip; 4 measured fastest: 4.56 / 4.44 / 4.39 ms per config-5 launch at 1 / 2 / 4, r04e-r04f) */
#ifndef SR_CKG
#define SR_CKG 4
#endif
/* split-chain kernels (SP): the Gibbs checkpoints in LDS ((N/32)/SR_CKG + 1 slots per thread) instead of HBM
   scratch, room made by one block-shared copy of the hard-site and 4-step tables instead of one per wave
   (16 waves: 66 KB + 20 KB at N = 1024).  The checkpoints were a quarter of config 5's HBM traffic (all of its
   writes) and two dependent memory round trips of every walk's pass 2 (0 = HBM scratch, round 4's form) */
/* test builds: every certification margin -- the Gibbs picks' REL / ABS (draw_fast, walk_pick_s, draw_pair9) and
   phase C's Eb (pc_classify) -- scaled by 2^-SR_CERT_SHIFT.  The product is 0; the negative control of
   tests/test_gpu_cert.py builds the library at 8 and must then see wrong picks and decisions, which shows that the
   self-tests (sr_device_selftest_gibbs / _decide) can see an understated bound. */
#ifndef SR_CERT_SHIFT
#define SR_CERT_SHIFT 0
#endif
#define SR_CERT_SCALE (1.0 / (double)(1ull << SR_CERT_SHIFT))
#ifndef SR_SP_LCK
#define SR_SP_LCK 1
#endif
/* split kernels whose LDS layout has room (LK): the own half's column prefix table in LDS (stride = the half's
   taxa) and the Gibbs checkpoints in HBM scratch, instead of the checkpoints in LDS and the prefixes in HBM: the
   prefixes are read several times per proposal and taxon, the checkpoints once per walk, and the L2 holds the
   columns of 25 half-chains per XCD (config 5: 4.208 -> 4.151 ms per launch, profiles/r06u_ab_c5_lpre.json) */
#ifndef SR_SP_LPRE
#define SR_SP_LPRE 1
#endif
/* HBM-column kernels: one block-shared copy of the hard-site and 4-step tables (16 waves at 1024 threads held 64 N
   bytes of per-wave hard tables: at N ~ 1250 the layout passed 160 KB; shared, N reaches 4095 at 1024 threads) */
#ifndef SR_GM_SHARED
#define SR_GM_SHARED 1
#endif
/* the sweep's proposal tables filled by all threads before the phase-A barrier, and the swap drawn from them
   (round 5; 0 = each wave fills its own at the start of phase C and the swap takes the scalar path) */
#ifndef SR_COOP_TABLES
#define SR_COOP_TABLES 1
#endif
/* the register form of an accepted pi1 in the HBM-column kernels too (off: in round 5 its registers spilled 37 more
   VGPRs there, r05l) */
#ifndef SR_GM_APPLY_REG
#define SR_GM_APPLY_REG 0
#endif
/* the proposal sums of a batch of at least this many proposals by one transposed reduction per wave
   (wave_sum32_t; 0 = one reduction per slot) */
#ifndef SR_TSUMS
#define SR_TSUMS 4
#endif
/* diagnostic builds (tools/build_variant.sh): SR_DOUBLE = k does phase k's work twice, the second result folded
   in through an opaque zero (the chain is unchanged), so the time difference is the phase's marginal cost:
   1 proposal terms, 2 proposal sums, 3 Gibbs draws, 4 the c, d draws, 5 K and the step tables, 7 the sweep's
   table fill, 8 the hard-site tables after a hard site moved */
#ifndef SR_DOUBLE
#define SR_DOUBLE 0
#endif
__device__ __forceinline__ int sr_opaque_zero()
{
  int z;
  __asm__ volatile("s_mov_b32 %0, 0" : "=s"(z));
  return z;
}
/* the swap drawn into one batch with proposals 1..15 (its acceptance, ~44 %, then wastes their terms) */
#ifndef SR_MERGE_SWAP
#define SR_MERGE_SWAP 1
#endif
#ifndef SR_MERGE_SWAP_GM   /* ... also in the HBM-column kernels (their proposal terms cost far more) */
#define SR_MERGE_SWAP_GM 0
#endif
/* the c, d draws' ziggurat steps read before the phase-A barrier (measured +0.5 %: off, r05q) */
#ifndef SR_CD_PREFETCH
#define SR_CD_PREFETCH 0
#endif
/* pi1's taxon change by one unsigned compare per limit */
#ifndef SR_PI1_FAST
#define SR_PI1_FAST 1
#endif
/* the per-lane "owns a taxon" test as a constant in shape-specialised kernels whose taxa fill the block */
#ifndef SR_OWN_CONST
#define SR_OWN_CONST 1
#endif
/* at most this many proposals per batch (a smaller batch wastes fewer evaluations after an accepted proposal,
   at the cost of more batches) */
#ifndef SR_BATCH_MAX
#define SR_BATCH_MAX 16
#endif
/* ininterval as one unsigned range compare per lane */
#ifndef SR_ININT_FAST
#define SR_ININT_FAST 1
#endif
/* an accepted pi1 applied from registers: the taxon's words, moved bit and prefix read before any write */
#ifndef SR_APPLY_REG
#define SR_APPLY_REG 1
#endif
/* the main batch's proposal slots without per-slot branches (one-taxon kernels) */
#ifndef SR_FULL_BATCH
#define SR_FULL_BATCH 0
#endif
/* branch-free proposal terms (taxon_dt: no exec-mask branches, indices clamped, results selected) */
#ifndef SR_BF_TERMS
#define SR_BF_TERMS 0
#endif
#ifndef SR_KARG_RELOAD
#define SR_KARG_RELOAD 0
#endif
__device__ __forceinline__ const KArgs &kargs_late(const KArgs &A)
{
#if SR_KARG_RELOAD
  (void)A;
  const KArgs *p = (const KArgs *)__builtin_amdgcn_kernarg_segment_ptr();
  __asm__ volatile("" : "+s"(p));   /* an opaque pointer: the loads stay here, after the loop */
  return *p;
#else
  return A;
#endif
}

/* ---------------------------------------------------------------- LDS carve */
struct Lay {
  size_t tab, cbuf, lbuf, mt, P, rpi0, rpi1, ht, ck, ccnt, sab, scnt, hpw, hbw, t4, t8, pre, part, tot, xs, ptab, misc, total;
};
__host__ __device__ static constexpr inline size_t sr_al16(size_t x) { return (x + 15) & ~(size_t)15; }
/* walk words held in registers by the register-column kernels (NWM template argument): 9 for
 * N <= 287, 17 for N <= 543, else 0 (columns walked in LDS, Gibbs checkpoints in LDS) */
__host__ __device__ static constexpr inline int sr_nwm(int N) { const int nk = (N >> 5) + 1; return nk <= 9 ? 9 : (nk <= 17 ? 17 : 0); }
/* the register-column kernels exist for TB 256 and 512 (LDS columns only) */
/* (and their 32-bit hard-site masks: more than 32 hard sites take the LDS-walk kernels, 64-bit masks;
 * one taxon per thread, M <= TB: the several-taxa branches are compiled out of them) */
__host__ __device__ static constexpr inline bool sr_regwalk(int N, int M, int TB, bool gm, int nh)
{
  return !gm && TB <= 512 && M <= TB && sr_nwm(N) > 0 && nh <= 32;
}
#define T8STRIDE 514   /* doubles per wave: 256 byte entries {sum, product} + the dead entry {0, 1} */
/* Gibbs checkpoint slots per word: one per thread that owns a taxon */
__host__ __device__ static constexpr inline int sr_ckstride(int M, int TB) { return M >= TB ? TB : ((M + 63) & ~63); }
/* gm: the global-memory variant (columns too large for LDS, e.g. 1024 x 2048): the per-taxon
 * arrays (P, pre, ck, a/b, counts, logl terms, exact-delta terms) live in HBM (chain-private,
 * owner-thread access, L2/MALL-resident) and get no LDS slot */
/* taxa per exact-delta chunk (one wave's taxa): 64, or 32 in the pair kernels (two lanes per taxon) */
__host__ __device__ static constexpr inline int sr_chunk(bool pr) { return pr ? 32 : 64; }
/* gm (SR_GM_SHARED): shared hard-site and 4-step tables; lck (split-chain kernels, SR_SP_LCK): Gibbs checkpoints in LDS */
__host__ __device__ static constexpr inline int sr_lck_slots(int N) { return (N >> 5) / SR_CKG + 1; }
__host__ __device__ static constexpr inline Lay sr_layout(int N, int M, int NW, int TB, bool gm, bool pr = false, int nh = 0,
                                                          bool lck = false)
{
  Lay L{};
  size_t o = 0;
  const int CH = sr_chunk(pr), KT = (M + CH - 1) / CH, NWV = TB / 64;
  const size_t g = gm ? 0 : 1;
  lck = lck && gm;
  const bool sht = gm && SR_GM_SHARED;
  /* step tables: one copy per wave, or one shared copy behind a barrier (pair kernels: 16 waves) */
  const size_t NT = (pr || sht) ? 1 : NWV;
  L.tab = o;   o = sr_al16(o + 512 * sizeof(double));   /* glibc exp/log tables */
  L.cbuf = o;  o = sr_al16(o + g * 2 * KT * CH * sizeof(double));       /* [2][KT*CH] by proposal parity */
  L.lbuf = o;  o = sr_al16(o + g * M * sizeof(double));
  L.mt = o;    o = sr_al16(o + (size_t)SR_RING * SR_MT_N * 4);
  L.P = o;     o = sr_al16(o + g * NW * M * 4);
  L.rpi0 = o;  o = sr_al16(o + (size_t)N * 4);
  L.rpi1 = o;  o = sr_al16(o + (size_t)N * 4);
  L.ht = o;    o = sr_al16(o + (sht ? 1 : (size_t)NWV) * (2 * N + 2) * 2);   /* per wave (gm: shared): hcnt[N+1], nhall[N] (int16) */
  const size_t rw = (pr || sr_regwalk(N, M, TB, gm, nh)) ? 1 : 0;   /* register walks (pair kernels too): byte tables instead of LDS checkpoints */
  L.ck = o;    o = sr_al16(o + g * (1 - rw) * ((N >> 5) + 1) * sr_ckstride(M, TB) * sizeof(double) +
                           ((lck && !SR_SP_LPRE) ? (size_t)sr_lck_slots(N) * TB * sizeof(double) : 0));
  L.ccnt = o;  o = sr_al16(o + (size_t)2 * KT * 4);
  L.sab = o;   o = sr_al16(o + g * 2 * M * 4);
  L.scnt = o;  o = sr_al16(o + g * 4 * M * 4);
  L.hpw = o;   o = sr_al16(o + (size_t)NWV * SR_NHCAP(nh) * 4);       /* per wave: hard positions */
  L.hbw = o;   o = sr_al16(o + (size_t)NWV * NW * 4);                 /* per wave: hard bitmap */
  L.t4 = o;    o = sr_al16(o + NT * 160 * 8);                         /* per wave: 4-entry step tables (T4STRIDE) */
  L.t8 = o;    o = sr_al16(o + (rw ? NT : (gm ? 1 : 0)) * T8STRIDE * 8);   /* per wave (gm: one shared copy): 8-entry step tables */
  /* column prefix ones per word boundary (SR_SP_LPRE split kernels: the own half's, (((M + 1) / 2 + 63) & ~63) taxa =
     sr_sp_half) */
  L.pre = o;   o = sr_al16(o + (g * M + ((lck && SR_SP_LPRE) ? (size_t)((((M + 1) / 2) + 63) & ~63) : 0)) * (NW + 1) * 2);
  L.part = o;  o = sr_al16(o + (size_t)2 * 16 * NWV * 8 * 4);         /* [2][proposal][wave] count sums */
  L.tot = o;   o = sr_al16(o + (size_t)2 * NWV * 4 * 4);               /* [2][wave] t0, f0, t1, f1 */
  L.xs = o;    o = sr_al16(o + (size_t)NWV * sizeof(double));          /* per-wave broadcast slot */
  L.ptab = o;  o = sr_al16(o + 5 * 128 * 4);                          /* lane-parallel proposal tables (shared) */
  L.misc = o;  o = sr_al16(o + 64 * 8);
  L.total = o;
  return L;
}
/* Split chains (SP kernels: HBM columns, two co-resident workgroups per chain, each owning half of
 * the taxa, one taxon per thread).  Half h owns taxa [h Mh, min(M, (h + 1) Mh)), Mh a multiple of 64
 * (whole exact-delta chunks); blocks 16 g + 8 h + x hold chain 8 g + x, so a chain's halves are
 * dispatched to the same XCD (round-robin placement) and exchange through the same L2.  Exchange
 * slots per chain (ints): [2 parity][2 half][4] totals, [2 parity][2 half][16][4] proposal sums,
 * [2 parity][KT] exact-delta chunk counts. */
__host__ __device__ static inline int sr_sp_half(int M) { return (((M + 1) / 2) + 63) & ~63; }
__host__ __device__ static inline size_t sr_sp_xb(int M) { return 16 + 256 + 2 * (size_t)((M + 63) / 64); }
/* per-chain HBM scratch of the gm variant (elements): pre u16, ck f64, lbuf f64, cbuf f64 */
__host__ __device__ static inline size_t sr_gm_pre(int M, int NW) { return (size_t)(NW + 1) * M; }
__host__ __device__ static inline size_t sr_gm_ck(int N, int M, int TB) { return (size_t)((N >> 5) + 1) * sr_ckstride(M, TB); }
__host__ __device__ static inline size_t sr_gm_cbuf(int M) { return (size_t)2 * ((M + 63) / 64) * 64; }
__host__ __device__ static inline size_t sr_sp_ck(int N, int TB) { return (size_t)((N >> 5) + 1) * 2 * TB; }   /* split chains */
/* misc slots (8-byte words) */
#define MS_TOT 0      /* 4 ints in 2 words */
#define MS_DELTA 2
#define MS_C 3
#define MS_D 4
#define MS_CC 5
#define MS_DD 6
#define MS_BLK 7
#define MS_OFF 8
#define MS_GEN 9
#define MS_LOGL 10
#define MS_CAB 11
#define MS_LLS 12
#define MS_NEXACT 13
#define MS_FBK 14   /* +1 prev fail, +2 here fail, +3 S==0 (slots 15,16,17) */
#define MS_RCUR 18
#define MS_ACC 24   /* 7 acceptance counters (thread 0) */
#define MS_CDSEQ 44 /* c/d draws by the sequential GSL path */

/* ---------------------------------------------------------------- sync */
template <bool WAVE>
__device__ __forceinline__ void gsync()
{
  if (WAVE) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  } else {
    __syncthreads();
  }
}

/* ---------------------------------------------------------------- stamps */
#ifdef SR_STAMPS
#define STAMP_DECL unsigned long long st_acc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; \
  unsigned long long st_t = __builtin_amdgcn_s_memtime();
#define STAMP_RAW(ph) do { unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[ph] += t_ - st_t; st_t = t_; } while (0)
#ifdef SR_STAMP_FINE   /* exact attribution: drain outstanding memory ops before each stamp (slows the kernel) */
#define STAMP(ph) do { } while (0)
#define FST(ph) do { __builtin_amdgcn_s_waitcnt(0); STAMP_RAW(ph); } while (0)
#else
#define STAMP(ph) STAMP_RAW(ph)
#define FST(ph) do { } while (0)
#endif
/* slots 0-7 in row 1 + wave, slots 8-15 (SR_STAMP_FINE, TB <= 512) in row 9 + wave */
#define STAMP_STORE(dst) do { if ((threadIdx.x & 63) == 0 && (dst)) for (int q_ = 0; q_ < 16; ++q_) \
  if (q_ < 8 || (threadIdx.x >> 6) < 8) \
    (dst)[(blockIdx.x * 17 + 1 + (threadIdx.x >> 6) + (q_ >= 8 ? 8 : 0)) * 8 + (q_ & 7)] += st_acc[q_]; } while (0)
#else
#define STAMP_DECL
#define STAMP(ph) do { } while (0)
#define FST(ph) do { } while (0)
#define STAMP_STORE(dst) do { } while (0)
#endif
/* SR_STAMP_BAR (with SR_STAMPS, diagnostic): the cycles each wave spends inside the sweep loop's workgroup barriers,
   accumulated in stamp slot 15 (tools/stamp_profile.py: "barrier wait") -- the part of SQ_WAIT_ANY that is barrier
   wait rather than s_waitcnt on LDS / memory */
#if defined(SR_STAMPS) && defined(SR_STAMP_BAR)
#define SR_SYNC() do { const unsigned long long tb_ = __builtin_amdgcn_s_memtime(); __syncthreads(); \
  st_acc[15] += __builtin_amdgcn_s_memtime() - tb_; } while (0)
#else
#define SR_SYNC() __syncthreads()
#endif
#ifdef SR_STAMP_GIBBS   /* phase B split: slots 1 prefix+pass0, 2 pass1, 3 pass2, 4 tail */
#define GSTAMP(ph) do { unsigned long long t_ = __builtin_amdgcn_s_memtime(); gst[ph] += t_ - *gst_t; *gst_t = t_; } while (0)
#define GSTAMP_ARGS , unsigned long long *gst, unsigned long long *gst_t
#define GSTAMP_PASS , st_acc, &st_t
#define GSTAMP_K4() STAMP(4)
#else
#define GSTAMP_K4() do { } while (0)
#define GSTAMP(ph) do { } while (0)
#define GSTAMP_ARGS
#define GSTAMP_PASS
#endif
#if defined(SR_STAMP_GIBBS)
#define STAMP_D(ph) do { } while (0)
#define STAMP_K(kind) STAMP(6)
#define STAMP_E(ph) do { } while (0)
#elif defined(SR_STAMP_DRAWS)   /* alternative split of phase C: batch setup / draw loop / taxon cache / terms / rest */
#define STAMP_D(ph) STAMP(ph)
#define STAMP_K(kind) STAMP(6)
#define STAMP_E(ph) do { } while (0)
#elif defined(SR_STAMP_DECIDE)   /* draws+cache / terms / barrier wait / decide+scan / apply+rest */
#define STAMP_D(ph) do { } while (0)
#define STAMP_K(kind) STAMP(4)
#define STAMP_E(ph) STAMP(ph)
#else
#define STAMP_E(ph) do { } while (0)
#define STAMP_D(ph) do { } while (0)
#define STAMP_K(kind) do { if ((kind) == PK_PI1) STAMP(4); else if ((kind) == PK_PI3) STAMP(6); else STAMP(5); } while (0)
#endif

/* ---------------------------------------------------------------- RNG */
struct DRng {
  uint32_t *ring;   /* LDS, SR_RING blocks of 624 raw words */
  uint32_t blk, off, gen;   /* next word = block blk, index off; blocks [.., gen) exist */
  uint32_t pk0, pk1;        /* Philox key (SR_F_RNG_PHILOX), */
  bool ph;                  /* else the MT19937 recurrence */
};

/* generate block `gen` from block gen-1 (three dependency phases of the MT recurrence), or in
 * the Philox mode from its counters alone (156 Philox4x32-10 calls, stored untempered so that
 * every read site's tempering returns the Philox word); by-value arguments so the caller's
 * cursor never escapes to scratch */
template <bool WAVE>
__device__ __noinline__ void rng_gen_block(uint32_t *ring, uint32_t gen, int t, int nthr, uint32_t pk0, uint32_t pk1, bool ph)
{
  const uint32_t *prev = ring + ((gen - 1) & (SR_RING - 1)) * SR_MT_N;
  uint32_t *nxt = ring + (gen & (SR_RING - 1)) * SR_MT_N;
  if (ph) {
    for (int i = t; i < SR_MT_N / 4; i += nthr) {
      const uint64_t cw = (uint64_t)gen * (SR_MT_N / 4) + (uint64_t)i;   /* word 4 cw + j of the stream */
      const uint32_t ctr[4] = {(uint32_t)cw, (uint32_t)(cw >> 32), 0u, 0u}, key[2] = {pk0, pk1};
      uint32_t o[4];
      sr_philox4x32_10(ctr, key, o);
#pragma unroll
      for (int j = 0; j < 4; ++j) nxt[4 * i + j] = sr_mt_untemper(o[j]);
    }
    gsync<WAVE>();
    return;
  }
  for (int k = t; k < 227; k += nthr) nxt[k] = sr_mt_mix(prev[k], prev[k + 1], prev[k + 397]);
  gsync<WAVE>();
  for (int k = 227 + t; k < 454; k += nthr) nxt[k] = sr_mt_mix(prev[k], prev[k + 1], nxt[k - 227]);
  gsync<WAVE>();
  for (int k = 454 + t; k < 624; k += nthr)
    nxt[k] = (k < 623) ? sr_mt_mix(prev[k], prev[k + 1], nxt[k - 227]) : sr_mt_mix(prev[623], nxt[0], nxt[396]);
  gsync<WAVE>();
}

template <bool WAVE>
__device__ __forceinline__ void rng_gen(DRng &r, int t, int nthr)
{
  rng_gen_block<WAVE>(r.ring, r.gen, t, nthr, r.pk0, r.pk1, r.ph);
  r.gen++;
}

/* uniform: every participating thread calls it in lockstep */
template <bool WAVE>
__device__ __forceinline__ uint32_t rng_get(DRng &r, int t, int nthr)
{
  if (r.blk >= r.gen) rng_gen<WAVE>(r, t, nthr);
  uint32_t w = r.ring[(r.blk & (SR_RING - 1)) * SR_MT_N + r.off];
  if (++r.off == SR_MT_N) { r.off = 0; r.blk++; }
  return sr_mt_temper(w);
}

/* make words [pos, pos+n) resident (cooperative) */
__device__ __forceinline__ void rng_ensure(DRng &r, int n, int t, int nthr)
{
  uint32_t last = r.blk + (r.off + (uint32_t)n - 1) / SR_MT_N;
  while (r.gen <= last) rng_gen<false>(r, t, nthr);
}

/* word at relative offset j from the cursor (must be resident) */
__device__ __forceinline__ uint32_t rng_peek(const DRng &r, uint32_t j)
{
  uint32_t p = r.off + j;
  uint32_t b = r.blk + p / SR_MT_N;
  return sr_mt_temper(r.ring[(b & (SR_RING - 1)) * SR_MT_N + (p % SR_MT_N)]);
}

__device__ __forceinline__ void rng_skip(DRng &r, uint32_t n)
{
  uint32_t p = r.off + n;
  r.blk += p / SR_MT_N;
  r.off = p % SR_MT_N;
}

template <bool WAVE>
__device__ __forceinline__ double rng_uniform(DRng &r, int t, int nthr) { return rng_get<WAVE>(r, t, nthr) / 4294967296.0; }

template <bool WAVE>
__device__ __forceinline__ double rng_uniform_pos(DRng &r, int t, int nthr)
{
  double x;
  do { x = rng_uniform<WAVE>(r, t, nthr); } while (x == 0);
  return x;
}

template <bool WAVE>
__device__ __forceinline__ uint32_t rng_uniform_int(DRng &r, uint32_t n, int t, int nthr)
{
  uint32_t scale = 0xffffffffu / n, k;
  do { k = rng_get<WAVE>(r, t, nthr) / scale; } while (k >= n);
  return k;
}

/* gsl_rng_uniform_int(n) with its divisor scale = 0xffffffff/n precomputed; the quotient
 * get()/scale is taken from a double reciprocal and corrected to the exact integer. */
struct UDiv { uint32_t n, scale; double rs; };
__device__ __forceinline__ UDiv make_udiv(uint32_t n)
{
  UDiv u;
  u.n = n;
  u.scale = 0xffffffffu / n;
  u.rs = 1.0 / (double)u.scale;
  return u;
}
template <bool WAVE>
__device__ __forceinline__ uint32_t rng_uint_fast(DRng &r, const UDiv &u, int t, int nthr)
{
  uint32_t k;
  do {
    const uint32_t g = rng_get<WAVE>(r, t, nthr);
    uint32_t q = (uint32_t)((double)g * u.rs);
    const uint64_t qs = (uint64_t)q * u.scale;
    if (qs > g) q--;
    else if (g - (uint32_t)qs >= u.scale) q++;
    k = q;
  } while (k >= u.n);
  return k;
}

/* quotient get()/scale of gsl_rng_uniform_int for a tempered word g (k >= n means GSL rejects g) */
__device__ __forceinline__ uint32_t udiv_word(uint32_t g, const UDiv &u)
{
  uint32_t q = (uint32_t)((double)g * u.rs);
  const uint64_t qs = (uint64_t)q * u.scale;
  if (qs > g) q--;
  else if (g - (uint32_t)qs >= u.scale) q++;
  return q;
}

/* gsl_rng_uniform_int's quotient g / scale by an invariant-divisor multiply (Hacker's Delight
 * round-up method, exact for every 32-bit g; scale >= 2 here since n <= 4095): scalar ALU only */
struct UDivM { uint32_t n, m; int l; };
__device__ __forceinline__ UDivM make_udivm(uint32_t n)
{
  UDivM u;
  const uint32_t d = 0xffffffffu / n;
  u.n = n;
  u.l = 32 - __builtin_clz(d - 1);
  u.m = (uint32_t)(((((uint64_t)1) << 32) * ((((uint64_t)1) << u.l) - d)) / d + 1);
  return u;
}
__device__ __forceinline__ uint32_t udivm(uint32_t g, const UDivM &u)
{
  const uint32_t t = __umulhi(u.m, g);
  return (t + ((g - t) >> 1)) >> (u.l - 1);
}

__device__ __forceinline__ uint32_t udivm_v(uint32_t g, uint32_t m, int l)
{
  const uint32_t t = __umulhi(m, g);
  return (t + ((g - t) >> 1)) >> (l - 1);
}

/* the next 8 tempered words from the cursor, loaded together, if they are resident (the ring
 * is a circular buffer of SR_RING * 624 words: block b lives at (b mod SR_RING) * 624) */
__device__ __forceinline__ bool rng_window8(const DRng &r, uint32_t (&w)[8])
{
  if (r.blk + (r.off + 7) / SR_MT_N >= r.gen) return false;
  const uint32_t base = (r.blk & (SR_RING - 1)) * SR_MT_N + r.off;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint32_t idx = base + k;
    idx = (idx >= SR_RING * SR_MT_N) ? idx - SR_RING * SR_MT_N : idx;
    w[k] = sr_mt_temper(r.ring[idx]);
  }
  return true;
}

/* ------------------------------------------------ GSL beta/gamma/ziggurat */
template <bool WAVE>
__device__ __forceinline__ double d_gauss_zig(DRng &r, int lane, int nthr, const sr_mtab &tb)
{
  for (;;) {
    /* the word is block-uniform: keep it (and the table index) in SGPRs so the ziggurat table
       lookups are scalar constant-cache loads */
    uint32_t k = (uint32_t)__builtin_amdgcn_readfirstlane((int)rng_get<WAVE>(r, lane, nthr));
    uint32_t i = k & 0xFF;
    uint32_t j = (k >> 8) & 0xFFFFFF;
    int sign = (i & 0x80) ? +1 : -1;
    i &= 0x7f;
    double x = j * c_zig_w[i];
    if (j < c_zig_k[i]) return sign * 1.0 * x;
    double y;
    if (i < 127) {
      double y0 = c_zig_y[i], y1 = c_zig_y[i + 1];
      double U1 = rng_uniform<WAVE>(r, lane, nthr);
      y = y1 + (y0 - y1) * U1;
    } else {
      double U1 = 1.0 - rng_uniform<WAVE>(r, lane, nthr);
      double U2 = rng_uniform<WAVE>(r, lane, nthr);
      x = SR_ZIGR - sr_log_m(U1, &tb) / SR_ZIGR;
      y = sr_exp_m(-SR_ZIGR * (x - 0.5 * SR_ZIGR), &tb) * U2;
    }
    if (y < sr_exp_m(-0.5 * x * x, &tb)) return sign * 1.0 * x;
  }
}

template <bool WAVE>
__device__ __forceinline__ double d_gamma(DRng &r, double a, int lane, int nthr, const sr_mtab &tb)
{
  double boost = 1.0;
  if (a < 1) { /* unreachable from the sampler (a = 1 + count); kept for GSL parity */
    double u = rng_uniform_pos<WAVE>(r, lane, nthr);
    boost = sr_exp_m(sr_log_m(u, &tb) * (1.0 / a), &tb);
    a = 1.0 + a;
  }
  double x, v, u;
  double d = a - 1.0 / 3.0;
  double c = (1.0 / 3.0) / __builtin_sqrt(d);
  for (;;) {
    do {
      x = d_gauss_zig<WAVE>(r, lane, nthr, tb);
      v = 1.0 + c * x;
    } while (v <= 0);
    v = v * v * v;
    u = rng_uniform_pos<WAVE>(r, lane, nthr);
    if (u < 1 - 0.0331 * x * x * x * x) break;
    if (sr_log_m(u, &tb) < 0.5 * x * x + d * (1 - v + sr_log_m(v, &tb))) break;
  }
  double g = 1.0 * d * v;
  return (boost == 1.0) ? g : g * boost;
}

/* mcmc_samplebeta: y = beta(1+a, 1+b); keep the old value unless log y in [low, high] */
template <bool WAVE>
__device__ __forceinline__ double d_samplebeta(DRng &r, double x, double a, double b, double low, double high, int lane,
                                               int nthr, const sr_mtab &tb)
{
  double y;
  if (a == 0. && b == 0.) {
    /* gsl_ran_beta's Johnk branch (both shapes <= 1; here both are exactly 1 + 0): pow(U, 1/1) = U,
       so X = U, Y = V, and X + Y > 0 always (oracle/om_gsl.h om_beta) */
    for (;;) {
      const double U = rng_uniform_pos<WAVE>(r, lane, nthr), V = rng_uniform_pos<WAVE>(r, lane, nthr);
      if (U + V <= 1.0) { y = U / (U + V); break; }
    }
  } else {
    double g[2];
    for (int k = 0; k < 2; ++k) g[k] = d_gamma<WAVE>(r, 1. + (k ? b : a), lane, nthr, tb);   /* one inlined copy */
    const double x1 = g[0], x2 = g[1];
    y = x1 / (x1 + x2);
  }
  if (y > 0.) {
    y = sr_log_m(y, &tb);
    if (low <= y && y <= high) x = y;
  }
  return x;
}

__device__ __forceinline__ double readlane_f64(double v, int l)
{
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

/* mcmc_samplec + mcmc_sampled (mcmc.c:751-825) with the four gammas evaluated lane-parallel.
 * Speculation: each gamma takes exactly two words (one ziggurat word inside the box, one
 * uniform_pos word accepted by the squeeze or the log test), so gamma g reads words 2g, 2g+1 from
 * the cursor.  Lanes 0..3 evaluate gamma(1+f1), gamma(1+t0), gamma(1+f0), gamma(1+t1) with the
 * expressions of d_gauss_zig / d_gamma verbatim; lanes 0, 1 then form the two betas.  Valid iff all
 * four gammas took their two-word path and the 8 words are resident -- otherwise returns false
 * and the caller runs the sequential draws from the same cursor.  Wave-level: every wave of the
 * block computes it identically (no block synchronisation). */
/* The part of draw_cd_fast that does not depend on the counts: lane g (& 3)'s two words from the cursor and its
 * ziggurat step (x, and whether the word falls inside the box), read before the phase-A barrier so that the table
 * lookups (global constant memory) overlap the wait.  ok = false: the words are not resident (no prefetch). */
struct CDPre { uint32_t w1; double x; bool box, ok; };
__device__ __forceinline__ CDPre cd_prefetch(const DRng &r, int lane)
{
  CDPre p{};
  p.ok = r.blk + (r.off + 7) / SR_MT_N < r.gen;
  if (!p.ok) return p;
  const uint32_t base = (r.blk & (SR_RING - 1)) * SR_MT_N + r.off;
  const int g = lane & 3;
  uint32_t i0 = base + 2 * g, i1 = base + 2 * g + 1;
  i0 = (i0 >= SR_RING * SR_MT_N) ? i0 - SR_RING * SR_MT_N : i0;
  i1 = (i1 >= SR_RING * SR_MT_N) ? i1 - SR_RING * SR_MT_N : i1;
  const uint32_t k = sr_mt_temper(r.ring[i0]);
  p.w1 = sr_mt_temper(r.ring[i1]);
  uint32_t i = k & 0xFF;
  const uint32_t j = (k >> 8) & 0xFFFFFF;
  const int sign = (i & 0x80) ? +1 : -1;
  i &= 0x7f;
  const double x = j * c_zig_w[i];
  p.box = j < c_zig_k[i];
  p.x = sign * 1.0 * x;
  return p;
}

__device__ __forceinline__ bool draw_cd_fast(DRng &r, double &c, double &d, int f1, int t0, int f0, int t1,
                                             const sr_mtab &tb, int lane, CDPre pf = CDPre{})
{
#ifdef SR_FORCE_EXACT   /* test build: the sequential GSL draws */
  return false;
#endif
  if (r.blk + (r.off + 7) / SR_MT_N >= r.gen) return false;
  if ((f1 == 0 && t0 == 0) || (f0 == 0 && t1 == 0)) return false;   /* a Johnk beta: the sequential path */
  if (!pf.ok) pf = cd_prefetch(r, lane);
  const int g = lane & 3;
  const uint32_t w1 = pf.w1;
  const int cnt = (g == 0) ? f1 : (g == 1) ? t0 : (g == 2) ? f0 : t1;
  const double a = 1. + (double)cnt;                   /* d_samplebeta: gamma(1. + a) */
  const double dd = a - 1.0 / 3.0;
  const double cc = (1.0 / 3.0) / __builtin_sqrt(dd);
  const double x = pf.x;
  bool ok = pf.box;
  double v = 1.0 + cc * x;
  ok = ok && v > 0 && w1 != 0u;
  v = v * v * v;
  const double u = w1 / 4294967296.0;
  bool acc = u < 1 - 0.0331 * x * x * x * x;
  if (ok && !acc) acc = sr_log_m(u, &tb) < 0.5 * x * x + dd * (1 - v + sr_log_m(v, &tb));
  ok = ok && acc;
  const double gv = 1.0 * dd * v;
  if ((__ballot(ok) & 0xFull) != 0xFull) return false;
  /* betas: lane 0 -> c (gammas 0, 1), lane 1 -> d (gammas 2, 3) */
  const double x1 = readlane_f64(gv, 0), x2 = readlane_f64(gv, 1), x3 = readlane_f64(gv, 2), x4 = readlane_f64(gv, 3);
  const bool isd = (lane & 1) != 0;
  const double ga = isd ? x3 : x1, gb = isd ? x4 : x2;
  double res = isd ? d : c;
  double y = ga / (ga + gb);
  if (y > 0.) {
    y = sr_log_m(y, &tb);
    if ((isd ? SR_MIND : SR_MINC) <= y && y <= (isd ? SR_MAXD : SR_MAXC)) res = y;
  }
  c = readlane_f64(res, 0);
  d = readlane_f64(res, 1);
  rng_skip(r, 8);
  return true;
}

/* ---------------------------------------------------------------- helpers */
struct CD { double c, d, cc, dd, ec; };

__device__ __forceinline__ double qval(int dt0, int df0, int dt1, int df1, const CD &k)
{
  double t = (double)dt0 * k.cc;
  t = t + (double)df0 * k.d;
  t = t + (double)dt1 * k.dd;
  t = t + (double)df1 * k.c;
  return t;
}

__device__ __forceinline__ int colbit(const uint32_t *Pm, int M, int p)
{
  return (Pm[(p >> 5) * M] >> (p & 31)) & 1;
}

/* ones of column m at positions [lo, hi) */
__device__ __forceinline__ int ones_range(const uint32_t *Pm, int M, int lo, int hi)
{
  if (hi <= lo) return 0;
  int wl = lo >> 5, wh = (hi - 1) >> 5, s = 0;
  for (int w = wl; w <= wh; ++w) {
    uint32_t mask = 0xffffffffu;
    if (w == wl) mask &= 0xffffffffu << (lo & 31);
    if (w == wh) {
      int e = ((hi - 1) & 31) + 1;
      if (e < 32) mask &= (1u << e) - 1u;
    }
    s += __popc(Pm[w * M] & mask);
  }
  return s;
}

struct BitWalk {
  const uint32_t *Pm;
  int M, N, cur;
  bool rev;
  uint32_t word;
  __device__ BitWalk(const uint32_t *p, int m, int n, bool r) : Pm(p), M(m), N(n), cur(-1), rev(r), word(0) {}
  __device__ __forceinline__ int bit(int w)
  {
    int p = rev ? (N - 1 - w) : w;
    int wi = p >> 5;
    if (wi != cur) { cur = wi; word = Pm[wi * M]; }
    return (word >> (p & 31)) & 1;
  }
};

/* mcmc_auxa + mcmc_logtop + mcmc_randompick for one limit of one taxon, in walk
 * coordinates (fwd: walk w = position w; rev: walk w = position N-1-w).  o = current limit,
 * entries w = 0..L.  Returns the picked entry (the caller derives the count deltas there).
 * Arguments by value and the result in a register: nothing of the caller lives in scratch. */
__device__ __noinline__ int draw_exact(const uint32_t *Pm, int M, int N, bool rev, int o, int L, double u,
                                      const CD k, const sr_mtab tb)
{
  const int POo = rev ? ones_range(Pm, M, N - o, N) : ones_range(Pm, M, 0, o);
  auto q_at = [&](int w, int PO) -> double {
    if (w == o) return 0.0;
    if (w < o) { int O = POo - PO; int Z = (o - w) - O; return qval(-Z, Z, O, -O, k); }
    int O = PO - POo; int Z = (w - o) - O; return qval(Z, -Z, -O, O, k);
  };
  auto wprefix = [&](int w) -> int { return rev ? ones_range(Pm, M, N - w, N) : ones_range(Pm, M, 0, w); };

  /* pass 1: max and the window of entries that can exceed LOGEPSILON (z >= q_o = 0) */
  double z = -__builtin_inf();
  int lo = -1, hi = -1, PO = 0;
  {
    BitWalk bw(Pm, M, N, rev);
    for (int w = 0; w <= L; ++w) {
      double q = q_at(w, PO);
      if (q > z) z = q;
      if (q > SR_LOGEPSILON) { if (lo < 0) lo = w; hi = w; }
      if (w < L) PO += bw.bit(w);
    }
  }
  /* pass 2: x = sequential sum of exp(max(LOGEPS, q - z)) (mcmc.c:731-737) */
  double x = sr_run_add(0.0, k.ec, lo);
  {
    BitWalk bw(Pm, M, N, rev);
    PO = wprefix(lo);
    for (int w = lo; w <= hi; ++w) {
      double t = q_at(w, PO) - z;
      double y = (t > SR_LOGEPSILON) ? sr_exp_m(t, &tb) : k.ec;
      x = x + y;
      if (w < L) PO += bw.bit(w);
    }
  }
  x = sr_run_add(x, k.ec, L - hi);
  /* pass 3: randompick (mcmc.c:901-915) with p_i = y_i / x (mcmc.c:738-739) */
  const double pe = k.ec / x;
  double r = u;
  int res = -1;
  if (lo > 0) {
    long s = sr_run_sub(&r, pe, lo);
    if (r <= 0.0) res = (int)s - 1;
  }
  if (res < 0) {
    BitWalk bw(Pm, M, N, rev);
    PO = wprefix(lo);
    for (int w = lo; w <= hi; ++w) {
      double t = q_at(w, PO) - z;
      double y = (t > SR_LOGEPSILON) ? sr_exp_m(t, &tb) : k.ec;
      r = r - y / x;
      if (r <= 0.0 || w == L) { res = w; break; }
      if (w < L) PO += bw.bit(w);
    }
  }
  if (res < 0) {
    long s = sr_run_sub(&r, pe, L - hi);
    res = (r <= 0.0) ? hi + (int)s : L;
  }
  return res;
}


/* ones of column m at positions [0, x) from the per-word prefix table (pre: column m's entries,
 * stride M; row k = ones in [0, 32k)) and one partial word */
__device__ __forceinline__ int col_pre(const uint16_t *prem, const uint32_t *Pm, int M, int x, int PS = 0)
{
  const int w = x >> 5, bits = x & 31;
  const uint32_t word = bits ? Pm[w * M] : 0u;
  return (int)prem[w * (PS ? PS : M)] + __popc(word & ((1u << bits) - 1u));   /* PS: the table's own stride */
}

/* the same without a branch: the word read always (row 0 when x is a multiple of 32, masked to nothing),
   so a proposal's taxon terms carry no exec-mask branches and the slots' reads can be in flight together */
__device__ __forceinline__ int col_pre_bf(const uint16_t *prem, const uint32_t *Pm, int M, int x, int PS = 0)
{
  const int w = x >> 5, bits = x & 31;
  const uint32_t word = Pm[(bits ? w : 0) * M];
  return (int)prem[w * (PS ? PS : M)] + __popc(word & ((1u << bits) - 1u));
}

/* 32 walk bits [32k, 32k+32): fwd = positions, rev = positions N-1-w (bit i = walk 32k+i) */
__device__ __forceinline__ uint32_t walk_word(const uint32_t *Pm, int M, int N, int NW, bool rev, int k)
{
  if (!rev) return (k < NW) ? Pm[k * M] : 0u;
  const int s = N - 32 - 32 * k;
  uint32_t v;
  if (s >= 0) {
    const int wi = s >> 5, sh = s & 31;
    const uint32_t lo = Pm[wi * M];
    const uint32_t hi = (sh && wi + 1 < NW) ? Pm[(wi + 1) * M] : 0u;
    v = sh ? ((lo >> sh) | (hi << (32 - sh))) : lo;
  } else {
    v = (s > -32) ? (Pm[0] << (-s)) : 0u;
  }
  return __brev(v);
}

/* ones among walk positions [0, w) */
__device__ __forceinline__ int walk_prefix(const uint32_t *Pm, int M, int N, int NW, bool rev, int w)
{
  int s = 0;
  const int full = w >> 5;
    for (int k = 0; k < full; ++k) s += __popc(walk_word(Pm, M, N, NW, rev, k));
  if (w & 31) s += __popc(walk_word(Pm, M, N, NW, rev, full) & ((1u << (w & 31)) - 1u));
  return s;
}

/* The 4-entry step tables of a wave, interleaved: entry (c, nib) = {sum of the first c prefix
 * products of the nibble's ratios, product of all four} -- one 16-byte LDS read per group
 * (c = valid entries of the group, 0..4; the product is the same in every row). */
#define T4STRIDE 160   /* doubles per wave */
__device__ __forceinline__ double2 t4sp(const double *T4, int c, uint32_t nib)
{
  return *reinterpret_cast<const double2 *>(T4 + 2 * (c * 16 + (int)nib));
}
__device__ __forceinline__ double t4s(const double *T4, int c, uint32_t nib) { return T4[2 * (c * 16 + (int)nib)]; }
__device__ __forceinline__ double t4p(const double *T4, uint32_t nib) { return T4[2 * (64 + (int)nib) + 1]; }

/* The Gibbs step tables' entries (rA = 2^-vA, rB = 2^-vB: the ratio of consecutive walk weights after a zero / a
 * one).  t4_row: nibble l's row, sc[c] = sum of the first c prefix products (c = 0..4), returns the product of all
 * four; t8_entry: byte e, {sum of its 8 prefix products, their product}.  Built per sweep by the sweep kernel and by
 * the certification self-test (sr_device_selftest_gibbs) alike. */
__device__ __forceinline__ double t4_row(int l, double rA, double rB, double (&sc)[5])
{
  double pr = 1.0, sm = 1.0;
  sc[0] = 0.0;
  sc[1] = sm;
  pr = pr * ((l & 1) ? rB : rA); sm = sm + pr; sc[2] = sm;
  pr = pr * ((l & 2) ? rB : rA); sm = sm + pr; sc[3] = sm;
  pr = pr * ((l & 4) ? rB : rA); sm = sm + pr; sc[4] = sm;
  pr = pr * ((l & 8) ? rB : rA);
  return pr;
}
__device__ __forceinline__ double2 t8_entry(int e, double rA, double rB)
{
  double pr = 1.0, sm = 0.0;
#pragma unroll
  for (int k = 0; k < 8; ++k) { sm = sm + pr; pr = pr * (((e >> k) & 1) ? rB : rA); }
  return make_double2(sm, pr);
}

/* 2^q (q <= ~0) to ~1.6e-7 relative: exact f64 split q = n + f, f in [0,1), v_exp_f32(f) */
__device__ __forceinline__ double exp2_split(double q)
{
  const double n = __builtin_floor(q);
  if (n < -1070.0) return 0.0;
  const float y = __builtin_amdgcn_exp2f((float)(q - n));
  return __builtin_amdgcn_ldexp((double)y, (int)n);
}

#define SR_WIN_T 40.0       /* words whose q stays 40 bits below q(o) are skipped (mass <= 2^-40 each entry) */

/* mcmc_auxa + mcmc_logtop + mcmc_randompick for one limit of one taxon (exact version:
 * draw_exact), certified fast path.  The picked index depends only on where u falls in the
 * cumulative distribution F_k = sum_{i<=k} y_i / x, y_i = exp(max(LOGEPS, q_i - z)).
 *
 * Walk coordinates w = 0..L; q(w) relative to the current limit o (q(o) = 0) in log2 units:
 * q(w+1) = q(w) - v(bit_w), v(0) = vA = (d - cc) log2e < 0 (zeros raise q), v(1) = vB =
 * (dd - c) log2e > 0 (ones lower it).  Approximation F^:
 *   - pass 0 (per 32-entry word, exact integer counts): an upper bound of q inside the word;
 *     words whose bound is <= -40 are outside the window [klo, khi] and contribute 0;
 *   - pass 1 over the window: y_{w+1} = y_w * r(bit_w), r = 2^-v computed to f64 accuracy
 *     (rA = e^(cc-d), rB = e^(c-dd)), S accumulated in order, checkpoint ck[k] after word k.
 *     The common factor of the first y (exp2_split) cancels in F; the chain contributes
 *     <= 3(N+1) 2^-52 relative error;
 *   - the reference's clamped terms (<= (N+1) e^LOGEPS), skipped words (<= (N+1) 2^-40) and
 *     its own sequential rounding are absorbed by the absolute slack.
 * Index k is accepted only if u - F^_{k-1} and F^_k - u both exceed the error bound; then the
 * reference's exact sequential computation provably returns the same k.  Otherwise (or on
 * overflow) the exact path runs.  ck: this lane's checkpoint slots (stride ckstride). */
#ifndef SR_WCH
#define SR_WCH 8   /* walk words read together: one memory round trip per 8 words (HBM columns: L2 / MALL latency) */
#endif
#define SR_QSPAN 600.0   /* window trim below the largest word-start q (log2 units), draw_fast */
template <bool B8>
__device__ __forceinline__ int draw_fast(const uint32_t *Pm, const uint16_t *prem, int M, int N, int NW, bool rev, int o, int L,
                                         int POo, double u, const CD &K, const sr_mtab &tb, double vA, double vB, double rA, double rB,
                                         const double *T4, const double *T8,
                                         typename std::conditional<B8 && SR_CK32, float, double>::type *ck,
                                         int ckstride, int PS, uint64_t *fbk, int &dt0, int &df0,
                                         int &dt1, int &df1 GSTAMP_ARGS)
{
  /* POo: ones among walk entries [0, o), from the caller's column prefix table */
  const int nk = (L >> 5) + 1;
  /* pass 0: window of words that can hold mass above 2^-40 relative to entry o; the ones before
     its first word are kept for the pick's count (no prefix walk afterwards).  Long walks (N up to
     4095) can span q ranges far beyond the f64 exponent range: the chain is scaled by the largest
     word-start q of the window (qmx), and window words whose start q lies more than SR_QSPAN below it
     are dropped from the ends (their entries hold < 2^-(SR_QSPAN-75) of the mass each; ABS covers it). */
  int klo = nk, khi = -1, Oklo = 0;
  double qlo = 0.0, qmx = -__builtin_inf(), qmn = __builtin_inf();
  {
    int O = 0;   /* ones among walk entries [0, 32k) */
    for (int k0 = 0; k0 < nk; k0 += SR_WCH) {
      uint32_t wv[SR_WCH];
#pragma unroll
      for (int t = 0; t < SR_WCH; ++t) wv[t] = (k0 + t < nk) ? walk_word(Pm, M, N, NW, rev, k0 + t) : 0u;
#pragma unroll
      for (int t = 0; t < SR_WCH; ++t) {
        const int k = k0 + t;
        if (k < nk) {
          const uint32_t ww = wv[t];
          const int nb = min(32, L + 1 - 32 * k);
          const uint32_t vm = (nb >= 32) ? 0xffffffffu : ((1u << nb) - 1u);
          const int w0 = 32 * k;
          /* q at entry w0 from exact counts */
          const double qs = (w0 <= o) ? ((double)((o - w0) - (POo - O)) * vA + (double)(POo - O) * vB)
                                      : -((double)((w0 - o) - (O - POo)) * vA + (double)(O - POo) * vB);
          const int ones = __popc(ww & vm);
          const double ub = qs - (double)(nb - ones) * vA;   /* every zero raises q by -vA */
          if (ub > -SR_WIN_T) {
            if (k < klo) { klo = k; qlo = qs; Oklo = O; }
            khi = k;
            qmx = fmax(qmx, qs);
            qmn = fmin(qmn, qs);
          }
          O += __popc(ww);
        }
      }
    }
  }
  if (klo <= khi && qmx - qmn > SR_QSPAN) {   /* trim the window's ends to start q >= qmx - SR_QSPAN (rare:
                                                 the word-start counts are recounted from the words) */
    const int k1 = klo, k2 = khi;
    int O = Oklo;
    klo = nk; khi = -1;
    for (int k0 = k1; k0 <= k2; k0 += SR_WCH) {
      uint32_t wv[SR_WCH];
#pragma unroll
      for (int t = 0; t < SR_WCH; ++t) wv[t] = (k0 + t <= k2) ? walk_word(Pm, M, N, NW, rev, k0 + t) : 0u;
#pragma unroll
      for (int t = 0; t < SR_WCH; ++t) {
        const int k = k0 + t, w0 = 32 * k;
        const double qs = (w0 <= o) ? ((double)((o - w0) - (POo - O)) * vA + (double)(POo - O) * vB)
                                    : -((double)((w0 - o) - (O - POo)) * vA + (double)(O - POo) * vB);
        if (k <= k2 && qs >= qmx - SR_QSPAN) {
          if (k < klo) { klo = k; qlo = qs; Oklo = O; }
          khi = k;
        }
        O += __popc(wv[t]);
      }
    }
  }
  GSTAMP(1);
#ifdef SR_STAMP_GIBBS
  {   /* window statistics: words per draw, wave max, walk words */
    const int wn = khi - klo + 1;
    int wmax = wn;
    for (int off_ = 32; off_ > 0; off_ >>= 1) wmax = max(wmax, __shfl_xor(wmax, off_));
    atomicAdd((unsigned long long *)fbk + 26, (unsigned long long)wn);
    if ((threadIdx.x & 63) == 0) atomicAdd((unsigned long long *)fbk + 27, (unsigned long long)wmax);
    atomicAdd((unsigned long long *)fbk + 28, (unsigned long long)nk);
    atomicAdd((unsigned long long *)fbk + 29, 1ull);
  }
#endif
  /* pass 1: S over the window, checkpoints; the chain scaled by 2^-qmx.  A chain that falls below
     2^-700 at a word start inside the window (q dipping far below qmx and possibly rising again)
     would lose precision: that draw takes the exact path (uf). */
  const double y0 = exp2_split(qlo - (klo <= khi ? qmx : 0.0));
  double S = 0.0;
  bool uf = false;
  {
    double y = y0;
    for (int k0 = klo; k0 <= khi; k0 += SR_WCH) {
      uint32_t wv[SR_WCH];
#pragma unroll
      for (int t = 0; t < SR_WCH; ++t) wv[t] = (k0 + t <= khi) ? walk_word(Pm, M, N, NW, rev, k0 + t) : 0u;
#pragma unroll
      for (int t = 0; t < SR_WCH; ++t) {
        const int k = k0 + t;
        if (k <= khi) {
          const uint32_t ww = wv[t];
          const int nb = min(32, L + 1 - 32 * k);
          uf |= y < 0x1p-700;
          if constexpr (B8) {
            /* (HBM columns) the word's whole bytes from the shared 8-entry tables in Horner form (one
               multiply per word on the y chain, draw_fast_s); the walk's partial last byte from T4 */
            const int nfk = nb >> 3, c8 = nb & 7;
            double2 t8[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const uint32_t e = (g < nfk) ? ((ww >> (8 * g)) & 255u) : 256u;
              t8[g] = *reinterpret_cast<const double2 *>(T8 + 2 * e);
            }
            const double w23 = __builtin_fma(t8[2].y, t8[3].x, t8[2].x);
            const double w13 = __builtin_fma(t8[1].y, w23, t8[1].x);
            const double W = __builtin_fma(t8[0].y, w13, t8[0].x);
            const double pw = (t8[0].y * t8[1].y) * (t8[2].y * t8[3].y);
            S = __builtin_fma(y, W, S);
            y = y * pw;
            if (c8 > 0) {   /* only the walk's last word (y is not used after it) */
              const uint32_t eb = (ww >> (8 * nfk)) & 255u;
              const double2 tlo = t4sp(T4, min(c8, 4), eb & 15u);
              const double shi = t4s(T4, max(c8 - 4, 0), eb >> 4);
              S = __builtin_fma(y, tlo.x, S);
              S = __builtin_fma(y * tlo.y, shi, S);
            }
          } else {
            /* 4 entries per step: T4[c][nibble] = sum of the first c prefix products of the nibble's
               ratios (c = valid entries of the group, 0..4), T4[5][nibble] = product of all four */
#pragma unroll
            for (int g = 0; g < 8; ++g) {
              const uint32_t nib = (ww >> (4 * g)) & 15u;
              const int c = min(max(nb - 4 * g, 0), 4);
              const double2 t4 = t4sp(T4, c, nib);
              S = __builtin_fma(y, t4.x, S);
              y = y * t4.y;
            }
          }
          if (!B8 || SR_CKG == 1 || (k - klo) % SR_CKG == SR_CKG - 1)
            ck[(B8 && SR_CKG > 1 ? (k - klo) / SR_CKG : k) * ckstride] = S;   /* (B8: one per SR_CKG window words) */
        }
      }
    }
  }
  GSTAMP(2);
  /* pass 2: locate the word; y at its start from its own sum (no replay of the chain): the word's
     partial sums are Sp0 + y gs1[g] with gs1 its unscaled group-end sums (y = 1 at the word start)
     and y = (ck[j] - Sp0) / gs1[7], exact for j = klo (y0).  The reconstruction moves each partial
     sum by at most ~9 2^-53 S (the subtraction and the word's fma roundings in pass 1): the extra
     absolute slack 2^-46 in u covers it; the unscaled sums' own rounding (and, with the byte tables in
     pass 1, the relative difference of the two table forms, <= 2 x 16 ulp) is inside REL's + 32.
     B8 with SR_CK32 (HBM columns, not the default): the checkpoints are stored as f32: each is within
     2^-24 S of its f64 value, so the word search may land one word off (then the word's first or last
     entry fails its certification and the exact walk runs) and a reconstructed partial sum moves by at
     most 3 2^-24 S (Sp0, Sj and y = (Sj - Sp0) / sum): the absolute slack grows by 2^-21 -- and every
     entry with less mass than that slack fails certification, which measured 200x more exact walks.
     Ones before the word from the column prefix table. */
  int res = -1, POp = 0;
  if (S > 0.0 && S < 0x1p1000 && !uf) {
    const double inv = 1.0 / S;
    const double REL = (double)(N + 33) * 0x1p-50 * SR_CERT_SCALE;
    const double ABS = ((double)(N + 1) * 0x1p-39 + 0x1p-46 + ((B8 && SR_CK32) ? 0x1p-21 : 0.0)) * SR_CERT_SCALE;
    int j = klo;   /* first window word whose checkpoint reaches u (checkpoints ascend) */
    double Sp0, yj;   /* the partial sum before word j, y at its start */
    if (B8 && SR_CKG > 1) {
      /* checkpoints after every SR_CKG-th window word: the group holding u, then the word from the group's
         own unscaled sums (the byte tables as in pass 1, its words read in one round trip); y at the group
         start from its checkpoint difference.  The group's partial sums Sa + yg A_t (A_t the unscaled sum
         of its first t words) re-associate pass 1's chain: within REL's + 32 and the 2^-46 of ABS. */
      const int ngrp = (khi - klo + SR_CKG) / SR_CKG;
      int g = 0;
      for (int k0 = 0; k0 < ngrp - 1; k0 += SR_WCH) {
        double cv[SR_WCH];
#pragma unroll
        for (int t = 0; t < SR_WCH; ++t) cv[t] = (k0 + t < ngrp - 1) ? (double)ck[(k0 + t) * ckstride] : 0.0;
#pragma unroll
        for (int t = 0; t < SR_WCH; ++t) g += (k0 + t < ngrp - 1 && cv[t] * inv < u) ? 1 : 0;
      }
      const double Sa = (g == 0) ? 0.0 : (double)ck[(g - 1) * ckstride];
      const double Sb = (g == ngrp - 1) ? S : (double)ck[g * ckstride];
      const int k1 = klo + SR_CKG * g;
      uint32_t gw[SR_CKG];
#pragma unroll
      for (int t = 0; t < SR_CKG; ++t) gw[t] = (k1 + t <= khi) ? walk_word(Pm, M, N, NW, rev, k1 + t) : 0u;
      double A[SR_CKG], Yt[SR_CKG];   /* unscaled sum of the group's words before word t, product before t */
      double acc = 0.0, yy = 1.0;
#pragma unroll
      for (int t = 0; t < SR_CKG; ++t) {
        A[t] = acc;
        Yt[t] = yy;
        if (k1 + t <= khi) {
          const uint32_t ww = gw[t];
          const int nb = min(32, L + 1 - 32 * (k1 + t)), nfk = nb >> 3, c8 = nb & 7;
          double2 t8[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t e = (q < nfk) ? ((ww >> (8 * q)) & 255u) : 256u;
            t8[q] = *reinterpret_cast<const double2 *>(T8 + 2 * e);
          }
          const double w23 = __builtin_fma(t8[2].y, t8[3].x, t8[2].x);
          const double w13 = __builtin_fma(t8[1].y, w23, t8[1].x);
          double W = __builtin_fma(t8[0].y, w13, t8[0].x);
          const double P = (t8[0].y * t8[1].y) * (t8[2].y * t8[3].y);
          if (c8 > 0) {
            const uint32_t eb = (ww >> (8 * nfk)) & 255u;
            const double2 tlo = t4sp(T4, min(c8, 4), eb & 15u);
            W = __builtin_fma(P, tlo.x, W);
            W = __builtin_fma(P * tlo.y, t4s(T4, max(c8 - 4, 0), eb >> 4), W);
          }
          acc = __builtin_fma(yy, W, acc);
          yy = yy * P;
        }
      }
      const double yg = (g == 0) ? y0 : (Sb - Sa) / acc;
      int t_sel = 0;
#pragma unroll
      for (int t = 1; t < SR_CKG; ++t) t_sel += (k1 + t <= khi && __builtin_fma(yg, A[t], Sa) * inv < u) ? 1 : 0;
      double At = A[0], Yp = Yt[0];
#pragma unroll
      for (int t = 1; t < SR_CKG; ++t)
        if (t == t_sel) { At = A[t]; Yp = Yt[t]; }
      j = k1 + t_sel;
      Sp0 = __builtin_fma(yg, At, Sa);
      yj = yg * Yp;
    } else {
      for (int k0 = klo; k0 < khi; k0 += SR_WCH) {
        double cv[SR_WCH];
#pragma unroll
        for (int t = 0; t < SR_WCH; ++t) cv[t] = (k0 + t < khi) ? (double)ck[(k0 + t) * ckstride] : 0.0;
#pragma unroll
        for (int t = 0; t < SR_WCH; ++t) j += (k0 + t < khi && cv[t] * inv < u) ? 1 : 0;
      }
      Sp0 = (j == klo) ? 0.0 : (double)ck[(j - 1) * ckstride];
      yj = (j == khi) ? S : (double)ck[j * ckstride];   /* (Sj: y follows from it below) */
    }
    int Oj;   /* ones among walk entries [0, 32 j) */
    if (!rev) Oj = (int)prem[j * (PS ? PS : M)];
    else {    /* positions [N - 32 j, N) */
      const int x = N - 32 * j;
      Oj = (int)prem[NW * (PS ? PS : M)] - col_pre(prem, Pm, M, x, PS);
    }
    const int w0 = 32 * j;
    const uint32_t ww = walk_word(Pm, M, N, NW, rev, j);
    const int nb = min(32, L + 1 - w0);
    const int nvg = (nb + 3) >> 2;   /* groups of 4 holding valid entries */
    /* group-end sums of word j, then the group and the entry where u falls (branch-free) */
    double gsum[8], gy[8];
    int ng = 0;
    {
      double yy = 1.0, acc = 0.0;
#pragma unroll
      for (int g = 0; g < 8; ++g) {   /* unscaled */
        const uint32_t nib = (ww >> (4 * g)) & 15u;
        const int c = min(max(nb - 4 * g, 0), 4);
        gy[g] = yy;
        const double2 t = t4sp(T4, c, nib);
        acc = __builtin_fma(yy, t.x, acc);
        gsum[g] = acc;
        yy = yy * t.y;
      }
      const double y = (B8 && SR_CKG > 1) ? yj : ((j == klo) ? y0 : (yj - Sp0) / acc);
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        gsum[g] = __builtin_fma(y, gsum[g], Sp0);
        gy[g] = y * gy[g];
        ng += (g < nvg && gsum[g] * inv < u) ? 1 : 0;
      }
    }
    const int gsel = min(ng, nvg - 1);
    double base = Sp0, ys = gy[0];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      if (g == gsel) ys = gy[g];
      if (g + 1 == gsel) base = gsum[g];
    }
    const uint32_t nibs = (ww >> (4 * gsel)) & 15u;
    const int cmax = min(nb - 4 * gsel, 4);
    const double P1 = __builtin_fma(ys, t4s(T4, 1, nibs), base), P2 = __builtin_fma(ys, t4s(T4, 2, nibs), base);
    const double P3 = __builtin_fma(ys, t4s(T4, 3, nibs), base), P4 = __builtin_fma(ys, t4s(T4, 4, nibs), base);
    const int nc = ((cmax > 1 && P1 * inv < u) ? 1 : 0) + ((cmax > 2 && P2 * inv < u) ? 1 : 0) +
                   ((cmax > 3 && P3 * inv < u) ? 1 : 0);
    const double Ph = (nc == 0) ? P1 : (nc == 1) ? P2 : (nc == 2) ? P3 : P4;
    const double Pp = (nc == 0) ? base : (nc == 1) ? P1 : (nc == 2) ? P2 : P3;
    const int w = w0 + 4 * gsel + nc;
    const double t = u - Ph * inv, tprev = u - Pp * inv;
    const double e = 2.0 * REL * fmin(Ph, S - Ph) * inv + ABS;
    const double eprev = 2.0 * REL * fmin(Pp, S - Pp) * inv + ABS;
    const bool prev_ok = (w == 0) || (tprev > eprev);
    const bool here_ok = (w == L) || (t < -e);
#ifndef SR_FORCE_EXACT
    if (prev_ok && here_ok) {
      res = w;
      POp = Oj + __popc(ww & ((1u << (w & 31)) - 1u));
    }
#else   /* test build: every Gibbs draw takes the exact three-pass walk */
    (void)prev_ok; (void)here_ok; (void)w; (void)Oj;
#endif
#ifdef SR_STAMPS
    if (!(prev_ok && here_ok)) atomicAdd((unsigned long long *)fbk + (prev_ok ? 2 : 1), 1ull);
#endif
  }
  if (res < 0) {
    atomicAdd((unsigned long long *)fbk, 1ull);   /* exact-walk fallbacks (rare: counted always) */
#ifdef SR_STAMPS
    if (!(S > 0.0)) atomicAdd((unsigned long long *)fbk + 3, 1ull);
#endif
    res = draw_exact(Pm, M, N, rev, o, L, u, K, tb);
    POp = walk_prefix(Pm, M, N, NW, rev, res);
  }
  GSTAMP(3);
  /* count deltas at the pick (the dt arrays of mcmc_auxa) */
  if (res == o) { dt0 = df0 = dt1 = df1 = 0; }
  else if (res < o) { int O = POo - POp; int Z = (o - res) - O; dt0 = -Z; df0 = Z; dt1 = O; df1 = -O; }
  else { int O = POp - POo; int Z = (res - o) - O; dt0 = Z; df0 = -Z; dt1 = -O; df1 = O; }
  return res;
}

/* ---- static-size Gibbs draw (columns of <= NWM words held in registers) ----------------- */
/* element idx of a register array, idx block-uniform but not a compile-time constant */
template <int NWM, typename T>
__device__ __forceinline__ T sel_u(const T (&a)[NWM], int idx)
{
  T v = a[0];
#pragma unroll
  for (int k = 1; k < NWM; ++k) v = (idx == k) ? a[k] : v;
  return v;
}

/* ones among walk entries [0, w) of the walk words wk[] */
template <int NWM>
__device__ __forceinline__ int walk_prefix_s(const uint32_t (&wk)[NWM], int w)
{
  int s = 0;
#pragma unroll
  for (int k = 0; k < NWM; ++k) {
    const int lo = 32 * k;
    const uint32_t m = (w >= lo + 32) ? 0xffffffffu : ((w > lo) ? ((1u << (w - lo)) - 1u) : 0u);
    s += __popc(wk[k] & m);
  }
  return s;
}

/* count deltas at the pick (the dt arrays of mcmc_auxa): POo, POp = ones among walk entries [0, o), [0, res) */
__device__ __forceinline__ void pick_counts(int res, int o, int POo, int POp, int &dt0, int &df0, int &dt1, int &df1)
{
  if (res == o) { dt0 = df0 = dt1 = df1 = 0; }
  else if (res < o) { int O = POo - POp; int Z = (o - res) - O; dt0 = -Z; df0 = Z; dt1 = O; df1 = -O; }
  else { int O = POp - POo; int Z = (res - o) - O; dt0 = Z; df0 = -Z; dt1 = -O; df1 = O; }
}

/* pass 2 of a register walk (draw_fast_s): locate the word, then the byte, nibble and
 * entry where u falls (the searches compare against u S), and certify the pick; -1 when it is not
 * certified (the caller runs the exact walk).  ckr / yst: S after and y at the start of each word
 * (0 / y0 before the window, unchanged after it), S the walk's total over entries [0, L]. */
template <int NWM>
__device__ __forceinline__ int walk_pick_s(const uint32_t (&wk)[NWM], const double (&ckr)[NWM], const double (&yst)[NWM],
                                           double S, int klo, int khi, int L, int N, double u, const double *T4,
                                           const double *T8, int &POp)
{
  int res = -1;
  {
    const double inv = 1.0 / S;
    const double REL = (double)(N + 33) * 0x1p-50 * SR_CERT_SCALE;   /* + the byte tables' own rounding (<= 16 ulp per entry) */
    const double ABS = (double)(N + 1) * 0x1p-39 * SR_CERT_SCALE;
    /* the words before the window hold S = 0 (< u S), so counting k < khi finds the word */
    const double uS = u * S;
    int j = 0;
#pragma unroll
    for (int k = 0; k < NWM; ++k) j += (k < khi && ckr[k] < uS) ? 1 : 0;
    j = max(j, klo);   /* (u = 0) */
    double Sp0 = 0.0, y = yst[0];
    uint32_t ww = wk[0];
    [[maybe_unused]] int Oj = 0, Ok = 0;   /* ones among walk entries [0, 32 j) (9-word walks) */
#pragma unroll
    for (int k = 0; k < NWM; ++k) {
      if (k == j) { y = yst[k]; ww = wk[k]; Oj = Ok; }
      if (k + 1 == j) Sp0 = ckr[k];   /* ckr[klo - 1] = 0 */
      if constexpr (NWM <= 9) Ok += __popc(wk[k]);
    }
    const int w0 = 32 * j;
    const int nb = min(32, L + 1 - w0);   /* walk entries in word j */
    /* byte level: the word's whole bytes from the 8-entry tables (the walk's partial last byte,
       if any, is the last candidate: its end is S itself); then the nibble, then the entry */
    const int nfb = nb >> 3, nlb = (nb + 7) >> 3;
    double2 tb8[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) tb8[g] = *reinterpret_cast<const double2 *>(T8 + 2 * ((ww >> (8 * g)) & 255u));
    double Bg[4], Yg[4];
    int nbc = 0;
    {
      double acc = Sp0, yy = y;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        Yg[g] = yy;
        acc = __builtin_fma(yy, tb8[g].x, acc);
        Bg[g] = acc;
        yy = yy * tb8[g].y;
        nbc += (g < nfb && acc < uS) ? 1 : 0;
      }
    }
    const int bsel = min(nbc, nlb - 1);
    double base_b = Sp0, y_b = y;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (g == bsel) y_b = Yg[g];
      if (g + 1 == bsel) base_b = Bg[g];
    }
    const uint32_t bv = (ww >> (8 * bsel)) & 255u;
    const int ce = min(nb - 8 * bsel, 8), c_lo = min(ce, 4), c_hi = ce - c_lo;
    const double2 tlo = t4sp(T4, c_lo, bv & 15u);
    const double N0 = __builtin_fma(y_b, tlo.x, base_b);
    const bool nsel = c_hi > 0 && N0 < uS;
    const int gsel = 2 * bsel + (nsel ? 1 : 0);
    const double base = nsel ? N0 : base_b, ys = nsel ? y_b * tlo.y : y_b;
    const uint32_t nibs = nsel ? (bv >> 4) : (bv & 15u);
    const int cmax = nsel ? c_hi : c_lo;
    const double P1 = __builtin_fma(ys, t4s(T4, 1, nibs), base), P2 = __builtin_fma(ys, t4s(T4, 2, nibs), base);
    const double P3 = __builtin_fma(ys, t4s(T4, 3, nibs), base), P4 = __builtin_fma(ys, t4s(T4, 4, nibs), base);
    const int nc = ((cmax > 1 && P1 < uS) ? 1 : 0) + ((cmax > 2 && P2 < uS) ? 1 : 0) + ((cmax > 3 && P3 < uS) ? 1 : 0);
    const double Ph = (nc == 0) ? P1 : (nc == 1) ? P2 : (nc == 2) ? P3 : P4;
    const double Pp = (nc == 0) ? base : (nc == 1) ? P1 : (nc == 2) ? P2 : P3;
    const int w = w0 + 4 * gsel + nc;
    const double t = u - Ph * inv, tprev = u - Pp * inv;
    const double e = 2.0 * REL * fmin(Ph, S - Ph) * inv + ABS;
    const double eprev = 2.0 * REL * fmin(Pp, S - Pp) * inv + ABS;
    const bool prev_ok = (w == 0) || (tprev > eprev);
    const bool here_ok = (w == L) || (t < -e);
#ifndef SR_FORCE_EXACT
    if (prev_ok && here_ok) {
      res = w;
      if constexpr (NWM <= 9) POp = Oj + __popc(ww & ((1u << (w & 31)) - 1u));
      else POp = walk_prefix_s<NWM>(wk, res);   /* (the tracked form spills in the 17-word kernel) */
    }
#else   /* test build: every Gibbs draw takes the exact three-pass walk */
    (void)prev_ok; (void)here_ok; (void)w;
#endif
  }
  return res;
}

/* draw_fast with the walk words in registers, fully unrolled and branch-free (the measured cost
 * of a loop trip with a taken branch on gfx950 is ~36 cycles, more than the work it guards).
 * Same approximation and certification as draw_fast; fallback to draw_exact on failure. */
template <int NWM>
__device__ __forceinline__ int draw_fast_s(const uint32_t (&wk)[NWM], const uint32_t *Pm, int M, int N, bool rev, int o,
                                           int L, int POo, double u, const CD &K, const sr_mtab &tb, double vA, double vB,
                                           const double *T4, const double *T8, uint64_t *fbk, int &dt0, int &df0, int &dt1,
                                           int &df1)
{
  /* POo: ones among walk entries [0, o), from the caller's column prefix table */
  const int nk = (L >> 5) + 1;
  /* pass 0: window of words that can hold mass above 2^-40 relative to entry o.  q at a word
     start w0 is F(o) - F(w0), F(w) = zeros before w * vA + ones before w * vB = w vA + O(w) (vB - vA)
     (the window only bounds the skipped mass: the pick is certified independently of it). */
  int klo = NWM, khi = -1;
  double qlo = 0.0;
  [[maybe_unused]] uint32_t lowm = 0u;   /* 17-word walks: words whose start q lies below -700 (pass 2) */
  const int kl = L >> 5, nbl = (L & 31) + 1;   /* the walk's last word and its entries */
  uint32_t wl = 0u;                              /* word kl */
  {
    const double dv = vB - vA;
    const double Fo = __builtin_fma((double)POo, dv, (double)o * vA);
    int O = 0;   /* ones among walk entries [0, 32k) */
    const uint32_t lastm = (2u << (L & 31)) - 1u;
#pragma unroll
    for (int k = 0; k < NWM; ++k) {
      const bool full = k < kl;   /* (words past kl are outside the walk: not in the window) */
      const int nb = full ? 32 : nbl;
      const uint32_t vm = full ? 0xffffffffu : lastm;
      double qs;
      if constexpr (NWM <= 9) qs = Fo - __builtin_fma((double)O, dv, (double)(32 * k) * vA);
      else {   /* the 17-word walks keep the two-sided form: the F form spills there (+9 % kernel time at N = 400) */
        const int w0 = 32 * k;
        qs = (w0 <= o) ? ((double)((o - w0) - (POo - O)) * vA + (double)(POo - O) * vB)
                       : -((double)((w0 - o) - (O - POo)) * vA + (double)(O - POo) * vB);
      }
      const int ones = __popc(wk[k] & vm);
      const double ub = qs - (double)(nb - ones) * vA;
      const bool in = (k < nk) && ub > -SR_WIN_T;
      if constexpr (NWM > 9) lowm |= (qs < -700.0 ? 1u : 0u) << k;
      const bool first = in && klo == NWM;
      qlo = first ? qs : qlo;
      klo = first ? k : klo;
      khi = in ? k : khi;
      O += __popc(wk[k]);
      if constexpr (NWM <= 9) wl = (k == kl) ? wk[k] : wl;
    }
  }
#ifdef SR_STAMP_FINE
  {   /* window statistics: words per draw, wave max, walk words */
    const int wn = khi - klo + 1;
    int wmax = wn;
    for (int off_ = 32; off_ > 0; off_ >>= 1) wmax = max(wmax, __shfl_xor(wmax, off_));
    atomicAdd((unsigned long long *)fbk + 26, (unsigned long long)wn);
    if ((threadIdx.x & 63) == 0) atomicAdd((unsigned long long *)fbk + 27, (unsigned long long)wmax);
    atomicAdd((unsigned long long *)fbk + 28, (unsigned long long)nk);
    atomicAdd((unsigned long long *)fbk + 29, 1ull);
  }
#endif
  /* pass 1: S over the window; word-start y and end-of-word checkpoints kept in registers.
     Byte steps: T8[byte] = {sum of the byte's 8 prefix products, their product}; T8[256] =
     {0, 1} is the dead entry, read for every byte outside the window or not wholly inside the
     walk (it leaves S and y unchanged), so no step needs a select.  A word's 4 entries are read
     together (one LDS round trip per word) and summed in Horner form, W = s0 + p0 (s1 + p1 (s2 +
     p2 s3)), y *= (p0 p1)(p2 p3): the y chain takes one multiply per word (dead entries are
     trailing, so W and the product stay exact for them); each entry's value keeps at most as many
     roundings as the byte-by-byte chain it replaces, inside REL.  The walk's partial last byte
     ((L + 1) mod 8 entries) follows from the 4-entry tables (T4 rows c = 0..4). */
  const double y0 = exp2_split(qlo);
  double S = 0.0;
  double ckr[NWM], yst[NWM];
  double y = y0;
  {
    /* word k's 4 entries (whole bytes of the walk inside the window; the dead entry otherwise) */
    auto wload = [&](int k, double2 (&t)[4]) {
      const bool inw = k >= klo && k <= khi;
      int nfk;   /* whole bytes of the walk in word k (khi <= kl) */
      if constexpr (NWM <= 9) nfk = inw ? ((k < kl) ? 4 : (nbl >> 3)) : 0;
      else nfk = inw ? min(max((L + 1 - 32 * k) >> 3, 0), 4) : 0;   /* (the form above is 1.8 % slower here) */
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint32_t e = (g < nfk) ? ((wk[k] >> (8 * g)) & 255u) : 256u;
        t[g] = *reinterpret_cast<const double2 *>(T8 + 2 * e);
      }
    };
    double2 t[4], tn[4];
    wload(0, t);
#pragma unroll
    for (int k = 0; k < NWM; ++k) {
      if (k + 1 < NWM) wload(k + 1, tn);   /* next word's reads in flight while this word is summed */
      yst[k] = y;
      {   /* the word's 4 byte steps in Horner form: one multiply on the y chain per word */
        const double w23 = __builtin_fma(t[2].y, t[3].x, t[2].x);
        const double w13 = __builtin_fma(t[1].y, w23, t[1].x);
        const double W = __builtin_fma(t[0].y, w13, t[0].x);
        const double pw = (t[0].y * t[1].y) * (t[2].y * t[3].y);
        S = __builtin_fma(y, W, S);
        y = y * pw;
      }
      ckr[k] = S;
#pragma unroll
      for (int g = 0; g < 4; ++g) t[g] = tn[g];
      __builtin_amdgcn_sched_barrier(0);   /* one word of reads ahead, no more (register pressure; two words
                                              ahead: 10 -> 19 VGPR spills, +0.7 %, profiles/r05r_ab_gibbs_ahead.json) */
    }
    /* the partial byte (c8 entries) when its word lies in the window */
    const int nfull = (L + 1) >> 3, c8 = (L + 1) & 7, kb = nfull >> 2;
    const bool actb = c8 > 0 && kb >= klo && kb <= khi;
    uint32_t wb = wl;   /* word kb = kl when c8 > 0 (the 17-word kernel selects it here: tracking spills there) */
    if constexpr (NWM > 9) {
#pragma unroll
      for (int k = 0; k < NWM; ++k) wb |= wk[k] & (0u - (uint32_t)(k == kb));
    }
    const uint32_t eb = (wb >> (8 * (nfull & 3))) & 255u;
    const double2 tlo = t4sp(T4, actb ? min(c8, 4) : 0, eb & 15u);
    const double shi = t4s(T4, actb ? max(c8 - 4, 0) : 0, eb >> 4);
    S = __builtin_fma(y, tlo.x, S);
    S = __builtin_fma(y * tlo.y, shi, S);
  }
  /* pass 2: locate the word, then the byte, nibble and entry where u falls (the searches compare
     against u S; the pick is certified below, independently of how it was found) */
  int res = -1, POp = 0;   /* the pick and the ones among walk entries [0, pick) */
  /* Underflow: y at a window word start is 2^q up to rounding, and a chain that sank into the
     subnormal range would lose its relative precision.  Only zeros raise q (by |vA| each) and the
     window's last word reaches q > -40, so every window word start lies above -40 - 32 nk |vA|;
     d >= 0.2 and c <= 0.1 always (mcmc_samplebeta's bounds MIND / MAXC, mcmc.h:27-30; the initial
     values log .01 / log .3, mcmc.c:419-420) give |vA| = log2((1 - c) / d) <= log2 5 = 2.33.  Walks of
     <= 9 words therefore stay above 2^-710 and next words' y above 2^-1018 (a word's product is
     >= 2^-32 vB >= 2^-309): no test.  17-word walks can sink further: a window word start below
     2^-700 sends the draw to the exact path (pass 0's exact q, a bit mask; a per-draw test costs
     2 % of the 9-word kernel, profiles/r03n_ab_yguard.json). */
  bool yok = true;
  if constexpr (NWM > 9) yok = klo > khi || (lowm & ((2u << khi) - 1u) & ~((1u << klo) - 1u)) == 0u;
  if (S > 0.0 && S < 0x1p1000 && yok) res = walk_pick_s<NWM>(wk, ckr, yst, S, klo, khi, L, N, u, T4, T8, POp);
  if (res < 0) {
    atomicAdd((unsigned long long *)fbk, 1ull);   /* exact-walk fallbacks (rare: counted always) */
    res = draw_exact(Pm, M, N, rev, o, L, u, K, tb);
    POp = walk_prefix_s<NWM>(wk, res);
  }
  pick_counts(res, o, POo, POp, dt0, df0, dt1, df1);
  return res;
}


/* ---- pair kernels: two lanes per taxon ---------------------------------------------------
 * Lanes 2t and 2t+1 of a wave share taxon t; the even lane ("lo") holds walk words 0..4 of a
 * Gibbs draw, the odd lane ("hi") words 5..8 (walks of <= 9 words: N <= 287).  Partner values
 * travel by one DPP quad_perm [1,0,3,2] (lane ^ 1) each. */
__device__ __forceinline__ int pair_swap_i32(int x) { return __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ double pair_swap_f64(double v)
{
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)pair_swap_i32((int)(uint32_t)b), hi = (uint32_t)pair_swap_i32((int)(uint32_t)(b >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

/* draw_fast_s<9> (mcmc_auxa + mcmc_logtop + mcmc_randompick, certified) with the walk split over a
 * lane pair: each lane runs passes 0 and 1 over its five words; the hi lane's chain starts from
 * y' = 1 at word 5 and is rescaled by the lo lane's y at word 5 (S = S_lo + y5 S'_hi, checkpoints
 * S_lo + y5 ck'_k: a re-association of the same products, two more roundings per value -- inside
 * REL, which gains 8 units for them); pass 2 runs identically in both lanes on word j's data taken
 * from the lane that holds it.  wk: this lane's words 5h .. 5h+4 (word 9 = 0).  Both lanes return
 * the same pick and count deltas.  Call pair-uniformly (both lanes active). */
__device__ __forceinline__ int draw_pair9(const uint32_t (&wk)[5], int h, const uint32_t *Pm, int M, int N, int NW, bool rev,
                                          int o, int L, int POo, double u, const CD &K, const sr_mtab &tb, double vA,
                                          double vB, const double *T4, const double *T8, uint64_t *fbk, int &dt0, int &df0,
                                          int &dt1, int &df1)
{
  constexpr int NWM = 9, NH = 5;
  const int k0 = NH * h;
  const int nk = (L >> 5) + 1;
  const int kl = L >> 5, nbl = (L & 31) + 1;
  /* ---- pass 0: window of words that can hold mass above 2^-40 relative to entry o */
  int Otot = 0;
#pragma unroll
  for (int i = 0; i < NH; ++i) Otot += __popc(wk[i]);
  const int Op = pair_swap_i32(Otot);
  int klo = NWM, khi = -1;
  double qlo = 0.0;
  uint32_t wl = 0u;
  {
    const double dv = vB - vA;
    const double Fo = __builtin_fma((double)POo, dv, (double)o * vA);
    int O = h ? Op : 0;
    const uint32_t lastm = (2u << (L & 31)) - 1u;
#pragma unroll
    for (int i = 0; i < NH; ++i) {
      const int k = k0 + i;
      const bool full = k < kl;
      const int nb = full ? 32 : nbl;
      const uint32_t vm = full ? 0xffffffffu : lastm;
      const double qs = Fo - __builtin_fma((double)O, dv, (double)(32 * k) * vA);
      const int ones = __popc(wk[i] & vm);
      const double ub = qs - (double)(nb - ones) * vA;
      const bool in = (k < nk) && ub > -SR_WIN_T;
      const bool first = in && klo == NWM;
      qlo = first ? qs : qlo;
      klo = first ? k : klo;
      khi = in ? k : khi;
      O += __popc(wk[i]);
      wl = (k == kl) ? wk[i] : wl;
    }
    const int klo_p = pair_swap_i32(klo), khi_p = pair_swap_i32(khi);
    const double qlo_p = pair_swap_f64(qlo);
    const uint32_t wl_p = (uint32_t)pair_swap_i32((int)wl);
    qlo = (klo <= klo_p) ? qlo : qlo_p;
    klo = min(klo, klo_p);
    khi = max(khi, khi_p);
    wl |= wl_p;
  }
  /* ---- pass 1: my words' sums (lo: from y0; hi: relative to y = 1 at word 5), then combined */
  const double y0 = exp2_split(qlo);
  double S = 0.0;
  double ckr[NH], yst[NH];
  double y = h ? 1.0 : y0;
  {
    auto wload = [&](int i, double2 (&t)[4]) {
      const int k = k0 + i;
      const bool inw = k >= klo && k <= khi;
      const int nfk = inw ? ((k < kl) ? 4 : (nbl >> 3)) : 0;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint32_t e = (g < nfk) ? ((wk[i] >> (8 * g)) & 255u) : 256u;
        t[g] = *reinterpret_cast<const double2 *>(T8 + 2 * e);
      }
    };
#pragma unroll
    for (int i = 0; i < NH; ++i) {
      double2 t[4];   /* no read-ahead: four waves per SIMD cover the table reads' latency */
      wload(i, t);
      yst[i] = y;
      {
        const double w23 = __builtin_fma(t[2].y, t[3].x, t[2].x);
        const double w13 = __builtin_fma(t[1].y, w23, t[1].x);
        const double W = __builtin_fma(t[0].y, w13, t[0].x);
        const double pw = (t[0].y * t[1].y) * (t[2].y * t[3].y);
        S = __builtin_fma(y, W, S);
        y = y * pw;
      }
      ckr[i] = S;
    }
    /* the partial byte (c8 entries), by the lane that holds its word, when it lies in the window */
    const int nfull = (L + 1) >> 3, c8 = (L + 1) & 7, kb = nfull >> 2;
    const bool actb = c8 > 0 && kb >= klo && kb <= khi && kb >= k0 && kb < k0 + NH;
    const uint32_t eb = (wl >> (8 * (nfull & 3))) & 255u;
    const double2 tlo = t4sp(T4, actb ? min(c8, 4) : 0, eb & 15u);
    const double shi = t4s(T4, actb ? max(c8 - 4, 0) : 0, eb >> 4);
    S = __builtin_fma(y, tlo.x, S);
    S = __builtin_fma(y * tlo.y, shi, S);
  }
  const double S_p = pair_swap_f64(S), y_p = pair_swap_f64(y);
  const double S_lo = h ? S_p : S, y5 = h ? y_p : y, S_hi = h ? S : S_p;
  const double St = S_lo + y5 * S_hi;
  {
    const double cb = h ? S_lo : 0.0, cs = h ? y5 : 1.0;
#pragma unroll
    for (int i = 0; i < NH; ++i) { ckr[i] = cb + cs * ckr[i]; yst[i] = cs * yst[i]; }
  }
  /* ---- pass 2 (both lanes, identical data): word, byte, nibble, entry; certification */
  int res = -1, POp = 0;
  bool uf = false;   /* as draw_fast_s: a window word start below 2^-700 takes the exact path */
#pragma unroll
  for (int i = 0; i < NH; ++i) uf |= k0 + i >= klo && k0 + i <= khi && yst[i] < 0x1p-700;
  uf = uf || pair_swap_i32(uf ? 1 : 0) != 0;
  if (St > 0.0 && St < 0x1p1000 && !uf) {
    const double inv = 1.0 / St;
    const double REL = (double)(N + 41) * 0x1p-50 * SR_CERT_SCALE;
    const double ABS = (double)(N + 1) * 0x1p-39 * SR_CERT_SCALE;
    const double uS = u * St;
    int jl = 0;
#pragma unroll
    for (int i = 0; i < NH; ++i) jl += (k0 + i < khi && ckr[i] < uS) ? 1 : 0;
    int j = jl + pair_swap_i32(jl);
    j = max(j, klo);
    const int ij = j - k0, ijm = j - 1 - k0;
    double cy = 0.0, csp = 0.0;
    uint32_t cww = 0u;
    int cO = h ? Op : 0;   /* ones among walk entries [0, 32 j) when I hold word j */
#pragma unroll
    for (int i = 0; i < NH; ++i) {
      if (i == ij) { cy = yst[i]; cww = wk[i]; }
      cO += (i < ij) ? __popc(wk[i]) : 0;
      if (i == ijm) csp = ckr[i];
    }
    const double cy_p = pair_swap_f64(cy), csp_p = pair_swap_f64(csp);
    const uint32_t cww_p = (uint32_t)pair_swap_i32((int)cww);
    const int cO_p = pair_swap_i32(cO);
    const bool own = ij >= 0 && ij < NH, ownm = ijm >= 0 && ijm < NH;
    const double yj = own ? cy : cy_p, Sp0 = ownm ? csp : csp_p;
    const uint32_t ww = own ? cww : cww_p;
    const int Oj = own ? cO : cO_p;
    const int w0 = 32 * j;
    const int nb = min(32, L + 1 - w0);
    const int nfb = nb >> 3, nlb = (nb + 7) >> 3;
    double2 tb8[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) tb8[g] = *reinterpret_cast<const double2 *>(T8 + 2 * ((ww >> (8 * g)) & 255u));
    double Bg[4], Yg[4];
    int nbc = 0;
    {
      double acc = Sp0, yy = yj;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        Yg[g] = yy;
        acc = __builtin_fma(yy, tb8[g].x, acc);
        Bg[g] = acc;
        yy = yy * tb8[g].y;
        nbc += (g < nfb && acc < uS) ? 1 : 0;
      }
    }
    const int bsel = min(nbc, nlb - 1);
    double base_b = Sp0, y_b = yj;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (g == bsel) y_b = Yg[g];
      if (g + 1 == bsel) base_b = Bg[g];
    }
    const uint32_t bv = (ww >> (8 * bsel)) & 255u;
    const int ce = min(nb - 8 * bsel, 8), c_lo = min(ce, 4), c_hi = ce - c_lo;
    const double2 tlo = t4sp(T4, c_lo, bv & 15u);
    const double N0 = __builtin_fma(y_b, tlo.x, base_b);
    const bool nsel = c_hi > 0 && N0 < uS;
    const int gsel = 2 * bsel + (nsel ? 1 : 0);
    const double base = nsel ? N0 : base_b, ys = nsel ? y_b * tlo.y : y_b;
    const uint32_t nibs = nsel ? (bv >> 4) : (bv & 15u);
    const int cmax = nsel ? c_hi : c_lo;
    const double P1 = __builtin_fma(ys, t4s(T4, 1, nibs), base), P2 = __builtin_fma(ys, t4s(T4, 2, nibs), base);
    const double P3 = __builtin_fma(ys, t4s(T4, 3, nibs), base), P4 = __builtin_fma(ys, t4s(T4, 4, nibs), base);
    const int nc = ((cmax > 1 && P1 < uS) ? 1 : 0) + ((cmax > 2 && P2 < uS) ? 1 : 0) + ((cmax > 3 && P3 < uS) ? 1 : 0);
    const double Ph = (nc == 0) ? P1 : (nc == 1) ? P2 : (nc == 2) ? P3 : P4;
    const double Pp = (nc == 0) ? base : (nc == 1) ? P1 : (nc == 2) ? P2 : P3;
    const int w = w0 + 4 * gsel + nc;
    const double t = u - Ph * inv, tprev = u - Pp * inv;
    const double e = 2.0 * REL * fmin(Ph, St - Ph) * inv + ABS;
    const double eprev = 2.0 * REL * fmin(Pp, St - Pp) * inv + ABS;
    const bool prev_ok = (w == 0) || (tprev > eprev);
    const bool here_ok = (w == L) || (t < -e);
#ifndef SR_FORCE_EXACT
    if (prev_ok && here_ok) {
      res = w;
      POp = Oj + __popc(ww & ((1u << (w & 31)) - 1u));
    }
#else
    (void)prev_ok; (void)here_ok; (void)w; (void)Oj;
#endif
  }
  if (res < 0) {
    if (h == 0) atomicAdd((unsigned long long *)fbk, 1ull);   /* exact-walk fallbacks (counted once per taxon) */
    res = draw_exact(Pm, M, N, rev, o, L, u, K, tb);
    POp = walk_prefix(Pm, M, N, NW, rev, res);
  }
  if (res == o) { dt0 = df0 = dt1 = df1 = 0; }
  else if (res < o) { int O = POo - POp; int Z = (o - res) - O; dt0 = -Z; df0 = Z; dt1 = O; df1 = -O; }
  else { int O = POp - POo; int Z = (res - o) - O; dt0 = Z; df0 = -Z; dt1 = -O; df1 = O; }
  return res;
}

/* the forward walk words of column m (positions), NW <= NWM */
template <int NWM>
__device__ __forceinline__ void load_fwd(const uint32_t *Pm, int M, int NW, uint32_t (&fw)[NWM])
{
#pragma unroll
  for (int k = 0; k < NWM; ++k) fw[k] = (k < NW) ? Pm[min(k, NW - 1) * M] : 0u;
}

/* the reversed walk words (positions N-1-w) built from the forward words fw[] */
template <int NWM>
__device__ __forceinline__ void make_rev(const uint32_t *Pm, int M, int N, int NW, const uint32_t (&fw)[NWM], uint32_t (&rw)[NWM])
{
  /* reversed word k = brev(column bits [s, s+32)), s = N - 32 - 32k = 32 (q - 1 - k) + r: built
     from fw[] with compile-time indices inside a block-uniform switch on q = N / 32 (a select at
     a runtime index made the compiler spill fw to scratch) */
  const int q = N >> 5, r = N & 31;
  bool done = false;
#pragma unroll
  for (int Q = 0; Q <= NWM; ++Q) {
    if (q != Q) continue;
#pragma unroll
    for (int k = 0; k < NWM; ++k) {
      const int wi = Q - 1 - k;
      const uint32_t lo = (wi >= 0 && wi < NWM) ? fw[wi >= 0 && wi < NWM ? wi : 0] : 0u;
      const uint32_t hi = (wi + 1 >= 0 && wi + 1 < NWM) ? fw[(wi + 1 >= 0 && wi + 1 < NWM) ? wi + 1 : 0] : 0u;
      const uint32_t hiv = (wi + 1 < NW) ? hi : 0u;
      const uint32_t v = r ? ((lo >> r) | (hiv << (32 - r))) : lo;
      rw[k] = (k < NW) ? __brev(v) : 0u;
    }
    done = true;
  }
  if (!done) {
#pragma unroll
    for (int k = 0; k < NWM; ++k) rw[k] = (k < NW) ? walk_word(Pm, M, N, NW, true, k) : 0u;
  }
}

/* bits of positions [lo, hi] inside word w */
__device__ __forceinline__ uint32_t range_mask(int w, int lo, int hi)
{
  const int b0 = 32 * w;
  lo = max(lo, b0);
  hi = min(hi, b0 + 31);
  if (hi < lo) return 0u;
  const int n = hi - lo + 1;
  return (n == 32) ? 0xffffffffu : (((1u << n) - 1u) << (lo - b0));
}

/* ones of column m in [lo, mid) and [mid, hi) (one pass over the words) */
__device__ __forceinline__ void ones_split(const uint32_t *Pm, int M, int lo, int mid, int hi, int &O1, int &O2)
{
  O1 = 0; O2 = 0;
  if (hi <= lo) return;
  for (int w = lo >> 5; w <= ((hi - 1) >> 5); ++w) {
    const uint32_t word = Pm[w * M];
    O1 += __popc(word & range_mask(w, lo, mid - 1));
    O2 += __popc(word & range_mask(w, mid, hi - 1));
  }
}

/* recompute column m's prefix table (rows 0..NW) */
__device__ __forceinline__ void col_pre_build(uint16_t *prem, const uint32_t *Pm, int M, int NW, int PS = 0)
{
  const int S = PS ? PS : M;
  int s = 0;
  for (int k0 = 0; k0 < NW; k0 += 8) {   /* 8 independent loads per round */
    uint32_t wv[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) wv[t] = Pm[min(k0 + t, NW - 1) * M];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      if (k0 + t < NW) prem[(k0 + t) * S] = (uint16_t)s;
      s += (k0 + t < NW) ? __popc(wv[t]) : 0;
    }
  }
  prem[NW * S] = (uint16_t)s;
}

__device__ __forceinline__ int ininterval(int i, int a, int b, int inc1, int inc2)   /* mcmc.c:1097-1124 */
{
  /* i inside the interval of ends a, b (ordered first; inc1 / inc2 include the lower / upper end): for integers
     that is L <= i <= H with L = lo + !inc1, H = hi - !inc2, one unsigned compare per lane (the ends and flags
     are block-uniform: scalar ALU) */
#if SR_ININT_FAST
  const int lo = min(a, b), hi = max(a, b);
  const int L = lo + (inc1 ? 0 : 1), H = hi - (inc2 ? 0 : 1);
  return (H >= L) && (uint32_t)(i - L) <= (uint32_t)(H - L);
#else
  int r;
  if (a > b) { r = a; a = b; b = r; }
  r = inc1 ? (a <= i) : (a < i);
  if (r) r = inc2 ? (i <= b) : (i < b);
  return r;
#endif
}

/* hard-site positions hp[0..nh) are ascending (their relative order never changes) */
__device__ __forceinline__ int hard_count(const int *hp, int nh, int lo, int hi)
{
  int s = 0;
  for (int k = 0; k < nh; ++k) s += (hp[k] >= lo && hp[k] <= hi) ? 1 : 0;
  return s;
}

__device__ __forceinline__ bool is_hard(const int *hp, int nh, int p)
{
  bool h = false;
  for (int k = 0; k < nh; ++k) h |= (hp[k] == p);
  return h;
}

__device__ __forceinline__ void wsync()
{
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

/* Wave-wide integer sum with DPP row operations (no LDS round trips); every lane of the wave
 * must be active.  Result is wave-uniform. */
__device__ __forceinline__ int wave_sum_i32(int x)
{
  x += __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);    /* quad_perm [1,0,3,2] */
  x += __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);    /* quad_perm [2,3,0,1] */
  x += __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false);   /* row_half_mirror */
  x += __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false);   /* row_mirror: row sums */
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);   /* row_bcast:15 -> rows 1, 3 */
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);   /* row_bcast:31 -> rows 2, 3 */
  return __builtin_amdgcn_readlane(x, 63);
}


/* The wave sums of 32 values at once by a transposed butterfly: at exchange step k (partner lane ^ 2^k) a lane
 * keeps one half of the values it holds (by lane bit k) and adds its partner's copy of that half, so 32 values
 * cost 16 + 8 + 4 + 2 + 1 + 1 adds (plus the selects and moves) instead of 32 six-step reductions each read
 * out by one lane.  Partners: quad_perm (xor 1, 2), row_shl/row_shr by 4 and 8 with bank masks (xor 4, 8),
 * ds_swizzle (xor 16), ds_bpermute (xor 32).  Integer adds: exact in any order.  On return lane l (and l ^ 32)
 * holds the total of value u[16 (l & 1) + s], s = 8 b1 + 4 b2 + 2 b3 + b4 with b_k = bit k of l. */
__device__ __forceinline__ uint32_t wave_sum32_t(uint32_t (&u)[32], int lane)
{
  {
    const bool b = lane & 1;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t keep = b ? u[16 + k] : u[k], send = b ? u[k] : u[16 + k];
      u[k] = keep + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)send, 0xB1, 0xF, 0xF, false);   /* xor 1 */
    }
  }
  {
    const bool b = (lane >> 1) & 1;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t keep = b ? u[8 + k] : u[k], send = b ? u[k] : u[8 + k];
      u[k] = keep + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)send, 0x4E, 0xF, 0xF, false);   /* xor 2 */
    }
  }
  {
    const bool b = (lane >> 2) & 1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t keep = b ? u[4 + k] : u[k], send = b ? u[k] : u[4 + k];
      int r = __builtin_amdgcn_update_dpp(0, (int)send, 0x104, 0xF, 0x5, false);   /* row_shl:4 into banks 0, 2 */
      r = __builtin_amdgcn_update_dpp(r, (int)send, 0x114, 0xF, 0xA, false);       /* row_shr:4 into banks 1, 3 */
      u[k] = keep + (uint32_t)r;
    }
  }
  {
    const bool b = (lane >> 3) & 1;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t keep = b ? u[2 + k] : u[k], send = b ? u[k] : u[2 + k];
      int r = __builtin_amdgcn_update_dpp(0, (int)send, 0x108, 0xF, 0x3, false);   /* row_shl:8 into banks 0, 1 */
      r = __builtin_amdgcn_update_dpp(r, (int)send, 0x118, 0xF, 0xC, false);       /* row_shr:8 into banks 2, 3 */
      u[k] = keep + (uint32_t)r;
    }
  }
  {
    const bool b = (lane >> 4) & 1;
    const uint32_t keep = b ? u[1] : u[0], send = b ? u[0] : u[1];
    u[0] = keep + (uint32_t)__builtin_amdgcn_ds_swizzle((int)send, 0x401F);   /* bit mode: lane ^ 16 */
  }
  return u[0] + (uint32_t)__builtin_amdgcn_ds_bpermute((lane ^ 32) << 2, (int)u[0]);
}

/* Exact delta: the reference's sequential `delta += term` over ascending m (mcmc.c:1214,
 * 1435, 1630), computed by lane 0 of the calling wave and broadcast through its slot.
 * Zero terms are skipped (adding +-0 is exact; s is never -0.0).  Nonzero terms were
 * compacted per 64-taxon chunk (ascending m) into cbuf with counts ccnt. */
__device__ __forceinline__ double exact_sum_wave(const double *cbuf, const int *ccnt, int nch, double *slot, int lane,
                                                 int CH = 64)
{
  if (lane == 0) {
    double s = 0.0;
    for (int ch = 0; ch < nch; ++ch) {
      const int n = ccnt[ch];
      const double *p = cbuf + ch * CH;
      int j = 0;
      for (; j + 4 <= n; j += 4) {
        const double a0 = p[j], a1 = p[j + 1], a2 = p[j + 2], a3 = p[j + 3];
        s = s + a0; s = s + a1; s = s + a2; s = s + a3;
      }
      for (; j < n; ++j) s = s + p[j];
    }
    *slot = s;
  }
  wsync();
  const double r = *slot;
  wsync();
  return r;
}

/* Split chains: the exchange data crosses workgroups (other CUs, possibly other XCDs), so it is
 * written and read with relaxed agent-scope atomics -- accesses that bypass the caches not coherent
 * across the agent -- and a flag store follows the data only after s_waitcnt (xsync in the kernel). */
template <typename T> __device__ __forceinline__ void xst(T *p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <typename T> __device__ __forceinline__ T xld(const T *p)
{
  return __hip_atomic_load(const_cast<T *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* exact_sum_wave for terms in HBM (gm kernels): every wave reads 4 chunks per round trip (one
 * coalesced load per lane) and adds them in chunk and position order through readlane, so the
 * sum is the same sequential sum and is wave-uniform in every wave (no broadcast).  XA: terms and
 * counts written by the other half of a split chain (agent-scope loads). */
template <bool XA>
__device__ __forceinline__ double exact_sum_gm(const double *cbuf, const int *ccnt, int nch, int lane, int CH)
{
  double s = 0.0;
  for (int c0 = 0; c0 < nch; c0 += 4) {
    double v[4];
    int n[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      n[q] = (c0 + q < nch) ? (XA ? xld(ccnt + c0 + q) : ccnt[c0 + q]) : 0;
      n[q] = __builtin_amdgcn_readfirstlane(n[q]);
      const double *pq = cbuf + (size_t)(c0 + q) * CH + lane;
      v[q] = (lane < n[q]) ? (XA ? xld(pq) : *pq) : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      for (int l = 0; l < n[q]; ++l) s = s + readlane_f64(v[q], l);
  }
  return s;
}

/* ---------------------------------------------------------------- proposals */
#define PK_PI1 1
#define PK_PI2 20
#define PK_SWAP 21
#define PK_PI3 3
/* order within a sweep: pi2(swap), then 5 x (pi1, pi2, pi3) (mcmc.c:237-243) */
__device__ __forceinline__ int prop_kind(int p) { return p == 0 ? PK_SWAP : ((p - 1) % 3 == 0 ? PK_PI1 : ((p - 1) % 3 == 1 ? PK_PI2 : PK_PI3)); }

/* a drawn proposal (block-uniform values) */
struct Prop { int i, j, ii, jj, inc1, inc2, Kn, r0; };   /* r0: non-hard rank of i (pi3) */

/* Per-wave hard-site tables (hard positions hp[] ascending): hcnt[x] = #hard positions < x
 * (x = 0..N), nhall[r] = position of the r-th non-hard position.  Rebuilt whenever hp moves. */
/* wt: this wave writes hcnt / nhall (false: another wave writes the block's shared copy; hbw is always the wave's) */
__device__ __forceinline__ void build_hard_tables(const int *hp, int nh, int N, int NW, uint32_t *hbw, int16_t *hcnt,
                                                  int16_t *nhall, int lane, bool wt = true)
{
  /* hard bitmap (hbw: this wave's NW words, NW <= 64), then ranks by ballot over positions */
  for (int w = lane; w < NW; w += 64) hbw[w] = 0u;
  wsync();
  for (int k = lane; k < nh; k += 64) { const int h = hp[k]; atomicOr(&hbw[h >> 5], 1u << (h & 31)); }
  wsync();
  int base = 0;
  for (int x0 = 0; x0 <= N; x0 += 64) {
    const int x = x0 + lane;
    const bool h = (x < N) && ((hbw[min(x, N - 1) >> 5] >> (x & 31)) & 1u);
    const uint64_t msk = __ballot(h && x < N);
    const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(msk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)msk, 0u));
    if (wt && x <= N) hcnt[x] = (int16_t)(base + below);
    if (wt && x < N && !h) nhall[x - (base + below)] = (int16_t)x;
    base += __popcll(msk);
  }
  wsync();
}

/* One entry of the lane-parallel proposal tables (ptab, [5][128] u32 in LDS): "a proposal of kind `part`
 * starting at word offset o" from the stream position whose ring index is `base` (`avail` words resident
 * from it), with the GSL draws of mcmc.c under the hypothesis that no uniform_int rejects and the
 * uniform_pos word is nonzero (ok bit 25; else the scalar path takes over at that proposal):
 *   part 0  pi1  (mcmc.c:1133-1160): words o, o+1, uniform_pos at o+2;  i | j << 12 | veto << 24 | ok << 25
 *   part 1  pi2  (mcmc.c:1317-1364): words o, o+1, [o+2, o+3 inc], uniform_pos at o+4; + inc1 << 26 | inc2 << 27
 *   part 2  pi3  (mcmc.c:1495-1565): words o..o+3, uniform_pos at o+4; + ranks {r0, Kn} at ptab[384 + o]
 *   part 3  swap (mcmc.c:1317-1364, j = i + 1): word o, [o+1, o+2 inc], uniform_pos at o+3 (at 512 + o)
 * part -1: parts 0-2 together from one load of the words (a wave's own refresh).
 * hcnt / nhall: the caller's wave copy of the hard-site tables (identical in every wave). */
__device__ __forceinline__ void ptab_fill(uint32_t *ptab, const uint32_t *ring, uint32_t base, int avail, int o, int part,
                                          int N, int nh, const int16_t *hcnt, const int16_t *nhall, const UDivM &mdN,
                                          const UDivM &mdN1, const UDivM &md2, const UDivM &mdH, const UDivM &mdH1)
{
  uint32_t w[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    uint32_t idx = base + (uint32_t)min(o + k, avail - 1);
    idx = (idx >= SR_RING * SR_MT_N) ? idx - SR_RING * SR_MT_N : idx;
    w[k] = sr_mt_temper(ring[idx]);
  }
  if (part == 3) {   /* the swap: i uniform_int(N - 1), j = i + 1 */
    const bool in = o + 4 <= avail;
    const uint32_t qi = udivm_v(w[0], mdN1.m, mdN1.l);
    const uint32_t qa = udivm_v(w[1], md2.m, md2.l), qb = udivm_v(w[2], md2.m, md2.l);
    const int ic = min((int)qi, N - 2);
    const bool veto = hcnt[ic + 2] - hcnt[ic] > 1;
    const bool ok = in && qi < mdN1.n && (veto || (qa < 2u && qb < 2u && w[3] != 0u));
    ptab[512 + o] = (uint32_t)ic | (veto ? 1u << 24 : 0u) | (ok ? 1u << 25 : 0u) | ((qa & 1u) << 26) | ((qb & 1u) << 27);
    return;
  }
  const bool in = o + 5 <= avail;
  const uint32_t qN = udivm_v(w[0], mdN.m, mdN.l), qN1 = udivm_v(w[1], mdN1.m, mdN1.l);
  const uint32_t qa = udivm_v(w[2], md2.m, md2.l), qb = udivm_v(w[3], md2.m, md2.l);
  const bool okN = in && qN < mdN.n && qN1 < mdN1.n;
  const bool okab = qa < 2u && qb < 2u;
  if (part <= 0) {
    const int i = (int)qN, j = (int)qN1 + ((int)qN1 >= (int)qN ? 1 : 0);
    const int ic = min(i, N - 1), jc = min(j, N - 1);
    const bool veto = (hcnt[ic + 1] != hcnt[ic]) && (hcnt[max(ic, jc) + 1] - hcnt[min(ic, jc)] > 1);
    const bool ok = okN && (veto || w[2] != 0u);
    ptab[o] = (uint32_t)ic | ((uint32_t)jc << 12) | (veto ? 1u << 24 : 0u) | (ok ? 1u << 25 : 0u);
  }
  if (part < 0 || part == 1) {
    int i = (int)qN, j = (int)qN1;
    if (j >= i) j++; else { const int t = i; i = j; j = t; }
    const int ic = min(i, N - 1), jc = min(j, N - 1);
    const bool veto = hcnt[jc + 1] - hcnt[ic] > 1;
    const bool ok = okN && (veto || (okab && w[4] != 0u));
    ptab[128 + o] = (uint32_t)ic | ((uint32_t)jc << 12) | (veto ? 1u << 24 : 0u) | (ok ? 1u << 25 : 0u) | ((qa & 1u) << 26) |
                    ((qb & 1u) << 27);
  }
  if (part < 0 || part == 2) {
    const uint32_t qH = udivm_v(w[0], mdH.m, mdH.l), qH1 = udivm_v(w[1], mdH1.m, mdH1.l);
    int ri, rj;
    if ((int)qH <= (int)qH1) { ri = (int)qH; rj = (int)qH1 + 1; } else { ri = (int)qH1; rj = (int)qH; }
    const int NH = N - nh;
    ri = min(ri, max(NH - 1, 0)); rj = min(rj, max(NH - 1, 0));
    const int i = nhall[ri], j = nhall[rj];
    const bool ok = in && NH >= 2 && qH < mdH.n && qH1 < mdH1.n && okab && w[4] != 0u;
    ptab[256 + o] = (uint32_t)i | ((uint32_t)j << 12) | (ok ? 1u << 25 : 0u) | ((qa & 1u) << 26) | ((qb & 1u) << 27);
    ptab[384 + o] = (uint32_t)ri | ((uint32_t)(rj - ri + 1) << 16);
  }
}

/* Count changes of one taxon (limits a, b; position-ordered column Pm) under proposal q:
 * dt0 (zeros inside), dt1 (ones inside); the reference's df0 = -dt0 and df1 = -dt1 always
 * (mcmc.c:1175-1256 pi1, 1367-1436 pi2, 1568-1631 pi3).  hcnt/nhall: the wave's hard-site tables. */
/* column bits at the hard positions, bit k = hard site k (input of the pi3 count change) */
/* hl: lane k holds hard position k (loaded by the caller with every lane active) */
/* HM: uint32_t (register-walk kernels, <= 32 hard sites) or uint64_t (LDS-walk kernels, <= SR_NHMAX = 64) */
template <typename HM = uint64_t>
__device__ __forceinline__ HM hard_bits_col(const uint32_t *Pm, int M, int hl, int nh)
{
  HM hbm = 0;
  if (nh > 0 && nh <= SR_NHMAX) {   /* (more hard sites: the bitmap path of taxon_dt) */
#pragma unroll
    for (int k = 0; k < 16; ++k) {   /* independent loads, one round trip */
      const int h = __builtin_amdgcn_readlane(hl, min(k, nh - 1));
      const HM bit = (Pm[(h >> 5) * M] >> (h & 31)) & 1u;
      hbm |= (k < nh ? bit : (HM)0) << k;
    }
    for (int k = 16; k < nh; ++k) {
      const int h = __builtin_amdgcn_readlane(hl, k);
      hbm |= (HM)((Pm[(h >> 5) * M] >> (h & 31)) & 1u) << k;
    }
  }
  return hbm;
}

/* hbx: the wave's hard bitmap when there are more than SR_NHMAX hard sites (the column's ones at hard
 * positions then come from the bitmap, word by word), else nullptr (the mask hbm) */
template <typename HM>
__device__ __forceinline__ void taxon_dt(int kind, const Prop &q, int a, int b, const uint32_t *Pm, const uint16_t *prem,
                                         int M, HM hbm, const int16_t *hcnt, const int16_t *nhall, int &dt0, int &dt1,
                                         const uint32_t *hbx, int N_, int PS = 0)
{
  const int i = q.i, j = q.j;
  dt0 = 0; dt1 = 0;
  if (kind == PK_PI1) {
    const int ii = q.ii, jj = q.jj;
    const int v = (Pm[(i >> 5) * M] >> (i & 31)) & 1;
    int sgn = 0;   /* +1: the moved site enters the taxon's range, -1: leaves it */
#if SR_PI1_FAST
    {   /* i < j: a, b tested against [ii + 1, jj + 1], sgn = ain - bin; i > j: against [ii, jj], sgn = bin - ain
           (block-uniform bounds: one unsigned compare per limit) */
      const int up = i < j ? 1 : 0, L = ii + up, span = jj - ii;
      const int ain = (uint32_t)(a - L) <= (uint32_t)span, bin = (uint32_t)(b - L) <= (uint32_t)span;
      sgn = up ? ain - bin : bin - ain;
    }
#else
    if (i < j) {
      const bool ain = (ii < a && a <= jj + 1), bin = (ii < b && b <= jj + 1);
      sgn = (ain && !bin) ? 1 : ((!ain && bin) ? -1 : 0);
    } else {
      const bool ain = (ii <= a && a <= jj), bin = (ii <= b && b <= jj);
      sgn = (!ain && bin) ? 1 : ((ain && !bin) ? -1 : 0);
    }
#endif
    if (v) dt1 = sgn; else dt0 = -sgn;
  } else if (kind != PK_PI3) {
    const int ain = ininterval(a, i, j + 1, q.inc1, q.inc2);
    const int bin = ininterval(b, i, j + 1, q.inc1, q.inc2);
#if SR_BF_TERMS
    {   /* branch-free: every lane reads the three prefixes, lanes with ain == bin keep zeros */
      const int sp = ain ? a : b;
      const int c0 = col_pre_bf(prem, Pm, M, i, PS), c1 = col_pre_bf(prem, Pm, M, sp, PS), c2 = col_pre_bf(prem, Pm, M, j + 1, PS);
      const int O1 = c1 - c0, O2 = c2 - c1;
      const int Z1 = (sp - i) - O1, Z2 = (j + 1 - sp) - O2;
      const bool on = ain != bin;
      dt1 = on ? (ain ? O1 - O2 : O2 - O1) : 0;
      dt0 = on ? (ain ? Z2 - Z1 : Z1 - Z2) : 0;
    }
#else
    if (ain != bin) {
      const int sp = ain ? a : b;
      const int c0 = col_pre(prem, Pm, M, i, PS), c1 = col_pre(prem, Pm, M, sp, PS), c2 = col_pre(prem, Pm, M, j + 1, PS);
      const int O1 = c1 - c0, O2 = c2 - c1;
      const int Z1 = (sp - i) - O1, Z2 = (j + 1 - sp) - O2;
      if (ain) { dt1 = O1 - O2; dt0 = Z2 - Z1; }
      else { dt1 = O2 - O1; dt0 = Z1 - Z2; }
    }
#endif
  } else {
    const int ain = ininterval(a, i, j + 1, q.inc1, q.inc2);
    const int bin = ininterval(b, i, j + 1, q.inc1, q.inc2);
    int na, nb;
    if (ain && !bin) { na = i + j + 1 - a; nb = b; }
    else if (!ain && bin) { na = a; nb = i + j + 1 - b; }
    else if (ain && bin) { na = i + j + 1 - b; nb = i + j + 1 - a; }
    else { na = a; nb = b; }
    /* Sets of pre-move positions inside [i, j]: W = alive before = [max(a,i), min(b-1,j)];
       I = alive after = the non-hard positions whose mirrored non-hard rank lands in [na, nb)
       (ranks [Kn-s_hi, Kn-s_lo) -> positions nhall[r0 + ...]) plus the hard positions of
       [na, nb) (fixed points).  dt1 = ones(I) - ones(W), dt0 = zeros(W) - zeros(I). */
    const int xa = min(max(na, i), j + 1), xb = min(max(nb, i), j + 1);
    const int ri = q.r0;                                   /* = i - hcnt[i] */
    const int s_lo = (xa - hcnt[xa]) - ri, s_hi = (xb - hcnt[xb]) - ri;
    auto hard_ones = [&](int lo, int hi, int &cnt) -> int {   /* hard positions in [lo, hi] */
#if SR_BF_TERMS
      if (!hbx) {   /* branch-free: indices clamped into the tables, an empty range counts nothing */
        const bool e = hi < lo;
        const int kl = hcnt[min(max(lo, 0), N_)], kh = hcnt[min(max(hi + 1, 0), N_)];
        cnt = e ? 0 : kh - kl;
        constexpr int HB = 8 * (int)sizeof(HM);
        const HM km = ((kh >= HB) ? ~(HM)0 : (((HM)1 << kh) - (HM)1)) & ~((kl >= HB) ? ~(HM)0 : (((HM)1 << kl) - (HM)1));
        return e ? 0 : (int)__popcll((uint64_t)(hbm & km));
      }
#endif
      if (hi < lo) { cnt = 0; return 0; }
      const int kl = hcnt[lo], kh = hcnt[hi + 1];
      cnt = kh - kl;
      if (hbx) {   /* many hard sites: ones of the column at the hard positions of [lo, hi], word by word */
        int o = 0;
        for (int w = lo >> 5; w <= (hi >> 5); ++w) o += __popc(Pm[w * M] & hbx[w] & range_mask(w, lo, hi));
        return o;
      }
      constexpr int HB = 8 * (int)sizeof(HM);
      const HM km = ((kh >= HB) ? ~(HM)0 : (((HM)1 << kh) - (HM)1)) & ~((kl >= HB) ? ~(HM)0 : (((HM)1 << kl) - (HM)1));
      return (int)__popcll((uint64_t)(hbm & km));
    };
    const int wlo = max(a, i), whi = min(b - 1, j);
    const int sizeW = max(0, whi - wlo + 1);
    int onesI = 0, sizeI = 0;
#if SR_BF_TERMS
    const int onesW = (whi >= wlo) ? col_pre_bf(prem, Pm, M, max(whi + 1, 0), PS) - col_pre_bf(prem, Pm, M, wlo, PS) : 0;
    {   /* branch-free: nhall indices and the positions read clamped into range, an empty rank range adds 0 */
      const bool on = s_lo < s_hi;
      const int pl = min(max((int)nhall[min(max(ri + q.Kn - s_hi, 0), N_ - 1)], 0), N_ - 1);
      const int ph = min(max((int)nhall[min(max(ri + q.Kn - s_lo - 1, 0), N_ - 1)], 0), N_ - 1);
      int hc;
      const int ho = hard_ones(pl, ph, hc);
      const int oI = col_pre_bf(prem, Pm, M, ph + 1, PS) - col_pre_bf(prem, Pm, M, pl, PS) - ho;
      onesI = on ? oI : 0;
      sizeI = on ? s_hi - s_lo : 0;
    }
#else
    const int onesW = (whi >= wlo) ? col_pre(prem, Pm, M, whi + 1, PS) - col_pre(prem, Pm, M, wlo, PS) : 0;
    if (s_lo < s_hi) {
      const int pl = nhall[ri + q.Kn - s_hi], ph = nhall[ri + q.Kn - s_lo - 1];
      int hc;
      const int ho = hard_ones(pl, ph, hc);
      onesI = col_pre(prem, Pm, M, ph + 1, PS) - col_pre(prem, Pm, M, pl, PS) - ho;
      sizeI = s_hi - s_lo;
    }
#endif
    {
      int hc;
      const int ho = hard_ones(max(na, i), min(nb - 1, j), hc);
      onesI += ho;
      sizeI += hc;
    }
    dt1 = onesI - onesW;
    dt0 = (sizeW - onesW) - (sizeI - onesI);
  }
}


/* The exact delta of one proposal: the reference's per-taxon terms (qval, mcmc.c:1214,
 * 1435, 1630 term order) compacted per 64-taxon chunk into cb, then summed sequentially in
 * ascending m by lane 0 of every wave.  Block-uniform call (contains a barrier). */
/* PR (pair kernels): taxon m = m0 + lane / 2 is evaluated by its even lane; a wave's 32 taxa form
 * one chunk (ballot bits of even lanes in ascending lane order = ascending m).  KT = chunks. */
/* GM: terms in HBM (exact_sum_gm).  SP (split chains): this half evaluates its own taxa [olo, ohi)
 * (whole chunks), the terms and counts go through the exchange (xsync: both halves' writes done),
 * and both halves compute the same sum. */
/* kv (manycd sessions, MCD kernels): per-taxon c, d ([2M]) and cc, dd ([2M]) replace K's shared ones in
 * each taxon's term (mcmc.c:1212-1214 reads c, d per taxon) */
template <bool PR, bool GM, bool SP, typename XSync>
__device__ __forceinline__ double sr_exact_delta(int kind, Prop q, CD K, const int32_t *sab, const uint32_t *P, const uint16_t *pre,
                                              int M, int N, int KT, int olo, int ohi,
                                              int hl, int nh, const int16_t *hcnt, const int16_t *nhall, const uint32_t *hbx,
                                              double *cb, int *cc, double *xs,
                                              int lane, int wave, int TB, XSync &&xsync, const double *kv = nullptr,
                                              const double *kx = nullptr, int PS = 0)
{
  constexpr int CH = PR ? 32 : 64;
  const bool ev = PR ? (lane & 1) == 0 : true;
  for (int m0 = olo + wave * CH; m0 < ohi; m0 += (PR ? TB / 2 : TB)) {   /* (chunk starts below M: KT chunks) */
    const int ch = m0 / CH, m = m0 + (PR ? (lane >> 1) : lane);
    int dt0 = 0, dt1 = 0;
    if (m < M && ev)
      taxon_dt(kind, q, sab[m], sab[M + m], P + m, pre + m, M, kind == PK_PI3 ? hard_bits_col<uint64_t>(P + m, M, hl, nh) : 0ull,
               hcnt, nhall, dt0, dt1, hbx, N, PS);
    CD Km = K;
    if (kv && m < M) { Km.c = kv[m]; Km.d = kv[M + m]; Km.cc = kx[m]; Km.dd = kx[M + m]; }
    const double tv = (m < M && ev) ? qval(dt0, -dt0, dt1, -dt1, Km) : 0.0;
    const uint64_t msk = __ballot(tv != 0.0);
    const int pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(msk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)msk, 0u));
    if (tv != 0.0) { if constexpr (SP) xst(cb + ch * CH + pos, tv); else cb[ch * CH + pos] = tv; }
    if (lane == 0) { if constexpr (SP) xst(cc + ch, (int)__popcll(msk)); else cc[ch] = __popcll(msk); }
  }
  if constexpr (SP) xsync(); else __syncthreads();
  if constexpr (GM) return exact_sum_gm<SP>(cb, cc, KT, lane, CH);
  else return exact_sum_wave(cb, cc, KT, xs, lane, CH);
}

/* words of slack kept resident after the Gibbs draws: the proposals and the next c, d
 * draws consume ~100 words; a refill inside them is still correct (block-uniform), only slower */
#define SR_RNG_SLACK 1024

/* ---------------------------------------------------------------- kernel */
/* One workgroup per chain, thread t owns taxa t, t+TB, ... for the whole launch (their
 * a, b, counts and position-ordered columns P live in LDS).  Every thread walks the same
 * MT19937 stream (ring in LDS) and computes every uniform decision itself -- the c, d
 * draws, the proposal draws, vetoes and MH decisions are identical in all threads, so
 * nothing is broadcast.  Phases of one sweep (mcmc.c:225-244):
 *   A  per-wave count totals -> barrier -> c, d (GSL beta via gamma/ziggurat)
 *   B  Gibbs (a_m, b_m) of own taxa (mcmc_sampleab); [barrier + logl on the last sweep]
 *   C  16 MH permutation proposals: draws, own taxa's count deltas and terms, per-wave
 *      partial sums -> one barrier -> certified decision -> apply to own taxa. */
/* MCD (manycd = 1, mcmc.c:777-786, 807-816): per-taxon c_m, d_m drawn one after another from Beta(1 + f1_m,
 * 1 + t0_m) / Beta(1 + f0_m, 1 + t1_m), every Gibbs draw, logl term and proposal delta with its taxon's own
 * coefficients -- the exact paths throughout (per-taxon step ratios leave nothing to share or certify by
 * integer sums).  One taxon or more per thread, one workgroup per chain, LDS or HBM columns. */
/* ---- phase C's certified Metropolis decision (mcmc.c:492 / 569 / 637: delta >= 0 || delta > log(uniform_pos)).
 * With X = sum dt, Y = sum |dt| (exact integers), S = X0 (cc - d) + X1 (dd - c) is the exact sum of the exact
 * per-taxon terms and B = Y0 (|cc|+|d|) + Y1 (|dd|+|c|) bounds their magnitudes; the reference's rounded terms
 * and sequential sum stay within (K + 7) 2^-53 B of S, K = #nonzero terms <= Knz = Y0 + Y1, so Eb = (Knz + 16)
 * 2^-52 B decides delta >= 0 and delta > log u whenever the true value is farther than Eb.  log u is first taken
 * in f32 (error << 2^-16 (1 + |log u|)), exactly only when that is too close.  The lane-parallel part: returns
 * cls 0 rejected, 1 accepted, 2 needs the exact delta or the exact log (pr: the pair kernels' packed Y). */
__device__ __forceinline__ int pc_classify(int X0, int X1, int Y0, int Y1, const CD &K, double aC, double aD, bool pr,
                                           uint32_t uw, double &Sp, double &Ebp, int &Knz)
{
  Sp = ((double)X0 * K.cc - (double)X0 * K.d) + ((double)X1 * K.dd - (double)X1 * K.c);
  /* PR: o[2] holds Y0 + Y1 (one packed field), o[3] = 0 -- bounded by the larger coefficient */
  const double B = pr ? (double)(Y0 + Y1) * fmax(aC, aD) : (double)Y0 * aC + (double)Y1 * aD;
  Knz = Y0 + Y1;   /* >= the number of nonzero terms: each has |dt0| + |dt1| >= 1 */
  Ebp = ((double)Knz + 16.0) * 0x1p-52 * B * SR_CERT_SCALE;
  if (Knz == 0 || Sp > Ebp) return 1;
  if (Sp < -Ebp) {
    const float uf = (float)((double)uw / 4294967296.0);
    const double lua = (double)__builtin_amdgcn_logf(uf) * 0.69314718055994531;
    const double dl = 0x1p-16 * (1.0 + __builtin_fabs(lua));
    return (Sp - Ebp > lua + dl) ? 1 : ((Sp + Ebp < lua - dl) ? 0 : 2);
  }
  return 2;
}

/* The serial part for a proposal classified 1 or 2 (S, Eb, kz = Knz of pc_classify): true when decided (accept;
 * udrawn: the uniform_pos was consumed), false when the exact sequential delta must decide.  dl: the delta the
 * accepted move adds to loglik when known exactly (have_exact). */
__device__ __forceinline__ bool pc_resolve(double S, double Eb, int c0, int kz, double u, const sr_mtab &tb, bool &accept,
                                           bool &udrawn, bool &have_exact, double &dl)
{
  accept = false; have_exact = false; dl = S;
  if (kz == 0) { accept = true; udrawn = false; have_exact = true; dl = 0.0; return true; }
  if (c0 == 1 && S > Eb) { accept = true; udrawn = false; return true; }
  if (c0 == 1) { accept = true; udrawn = true; return true; }
  if (S < -Eb) {   /* near a threshold: the exact log first */
    const double lu = sr_log_m(u, &tb);
    udrawn = true;
    if (S - Eb > lu) { accept = true; return true; }
    if (S + Eb < lu) return true;
  }
  return false;
}

template <int TB, int NWM, bool GM, bool PR = false, bool SP = false, bool MCD = false, bool LK = false>
__global__ __launch_bounds__(TB) void sr_sweep_kernel(KArgs A)
{
  static_assert(!SP || (GM && !PR && NWM == 0), "split chains: HBM-column kernels only");
  static_assert(!MCD || (!PR && !SP && NWM == 0), "manycd: generic one-workgroup kernels only");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NWV = TB / 64;
  /* wave: scalar in the HBM-column kernels (readfirstlane), so their per-wave LDS pointers live in SGPRs */
  const int tid = threadIdx.x, lane = tid & 63, wave = GM ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
  /* PR (pair kernels): lanes 2t, 2t+1 own taxon t (tx) together, hf = which half of the pair;
     otherwise one thread per taxon */
  const int tx = PR ? (tid >> 1) : tid;   /* (hf: per sweep, below) */
  constexpr int TXS = PR ? TB / 2 : TB;   /* taxon stride */
  /* SP: two workgroups per chain (sr_sp_half); both hold the whole block-uniform state (RNG ring,
     rpi, hard tables, c, d, loglik) and take every decision identically, each from sums exchanged
     with the other half; each owns half of the taxa (one per thread) */
  const int chain = SP ? (int)((blockIdx.x >> 4) << 3) + (int)(blockIdx.x & 7) : (int)blockIdx.x;
  const int half = SP ? (int)((blockIdx.x >> 3) & 1) : 0;
  if (SP && chain >= A.nchains) return;   /* grid padding (whole blocks) */
  const int N = SR_FN > 0 ? SR_FN : A.N, M = SR_FM > 0 ? SR_FM : A.M;
  const int NW = SR_FN > 0 ? (SR_FN + 31) / 32 : A.NW, nh = SR_FH >= 0 ? SR_FH : A.nh;
  const int olo = SP ? half * sr_sp_half(M) : 0, ohi = SP ? min(M, olo + sr_sp_half(M)) : M;   /* own taxa */
  const int mt = olo + tx;   /* own taxon, one-taxon-per-thread kernels */
  const int KTC = (M + sr_chunk(PR) - 1) / sr_chunk(PR);   /* exact-delta chunks */
  constexpr bool LCK = SP && LK && !SR_SP_LPRE;   /* Gibbs checkpoints in LDS (split kernels whose layout fits them, SR_SP_LCK) */
  constexpr bool LPRE = SP && LK && SR_SP_LPRE;   /* ... or the own half's column prefixes in LDS instead (SR_SP_LPRE) */
  const int PS = LPRE ? sr_sp_half(M) : M;          /* the prefix table's stride */
  constexpr bool SHT = GM && SR_GM_SHARED;   /* block-shared hard-site / 4-step tables */
  const Lay L = sr_layout(N, M, NW, TB, GM, PR, nh, SP && LK);
  double *tabs = (double *)(smem + L.tab);
  /* GM: the per-taxon arrays are the chain's HBM state itself (P, a/b, counts: updated in
     place) or its HBM scratch; otherwise LDS copies loaded here and stored at the end */
  double *cbuf = GM ? A.gcbuf + (size_t)chain * sr_gm_cbuf(M) : (double *)(smem + L.cbuf);
  double *lbuf = GM ? A.glbuf + (size_t)chain * M : (double *)(smem + L.lbuf);
  uint32_t *ring = (uint32_t *)(smem + L.mt);
  uint32_t *P = GM ? A.P + (size_t)chain * NW * M : (uint32_t *)(smem + L.P);
  int32_t *rpiA = (int32_t *)(smem + L.rpi0);
  int32_t *rpiB = (int32_t *)(smem + L.rpi1);
  uint16_t *pre = LPRE ? (uint16_t *)(smem + L.pre) - olo   /* (own taxa [olo, ohi) only) */
                 : GM ? A.gpre + (size_t)chain * sr_gm_pre(M, NW) : (uint16_t *)(smem + L.pre);   /* column prefix ones */
  int16_t *hcnt = (int16_t *)(smem + L.ht) + (SHT ? 0 : wave) * (2 * N + 2);    /* this wave's (SHT: the block's) hard-site tables */
  int16_t *nhall = hcnt + N + 1;
  const int CKS = LCK ? TB : SP ? 2 * TB : sr_ckstride(M, TB);   /* SP: slots [half TB + tid] (LCK: [tid] in LDS) */
  using CKT = typename std::conditional<GM && SR_CK32, float, double>::type;   /* Gibbs checkpoints: f32 in HBM scratch, f64 in LDS */
  CKT *ckb = (GM && !LCK) ? (CKT *)A.gck + (size_t)chain * (SP ? sr_sp_ck(N, TB) : sr_gm_ck(N, M, TB)) : (CKT *)(void *)(smem + L.ck);
  int *ccnt = (int *)(smem + L.ccnt);
  int32_t *sab = GM ? A.ab + (size_t)chain * 2 * M : (int32_t *)(smem + L.sab);     /* a[M], b[M] */
  int32_t *scnt = GM ? A.cnt + (size_t)chain * 4 * M : (int32_t *)(smem + L.scnt);  /* t0[M], f0[M], t1[M], f1[M] */
  const int NHC = SR_NHCAP(nh);   /* hard positions per chain in the state (64, or nh in whole waves) */
  int *hp = (int *)(smem + L.hpw) + wave * NHC;   /* this wave's copy of the hard positions */
  uint32_t *hbw = (uint32_t *)(smem + L.hbw) + wave * NW;   /* this wave's hard bitmap */
  const uint32_t *hbx = nh > SR_NHMAX ? hbw : nullptr;   /* many hard sites: hard ones from the bitmap */
  double *T4w = (double *)(smem + L.t4) + ((PR || SHT) ? 0 : wave) * T4STRIDE;   /* this wave's (PR, SHT: the block's) 4-step tables */
  constexpr bool SH8 = PR || GM;   /* one shared copy of the 8-step tables (built by waves 0-3, then a barrier) */
  double *T8w = (double *)(smem + L.t8) + (SH8 ? 0 : wave) * T8STRIDE;   /* this wave's (SH8: the block's) 8-step tables */
  int *part = (int *)(smem + L.part);
  int *tot = (int *)(smem + L.tot);
  double *xs = (double *)(smem + L.xs) + wave;
  uint64_t *misc = (uint64_t *)(smem + L.misc);
  uint32_t *ptab = (uint32_t *)(smem + L.ptab);   /* [5][128]: pi1, pi2, pi3 records, pi3 ranks, swaps per word offset */
  /* SP exchange: flags [2], slots (sr_sp_xb); xseq counts exchanges (block-uniform, the same
     sequence in both halves) */
  int *xfl = SP ? A.xflag + 2 * (size_t)chain : nullptr;
  int *xb = SP ? A.xbuf + (size_t)chain * sr_sp_xb(M) : nullptr;
  int xseq = 0;
  bool xbroken = false;   /* thread 0: the other half missed a deadline once; stop waiting */
  /* both halves' exchange writes done and visible: each thread's stores acknowledged, the block's
     flag raised, the other half's flag awaited (bounded: a half that never arrives -- not
     co-resident -- sets xerr and the launch completes with garbage the host refuses) */
  auto xsync = [&]() {
    if constexpr (SP) {
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      ++xseq;
      if (tid == 0) {
        xst(xfl + half, xseq);
        if (!xbroken) {
          int n = 0;
          while (xld(xfl + (half ^ 1)) < xseq) {
            __builtin_amdgcn_s_sleep(2);
            if (++n > (1 << 22)) { xbroken = true; xst(A.xerr, 1); break; }
          }
        }
      }
      __syncthreads();
    }
  };

  /* ---- load tables and state */
  for (int i = tid; i < 256; i += TB) {
    ((uint64_t *)tabs)[i] = c_exp_tab[i];
    tabs[256 + i] = c_log_tab[i];
  }
  sr_mtab tb;
  tb.exp_tab = (const uint64_t *)tabs; tb.log_tab = tabs + 256;
  {
    const uint32_t *gP = A.P + (size_t)chain * NW * M;
    if (!GM) for (int i = tid; i < NW * M; i += TB) P[i] = gP[i];
    const int32_t *grpi = A.rpi + (size_t)chain * N;
    for (int i = tid; i < N; i += TB) rpiA[i] = grpi[i];
    const uint32_t *gmt = A.mt + (size_t)chain * SR_RING * SR_MT_N;
    for (int i = tid; i < SR_RING * SR_MT_N; i += TB) ring[i] = gmt[i];
    const int32_t *gab = A.ab + (size_t)chain * 2 * M;
    if (!GM) for (int i = tid; i < 2 * M; i += TB) sab[i] = gab[i];
    const int32_t *gcnt = A.cnt + (size_t)chain * 4 * M;
    if (!GM) for (int i = tid; i < 4 * M; i += TB) scnt[i] = gcnt[i];
  }
  if (tid == 0) for (int q = MS_CAB; q < 64; ++q) misc[q] = 0;

  for (int k = lane; k < NHC; k += 64) hp[k] = (k < nh) ? A.hp[(size_t)chain * NHC + k] : -1;
  wsync();
  double c = A.cdl[(size_t)chain * 4 + 0];
  double d = A.cdl[(size_t)chain * 4 + 1];
  double *cv = MCD ? A.cdv + (size_t)chain * 2 * M : nullptr;   /* manycd: c[M], d[M] (HBM state, updated in place) */
  double *cx = MCD ? A.cdx + (size_t)chain * 2 * M : nullptr;   /* manycd: log(1 - e^c[m]), log(1 - e^d[m]) */
  double loglik = A.cdl[(size_t)chain * 4 + 2];   /* identical in every thread */
  DRng R;
  R.ring = ring;
  {
    const uint64_t pos = A.rng[(size_t)chain * 2 + 0];
    const uint64_t gen = A.rng[(size_t)chain * 2 + 1];
    R.blk = (uint32_t)(pos / SR_MT_N);
    R.off = (uint32_t)(pos % SR_MT_N);
    R.gen = (uint32_t)gen;
    R.ph = A.pkey != nullptr;
    R.pk0 = R.ph ? A.pkey[(size_t)chain * 2 + 0] : 0u;
    R.pk1 = R.ph ? A.pkey[(size_t)chain * 2 + 1] : 0u;
  }
  if (tid == 0) for (int k = 0; k < 7; ++k) misc[MS_ACC + k] = 0;
  int rcur = 0;     /* current rpi buffer */
  /* own taxon's column bits at the hard sites, bit k = hard site k in position order (one-taxon
     kernels).  Invariant for the whole run: every move that would change the hard sites' relative
     order is vetoed (mcmc.c:1153-1160, 1343-1348; pi3 moves non-hard sites only), so position hp[k]
     always holds the same site and its bits travel with it. */
  using HM = typename std::conditional<(NWM > 0), uint32_t, uint64_t>::type;   /* hard-site mask type */
  HM hbc = 0;
  int par = 0;      /* parity of the double-buffered totals */
  int bpar = 0;     /* parity of the double-buffered proposal count sums */
  int xpar = 0;     /* parity of the double-buffered exact-delta term lists */
  __syncthreads();

  build_hard_tables(hp, nh, N, NW, hbw, hcnt, nhall, lane, !SHT || wave == 0);   /* (SHT: read after the phase-A barrier) */
  for (int m = olo + tid; m < ohi; m += TB) col_pre_build(pre + m, P + m, M, NW, PS);   /* own columns */
  {
    const int hl0 = (lane < nh) ? hp[lane] : 0;   /* loaded with every lane active */
    if ((SP || M <= TXS) && mt < ohi) hbc = hard_bits_col<HM>(P + mt, M, hl0, nh);
  }
  const double ec = sr_exp_m(SR_LOGEPSILON, &tb);
  const uint32_t nhard = (uint32_t)nh;
  const UDivM mdN = make_udivm((uint32_t)N), mdN1 = make_udivm((uint32_t)(N - 1)), md2 = make_udivm(2u);
  const UDivM mdH = make_udivm((uint32_t)N - nhard > 0 ? (uint32_t)N - nhard : 1u);
  const UDivM mdH1 = make_udivm((uint32_t)N - nhard > 1 ? (uint32_t)N - nhard - 1 : 1u);
  STAMP_DECL

  for (int call = 0; call < A.calls; ++call) {
    for (int sw = 0; sw < A.spc; ++sw) {
      /* HBM-column kernels: the per-lane indices re-derived from an opaque copy of the thread index each sweep, so
         the addresses and lane masks built from them are computed where they are used instead of being hoisted out
         of the sweep loop and spilled (config 5's split kernel: 53 -> 24 VGPR spills, one spilled dword reloaded
         inside the loop; the LDS-column kernels run slower with it) */
      int tid_sw = tid;
      if constexpr (GM) __asm__ volatile("" : "+v"(tid_sw));
      {
      const int tid = tid_sw, lane = tid & 63;
      const int hf = PR ? (tid & 1) : 0, tx = PR ? (tid >> 1) : tid;
      const int mt = olo + tx;
      const int ckslot = (SP && !LCK) ? half * TB + tid : tid;   /* this thread's Gibbs checkpoint slots */
      (void)hf; (void)mt; (void)ckslot;
      const bool want_logl = (sw == A.spc - 1);
      /* this sweep's lane-parallel proposal tables, filled cooperatively (one entry per thread) before the
         phase-A barrier, at the stream position phase C most likely starts from: the c, d draws' fast path
         takes 8 words, the Gibbs step 2M (one round: the ring holds them all).  Phase C uses them when it
         starts there or a little later and no hard site has moved since; otherwise each wave refreshes its
         own copy as before (ptab_fill).  The previous sweep's readers are past the end-of-sweep barrier. */
      uint32_t tblk = 0u, toff = 0u;
      bool tvalid = false;
      if constexpr (!MCD && !GM && SR_COOP_TABLES) {   /* (GM: its registers spill 37 more VGPRs, r05l) */
        if (8 + 2 * M + SR_RNG_SLACK <= (SR_RING - 1) * SR_MT_N - (SR_MT_N - 1)) {
          rng_ensure(R, 8 + 2 * M + SR_RNG_SLACK, tid, TB);
          const uint32_t sp = R.off + 8u + 2u * (uint32_t)M;
          tblk = R.blk + sp / SR_MT_N;
          toff = sp % SR_MT_N;
          const uint32_t sbase = (tblk & (SR_RING - 1)) * SR_MT_N + toff;
          const int savail = min((int)((R.gen - tblk) * SR_MT_N - toff), 128);
          for (int k = tid; k < 4 * 128; k += TB)
            ptab_fill(ptab, ring, sbase, savail, k & 127, k >> 7, N, nh, hcnt, nhall, mdN, mdN1, md2, mdH, mdH1);
          if (SR_DOUBLE == 7) {   /* (the same entries again) */
            const int z = sr_opaque_zero();
            for (int k = tid; k < 4 * 128; k += TB)
              ptab_fill(ptab, ring, sbase, savail + z, (k & 127) + z, k >> 7, N, nh, hcnt, nhall, mdN, mdN1, md2, mdH, mdH1);
          }
          tvalid = true;
        }
      }
      /* the c, d draws' ziggurat steps, before the phase-A barrier (their table loads overlap the wait) */
      const CDPre cdpf = (SR_CD_PREFETCH && !MCD && !GM) ? cd_prefetch(R, lane) : CDPre{};
      FST(15);
      /* ============ phase A: totals and the c, d draws (mcmc.c:768-825) */
      {
        int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        for (int m = olo + tid; m < ohi; m += TB) { s0 += scnt[m]; s1 += scnt[M + m]; s2 += scnt[2 * M + m]; s3 += scnt[3 * M + m]; }
        s0 = wave_sum_i32(s0); s1 = wave_sum_i32(s1); s2 = wave_sum_i32(s2); s3 = wave_sum_i32(s3);
        int *tw = tot + (par * NWV + wave) * 4;
        if (lane == 0) { tw[0] = s0; tw[1] = s1; tw[2] = s2; tw[3] = s3; }
      }
      STAMP(0);
      FST(11);
      SR_SYNC();
      FST(11);
      {
        int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
        for (int w = 0; w < NWV; ++w) {
          const int *tw = tot + (par * NWV + w) * 4;
          s0 += tw[0]; s1 += tw[1]; s2 += tw[2]; s3 += tw[3];
        }
        if constexpr (SP) {   /* + the other half's totals */
          int *xt = xb + par * 8;
          if (tid == 0) { xst(xt + 4 * half, s0); xst(xt + 4 * half + 1, s1); xst(xt + 4 * half + 2, s2); xst(xt + 4 * half + 3, s3); }
          xsync();
          const int *yt = xt + 4 * (half ^ 1);
          s0 += xld(yt); s1 += xld(yt + 1); s2 += xld(yt + 2); s3 += xld(yt + 3);
        }
        /* mcmc_samplec then mcmc_sampled: Beta(1 + f1, 1 + t0), Beta(1 + f0, 1 + t1) */
        if constexpr (MCD) {
          /* manycd: c_m for m = 0..M-1, then d_m, each a GSL beta of the taxon's own counts (mcmc.c:777-786,
             807-816), in the reference's order from the one stream: every thread evaluates the same sequence
             (block-wide ring refills), thread 0 stores; then each thread its taxa's log(1 - e^x) */
          for (int k = 0; k < 2; ++k)
            for (int m = 0; m < M; ++m) {
              const double y = d_samplebeta<false>(R, cv[k * M + m], (double)(k ? scnt[M + m] : scnt[3 * M + m]),
                                                   (double)(k ? scnt[2 * M + m] : scnt[m]), k ? SR_MIND : SR_MINC,
                                                   k ? SR_MAXD : SR_MAXC, tid, TB, tb);
              SR_SYNC();   /* every thread has read cv[k M + m] */
              if (tid == 0) cv[k * M + m] = y;
            }
          SR_SYNC();
          for (int m = tid; m < 2 * M; m += TB) cx[m] = sr_log_m(1. - sr_exp_m(cv[m], &tb), &tb);
          SR_SYNC();
          c = cv[0];
          d = cv[M];
          if (tid == 0) { misc[MS_ACC + 0] += M - 1; misc[MS_ACC + 1] += M - 1; }   /* samplec returns M (mcmc.c:785) */
        } else if (SR_DOUBLE == 4 && [&] {   /* (diagnostic: the fast draw once more on a copy of the cursor) */
                     DRng R2 = R;
                     double c2 = c, d2 = d;
                     const int z = sr_opaque_zero();
                     const bool ok2 = draw_cd_fast(R2, c2, d2, s3 + z, s0, s1, s2, tb, lane);
                     c += (ok2 ? c2 : 1.0) * (double)z; d += d2 * (double)z;
                     return false; }()) {
        } else if (!draw_cd_fast(R, c, d, s3, s0, s1, s2, tb, lane, cdpf)) {
          if (tid == 0) misc[MS_CDSEQ]++;
          double cd2[2] = {c, d};
          for (int k = 0; k < 2; ++k)
            cd2[k] = d_samplebeta<false>(R, cd2[k], (double)(k ? s1 : s3), (double)(k ? s2 : s0), k ? SR_MIND : SR_MINC,
                                         k ? SR_MAXD : SR_MAXC, tid, TB, tb);
          c = cd2[0];
          d = cd2[1];
        }
        FST(12);
        if (tid == 0) { misc[MS_ACC + 0]++; misc[MS_ACC + 1]++; }
      }
      CD K;
      /* cc = log(1 - e^c) on even lanes, dd = log(1 - e^d) on odd lanes: one evaluation chain
         instead of two */
      const bool oddl = (lane & 1) != 0;
      const double l1 = sr_log_m(1. - sr_exp_m(oddl ? d : c, &tb), &tb);
      K.c = c; K.d = d; K.cc = readlane_f64(l1, 0); K.dd = readlane_f64(l1, 1); K.ec = ec;
      /* one position's value in q (log2 units): zero -> d - cc, one -> dd - c */
      const double vA = (K.d - K.cc) * 1.4426950408889634;
      const double vB = (K.dd - K.c) * 1.4426950408889634;
      const double r2 = sr_exp_m(oddl ? K.c - K.dd : K.cc - K.d, &tb);
      double rA = readlane_f64(r2, 0), rB = readlane_f64(r2, 1);   /* 2^-vA, 2^-vB */
      if (SR_DOUBLE == 5) {   /* (diagnostic: K's logs and exps and the step tables once more) */
        const double z = (double)sr_opaque_zero();
        const double l1b = sr_log_m(1. - sr_exp_m((oddl ? d : c) + z, &tb), &tb);
        const double r2b = sr_exp_m((oddl ? K.c - K.dd : K.cc - K.d) + z + l1b * z, &tb);
        rA += readlane_f64(r2b, 0) * z; rB += readlane_f64(r2b, 1) * z;
        if constexpr (NWM > 0 && !SH8) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int e = lane + 64 * q;
            double pr = 1.0, sm = 0.0;
#pragma unroll
            for (int k = 0; k < 8; ++k) { sm = sm + pr; pr = pr * (((e >> k) & 1) ? rB : rA); }
            *reinterpret_cast<double2 *>(T8w + 2 * e) = make_double2(sm, pr);
          }
        }
      }
      /* PR: one shared copy of the tables, built by waves 0-4 (T8 quarters, T4), then a barrier */
      if ((PR ? wave == 4 : (!SHT || wave == NWV - 1)) && lane < 16) {   /* per-wave (PR, SHT: shared) tables for 4 walk entries with bits = lane */
        double sc[5];
        const double pr = t4_row(lane, rA, rB, sc);
#pragma unroll
        for (int c = 0; c < 5; ++c) { T4w[2 * (c * 16 + lane)] = sc[c]; T4w[2 * (c * 16 + lane) + 1] = pr; }
      }
      if constexpr (NWM > 0 || GM) {   /* tables for 8 walk entries with bits = e: {sum of the 8 prefix products,
                                          product of all 8}; per wave 4 entries per lane, shared 1 per lane */
#pragma unroll
        for (int q = 0; q < (SH8 ? 1 : 4); ++q) {
          const int e = lane + 64 * (SH8 ? wave : q);
          const double2 te = t8_entry(e, rA, rB);
          if (!SH8 || wave < 4) *reinterpret_cast<double2 *>(T8w + 2 * e) = te;
        }
        if (lane == 0 && (!SH8 || wave == (PR ? 4 : 0))) *reinterpret_cast<double2 *>(T8w + 2 * 256) = make_double2(0.0, 1.0);
      }
      if constexpr (SH8) SR_SYNC(); else wsync();

#ifdef SR_STAMP_GIBBS
      STAMP(5);
#endif
      FST(0);
      /* ============ phase B: Gibbs update of own (a_m, b_m) (mcmc_sampleab) */
      /* taxa in rounds of TB (round r: m = r*TB + tid, words 2(m - r*TB), +1 from the round's
         cursor), each round's 2*TB words made resident first: the ring holds < 2M words when
         M > ~1870 (1024 x 2048) */
      {
        unsigned long long nchg = 0;
        const int rcap = (SR_RING - 1) * SR_MT_N - (SR_MT_N - 1);
        const int nround = (2 * M + SR_RNG_SLACK <= rcap) ? 1 : (M + TB - 1) / TB;
        for (int rd = 0; rd < nround; ++rd) {
        const int mlo = (nround == 1) ? 0 : rd * TB, mhi = (nround == 1) ? M : min(M, mlo + TB);
        if (rd > 0) SR_SYNC();   /* every thread is done with the previous round's words */
        FST(1);
        rng_ensure(R, min(2 * (mhi - mlo) + SR_RNG_SLACK, rcap), tid, TB);
        FST(8);
        for (int m = max(mlo, olo) + tx; m < min(mhi, ohi); m += TXS) {   /* PR: pair-uniform; SP: own taxa */
          const uint32_t *Pm = P + m;
          const double ua = rng_peek(R, 2 * (m - mlo)) / 4294967296.0;
          const double ub = rng_peek(R, 2 * (m - mlo) + 1) / 4294967296.0;
          const int a0 = sab[m], b0 = sab[M + m];
          int t0 = scnt[m], f0 = scnt[M + m], t1 = scnt[2 * M + m], f1 = scnt[3 * M + m];
          /* a_m over [0, b_m], then b_m over the reversed column with limit N - a_new: one
             inlined copy of the draw, two trips */
          int na = a0, nb = b0;
          if constexpr (PR) {   /* pair kernels: each lane of the pair walks half of the words */
            const uint16_t *prem = pre + m;
            const int POa = col_pre(prem, Pm, M, a0, PS);
            const int POb = (int)prem[NW * PS] - col_pre(prem, Pm, M, b0, PS);
            uint32_t wk[5];
            int d0, e0, d1, e1;
#pragma unroll
            for (int i = 0; i < 5; ++i) { const int k = 5 * hf + i; wk[i] = (k < NW) ? Pm[min(k, NW - 1) * M] : 0u; }
            na = draw_pair9(wk, hf, Pm, M, N, NW, false, a0, b0, POa, ua, K, tb, vA, vB, T4w, T8w, &misc[MS_FBK], d0, e0, d1, e1);
            t0 += d0; f0 += e0; t1 += d1; f1 += e1;
#pragma unroll
            for (int i = 0; i < 5; ++i) {
              const int k = 5 * hf + i;
              wk[i] = (k < NW) ? walk_word(Pm, M, N, NW, true, min(k, NW - 1)) : 0u;
            }
            nb = N - draw_pair9(wk, hf, Pm, M, N, NW, true, N - b0, N - na, POb, ub, K, tb, vA, vB, T4w, T8w, &misc[MS_FBK],
                                d0, e0, d1, e1);
            t0 += d0; f0 += e0; t1 += d1; f1 += e1;
          } else if constexpr (MCD) {   /* manycd: the taxon's own coefficients, the exact reference walk */
            const uint16_t *prem = pre + m;
            const int POa = col_pre(prem, Pm, M, a0, PS);
            const int POb = (int)prem[NW * PS] - col_pre(prem, Pm, M, b0, PS);
            CD Km = K;
            Km.c = cv[m]; Km.d = cv[M + m]; Km.cc = cx[m]; Km.dd = cx[M + m];
            for (int pass = 0; pass < 2; ++pass) {
              int d0, e0, d1, e1;
              const bool rev = pass != 0;
              const int o = rev ? N - b0 : a0, POo = rev ? POb : POa;
              const int res = draw_exact(Pm, M, N, rev, o, rev ? N - na : b0, rev ? ub : ua, Km, tb);
              pick_counts(res, o, POo, walk_prefix(Pm, M, N, NW, rev, res), d0, e0, d1, e1);
              t0 += d0; f0 += e0; t1 += d1; f1 += e1;
              if (rev) nb = N - res; else na = res;
            }
          } else if constexpr (NWM > 0) {   /* column in registers, branch-free draws */
            uint32_t wk[NWM];   /* forward walk words, then (second trip) the reversed ones */
            load_fwd<NWM>(Pm, M, NW, wk);
            /* ones before each trip's start entry from the column prefix table: forward, positions
               [0, a0); reversed, walk entries [0, N - b0) = positions [b0, N) */
            const uint16_t *prem = pre + m;
            const int POa = col_pre(prem, Pm, M, a0, PS);
            const int POb = (int)prem[NW * PS] - col_pre(prem, Pm, M, b0, PS);
            for (int pass = 0; pass < 2; ++pass) {
              int d0, e0, d1, e1;
              const bool rev = pass != 0;
              if (rev) {
                uint32_t rw[NWM];
                make_rev<NWM>(Pm, M, N, NW, wk, rw);
#pragma unroll
                for (int k = 0; k < NWM; ++k) wk[k] = rw[k];
              }
              int res = draw_fast_s<NWM>(wk, Pm, M, N, rev, rev ? N - b0 : a0, rev ? N - na : b0, rev ? POb : POa,
                                         rev ? ub : ua, K, tb, vA, vB, T4w, T8w, &misc[MS_FBK], d0, e0, d1, e1);
              if (SR_DOUBLE == 3) {
                const int z = sr_opaque_zero();
                int q0, q1, q2, q3;
                const int r2 = draw_fast_s<NWM>(wk, Pm, M, N, rev, (rev ? N - b0 : a0) + z, rev ? N - na : b0, rev ? POb : POa,
                                                (rev ? ub : ua) + (double)z, K, tb, vA, vB, T4w, T8w, &misc[MS_FBK], q0, q1, q2, q3);
                res |= r2 & z; d0 |= q0 & z; e0 |= q1 & z; d1 |= q2 & z; e1 |= q3 & z;
              }
              t0 += d0; f0 += e0; t1 += d1; f1 += e1;
              if (rev) nb = N - res; else na = res;
            }
          } else {
          const uint16_t *prem = pre + m;   /* ones before each trip's start entry, as above */
          const int POa = col_pre(prem, Pm, M, a0, PS);
          const int POb = (int)prem[NW * PS] - col_pre(prem, Pm, M, b0, PS);
          for (int pass = 0; pass < 2; ++pass) {
            int d0, e0, d1, e1;
            const bool rev = pass != 0;
            const int res = draw_fast<GM>(Pm, prem, M, N, NW, rev, rev ? N - b0 : a0, rev ? N - na : b0, rev ? POb : POa,
                                      rev ? ub : ua, K, tb, vA, vB, rA, rB, T4w, T8w, ckb + ckslot, CKS, PS, &misc[MS_FBK], d0, e0,
                                      d1, e1 GSTAMP_PASS);
            GSTAMP_K4();
            t0 += d0; f0 += e0; t1 += d1; f1 += e1;
            if (rev) nb = N - res; else na = res;
          }
          }
          if (!PR || hf == 0) {   /* PR: the even lane writes the pair's results */
            nchg += (na != a0) + (nb != b0);
            sab[m] = na; sab[M + m] = nb;
            scnt[m] = t0; scnt[M + m] = f0; scnt[2 * M + m] = t1; scnt[3 * M + m] = f1;
            if (want_logl) {   /* mcmc_logl term (mcmc.c:643-644); manycd: the taxon's c, d (mcmc.c:641-642) */
              const double kcc = MCD ? cx[m] : K.cc, kd = MCD ? cv[M + m] : K.d, kdd = MCD ? cx[M + m] : K.dd,
                           kc = MCD ? cv[m] : K.c;
              const double lt = (double)t0 * kcc + (double)f0 * kd + (double)t1 * kdd + (double)f1 * kc;
              if constexpr (SP) xst(lbuf + m, lt); else lbuf[m] = lt;
            }
          }
        }
        rng_skip(R, 2 * (mhi - mlo));
        }
        const int nw = wave_sum_i32((int)nchg);
        if (lane == 0 && nw) atomicAdd((unsigned long long *)&misc[MS_CAB], (unsigned long long)nw);
      }
      FST(1);
      STAMP(1);
      if (GM && want_logl) {   /* mcmc_logl with the terms in HBM: each wave reads them 64 at a time
                                  (coalesced, 4 chunks in flight) and adds them in m order through readlane */
        if constexpr (SP) xsync(); else SR_SYNC();
        double s = 0.0;
        for (int c0 = 0; c0 < M; c0 += 256) {
          double v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int m = c0 + 64 * q + lane;
            v[q] = (m < M) ? (SP ? xld(lbuf + m) : lbuf[m]) : 0.0;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int n = min(64, M - (c0 + 64 * q));
#pragma unroll 16
            for (int l = 0; l < 64; ++l)
              if (l < n) s = s + readlane_f64(v[q], l);
          }
        }
        loglik = s;
      } else if (want_logl) {   /* mcmc_logl (mcmc.c:639-645), sequential over m, lane 0 of every wave */
        SR_SYNC();
        if (PR ? tid == 0 : lane == 0) {
          double s = 0.0;
          int m = 0;
          for (; m + 4 <= M; m += 4) {
            const double a0 = lbuf[m], a1 = lbuf[m + 1], a2 = lbuf[m + 2], a3 = lbuf[m + 3];
            s = s + a0; s = s + a1; s = s + a2; s = s + a3;
          }
          for (; m < M; ++m) s = s + lbuf[m];
          if (PR) *reinterpret_cast<double *>(&misc[MS_LOGL]) = s; else *xs = s;
        }
        if constexpr (PR) {   /* one sum (thread 0), read by all behind a barrier */
          SR_SYNC();
          loglik = *reinterpret_cast<const double *>(&misc[MS_LOGL]);
        } else {
          wsync();
          loglik = *xs;
          wsync();
        }
      }
      STAMP(2);
      FST(0);

      /* ============ phase C: the permutation proposals (mcmc.c:237-243), speculatively batched.
         Hypothesis: every remaining proposal is rejected.  A rejected non-vetoed proposal has
         delta < 0, so it drew exactly one uniform_pos after its index draws; this fixes every
         proposal's RNG words in advance.  All remaining proposals are drawn, their count sums
         computed against the current state (one barrier), and decided lane-parallel; the first
         one that is accepted (or needs the exact delta) ends the batch: it is applied with the
         cursor it really consumed, and the proposals after it are re-batched. */
      {
        /* lane p: proposal p -- vpk = i | j << 12 | inc1 << 24 | inc2 << 25 | veto << 26 (one readlane per
           proposal where its fields are read), vkr = Kn | r0 << 16 (pi3) */
        int vpk = 1 << 26, vkr = 0, vuw = 1, vnd = 0, voff = 0;
        int p0 = 0;
        if constexpr (SP) {   /* the Gibbs step's rounds of TB taxa gave some of this half's taxa to other threads
                                 (a half not starting at a multiple of TB): their limits and counts, read by the
                                 owner threads below, are ordered by a barrier */
          const bool multi = 2 * M + SR_RNG_SLACK > (SR_RING - 1) * SR_MT_N - (SR_MT_N - 1);
          if (multi && (olo % TB) != 0 && (olo / TB + 1) * TB < ohi) SR_SYNC();
        }
        /* the lane-parallel proposal tables (ptab) hold "a proposal of each kind starting at word o"
           for the 128 words from stream position (tblk, toff) (the sweep's cooperative fill, or a wave's
           refresh); a later batch of the sweep reuses them while its proposals stay inside those words and
           no hard site moved (block-uniform state) */
        while (p0 < 16) {
          p0 = __builtin_amdgcn_readfirstlane(p0);   /* block-uniform: keep the control flow scalar */
          const int hl = (lane < nh) ? hp[lane] : 0;  /* lane k: hard position k */
          /* ---- draws of proposals p0.. under the hypothesis: block-uniform scalar code; the
             record of proposal p lives in lane p of the v* registers */
          const uint32_t rblk = __builtin_amdgcn_readfirstlane(R.blk), roff = __builtin_amdgcn_readfirstlane(R.off);
          const uint32_t rgen = __builtin_amdgcn_readfirstlane(R.gen);
          const int avail = min((int)((rgen - rblk) * SR_MT_N - roff), 128);   /* resident words, <= 2 per lane */
          const uint32_t base = (rblk & (SR_RING - 1)) * SR_MT_N + roff;
          /* the batch's next 128 tempered words for the scalar path (word k in lane k & 63 of
             vw[k >> 6]), loaded only when a proposal takes that path: the swap batch, or a fast-path
             stop (block-uniform flag) */
          uint32_t vw0 = 0u, vw1 = 0u;
          bool vw_ok = false;
          auto need_vw = [&]() {
            if (vw_ok) return;
            uint32_t i0 = base + (uint32_t)lane, i1 = base + 64u + (uint32_t)lane;
            i0 = (i0 >= SR_RING * SR_MT_N) ? i0 - SR_RING * SR_MT_N : i0;
            i1 = (i1 >= SR_RING * SR_MT_N) ? i1 - SR_RING * SR_MT_N : i1;
            i1 = (i1 >= SR_RING * SR_MT_N) ? i1 - SR_RING * SR_MT_N : i1;
            vw0 = sr_mt_temper(ring[i0]);
            vw1 = sr_mt_temper(ring[i1]);
            vw_ok = true;
          };
          FST(14);
          STAMP_D(3);
          int off = 0, pend = p0;
          /* one proposal drawn by block-uniform scalar code at word offset `off` (false: not enough
             resident words) */
          auto scalar_one = [&](int p) -> bool {
#if defined(SR_STAMPS) && !defined(SR_STAMP_FINE)
              if (tid == 0) misc[43] += 1;   /* proposals drawn by the scalar path */
#endif
              need_vw();
              const int kind = prop_kind(p);
              bool bad = false;
              auto word = [&](void) -> uint32_t {
                if (off >= avail) { bad = true; return 0u; }
                const int k = off++;
                return (uint32_t)__builtin_amdgcn_readlane((int)(k < 64 ? vw0 : vw1), k & 63);
              };
              auto uint_draw = [&](const UDivM &u) -> int {   /* gsl_rng_uniform_int */
                uint32_t k;
                do { k = udivm(word(), u); } while (!bad && k >= u.n);
                return (int)k;
              };
              auto hc = [&](int x) -> int { return __builtin_amdgcn_readfirstlane((int)hcnt[x]); };
              int i = 0, j = 0, inc1 = 0, inc2 = 0, Kn = 0, r0 = 0;
              bool veto = false;
              if (kind == PK_PI1) {                                  /* mcmc.c:1133-1160 */
                i = uint_draw(mdN);
                j = uint_draw(mdN1);
                if (j >= i) j++;
                if (!bad && hc(i + 1) != hc(i) && hc(max(i, j) + 1) - hc(min(i, j)) > 1) veto = true;
              } else if (kind == PK_PI2 || kind == PK_SWAP) {        /* mcmc.c:1317-1364 */
                if (kind == PK_PI2) {
                  i = uint_draw(mdN);
                  j = uint_draw(mdN1);
                  if (j >= i) j++;
                  else { const int t = i; i = j; j = t; }
                } else {
                  i = uint_draw(mdN1);
                  j = i + 1;
                }
                if (!bad && hc(j + 1) - hc(i) > 1) veto = true;
                if (!veto) { inc1 = uint_draw(md2); inc2 = uint_draw(md2); }
              } else {                                               /* mcmc.c:1495-1565 */
                if ((uint32_t)N - nhard < 2) veto = true;
                else {
                  const int n0 = uint_draw(mdH), m0 = uint_draw(mdH1);
                  inc1 = uint_draw(md2);
                  inc2 = uint_draw(md2);
                  /* non-hard ranks -> positions (mcmc.c:1505-1533) */
                  int ri, rj;
                  if (n0 <= m0) { ri = n0; rj = m0 + 1; } else { ri = m0; rj = n0; }
                  if (!bad) {
                    i = __builtin_amdgcn_readfirstlane((int)nhall[ri]);
                    j = __builtin_amdgcn_readfirstlane((int)nhall[rj]);
                  }
                  Kn = rj - ri + 1;
                  r0 = ri;
                }
              }
              const int nd = off;
              uint32_t uw = 0;
              if (!veto) { do { uw = word(); } while (!bad && uw == 0u); }   /* gsl_rng_uniform_pos */
              if (bad) return false;
              vpk = (lane == p) ? (i | (j << 12) | (inc1 << 24) | (inc2 << 25) | (veto ? 1 << 26 : 0)) : vpk;
              vkr = (lane == p) ? (Kn | (r0 << 16)) : vkr;
              vuw = (lane == p) ? ((int)uw) : vuw;
              vnd = (lane == p) ? (nd) : vnd;
              voff = (lane == p) ? (off) : voff;
              pend = p + 1;
              return true;
          };
          /* the swap (accepted ~44 %) is drawn first and forms its own batch: from the sweep's table when
             phase C starts inside it and the entry is on the fast path, else by the scalar path */
          if (p0 == 0) {
            const int dlt = tvalid ? (int)((rblk - tblk) * SR_MT_N + roff) - (int)toff : -1;
            const uint32_t e = (SR_COOP_TABLES && dlt >= 0 && dlt < 128) ? ptab[512 + dlt] : 0u;
            if ((e >> 25) & 1u) {
              const bool veto = (e >> 24) & 1u;
              const int i = (int)(e & 4095u);
              uint32_t iu = base + 3u;   /* the uniform_pos word (not drawn after a veto) */
              iu = (iu >= SR_RING * SR_MT_N) ? iu - SR_RING * SR_MT_N : iu;
              const uint32_t uw = veto ? 1u : sr_mt_temper(ring[iu]);
              vpk = (lane == 0) ? (i | ((i + 1) << 12) | (int)(((e >> 26) & 3u) << 24) | (veto ? 1 << 26 : 0)) : vpk;
              vkr = (lane == 0) ? 0 : vkr;
              vuw = (lane == 0) ? (int)uw : vuw;
              vnd = (lane == 0) ? (veto ? 1 : 3) : vnd;
              voff = (lane == 0) ? (veto ? 1 : 4) : voff;
              pend = 1;
              off = veto ? 1 : 4;
            } else {
              (void)scalar_one(0);
            }
          }
          /* (the swap in one batch with proposals 1..15 measured no faster at round 3: profiles/r03e_ab_phasec.json;
             SR_MERGE_SWAP re-tests it) */
          if (p0 > 0 || (SR_MERGE_SWAP && (!GM || SR_MERGE_SWAP_GM) && pend == 1)) {
            /* Lane-parallel draws: lane l evaluates "a pi1 / pi2 / pi3 proposal starting at word
               offset o" for o = l and o = l + 64 (words o..o+4) into ptab; the scan below then walks
               the batch's actual offsets reading those results.  ok = no GSL rejection and a nonzero
               uniform_pos word (else the scalar path below takes over at that proposal).  The tables
               are shared by the waves: every wave writes the same values (block-uniform inputs), and
               no wave reads them past the batch barrier that every wave's next write follows. */
            int delta = tvalid ? (int)((rblk - tblk) * SR_MT_N + roff) - (int)toff : 0;
            if (!tvalid || delta < 0 || delta + 5 * (16 - p0) + 5 > 128) {
              delta = 0;
              tblk = rblk; toff = roff; tvalid = true;
#if defined(SR_STAMPS) && !defined(SR_STAMP_FINE)
              if (tid == 0) misc[42] += 1;   /* table refills in phase C */
#endif
#pragma unroll
              for (int h = 0; h < 2; ++h)
                ptab_fill(ptab, ring, base, avail, lane + 64 * h, -1, N, nh, hcnt, nhall, mdN, mdN1, md2, mdH, mdH1);
              wsync();
            }
            FST(15);
            /* scan, two steps.  (1) the offset chain: proposal p starts where p-1 ended; a 5-bit
               entry per offset (lane l: offset l in bits 0-15, l + 64 in bits 16-31) holds, per kind,
               whether the fast path applies there and how many words it consumes (pi1 2 / 3,
               pi2 2 / 5, pi3 5), so each step is one readlane and a few scalar ops.  (2) lane p
               gathers its own proposal's record from the tables at its start offset. */
            uint32_t lent = 0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int t = delta + lane + 64 * h;   /* table index of batch offset lane + 64 h */
              const int tc = min(t, 127);
              const uint32_t a1 = ptab[tc], a2 = ptab[128 + tc], a3 = ptab[256 + tc];
              const uint32_t e = ((a1 >> 25) & 1u) | ((((a1 >> 24) & 1u) ^ 1u) << 1) | (((a2 >> 25) & 1u) << 2) |
                                 (((a2 >> 24) & 1u) << 3) | (((a3 >> 25) & 1u) << 4);
              lent |= (t < 128 ? e : 0u) << (16 * h);   /* past the tables: not ok (scalar path) */
            }
            const int sstart = pend;
            int vstart = 0;
#pragma unroll
            for (int sI = 1; sI < 16; ++sI) {
              if (sI < p0 || pend != sI || off + 5 > 128 || sI >= p0 + SR_BATCH_MAX) continue;
              const int kind = prop_kind(sI);
              const uint32_t e = (uint32_t)__builtin_amdgcn_readlane((int)lent, off & 63) >> (16 * (off >> 6));
              bool ok;
              int adv;
              if (kind == PK_PI1) { ok = e & 1u; adv = (e & 2u) ? 3 : 2; }
              else if (kind == PK_PI2) { ok = (e >> 2) & 1u; adv = (e & 8u) ? 2 : 5; }
              else { ok = (e >> 4) & 1u; adv = 5; }
              if (!ok) continue;   /* rejection or zero word: scalar path */
              vstart = (lane == sI) ? off : vstart;
              off += adv;
              pend = sI + 1;
            }
            {
              const int o = vstart;
              const int kind = prop_kind(lane & 15);
              const int tc = min(delta + o, 127);
              const uint32_t ra = ptab[(kind == PK_PI1 ? 0 : (kind == PK_PI2 ? 128 : 256)) + tc];
              const uint32_t rb = (kind == PK_PI3) ? ptab[384 + tc] : 0u;
              uint32_t iu = base + (uint32_t)min(o + (kind == PK_PI1 ? 2 : 4), avail - 1);   /* the uniform_pos word */
              iu = (iu >= SR_RING * SR_MT_N) ? iu - SR_RING * SR_MT_N : iu;
              const uint32_t ru = sr_mt_temper(ring[iu]);
              const bool veto = (ra >> 24) & 1u;
              const int nd = o + (kind == PK_PI1 ? 2 : (kind == PK_PI2 ? (veto ? 2 : 4) : 4));
              if (lane >= sstart && lane < pend) {
                vpk = (int)((ra & 0xffffffu) | (((ra >> 26) & 3u) << 24) | (veto ? 1u << 26 : 0u));
                vkr = (int)((rb >> 16) | ((rb & 0xffffu) << 16));
                vuw = (int)ru;
                vnd = nd;
                voff = nd + (veto ? 0 : 1);
              }
            }
          }
          for (int p = pend; p < 16; ++p) {   /* scalar path: the batch's first proposal after a fast-path stop */
            if (p0 == 0 && p == 1) break;     /* the swap batch (merged: the lane-parallel scan's proposals follow) */
            if (p > p0) break;                /* only the batch's first proposal goes scalar */
            if (!scalar_one(p)) break;
          }
          pend = __builtin_amdgcn_readfirstlane(pend);
#if defined(SR_STAMPS) && !defined(SR_STAMP_FINE)   /* batch statistics (slots 40-41 are the fine build's) */
          if (tid == 0 && pend > p0) { misc[40] += 1; misc[41] += (unsigned long long)(pend - p0); }
#endif
          FST(2);
          STAMP_D(4);
          if (pend == p0) {   /* not enough resident words for one proposal: make more, retry */
            rng_ensure(R, min(avail + 256, (SR_RING - 1) * SR_MT_N - (SR_MT_N - 1)), tid, TB);
            tvalid = false;
            continue;
          }
          auto load_prop = [&](int p) -> Prop {   /* fields unpacked by scalar ALU */
            Prop q;
            const uint32_t pk = (uint32_t)__builtin_amdgcn_readlane(vpk, p);
            q.i = (int)(pk & 4095u);
            q.j = (int)((pk >> 12) & 4095u);
            q.ii = min(q.i, q.j); q.jj = max(q.i, q.j);
            q.inc1 = (int)((pk >> 24) & 1u); q.inc2 = (int)((pk >> 25) & 1u);
            const uint32_t kr = (uint32_t)__builtin_amdgcn_readlane(vkr, p);
            q.Kn = (int)(kr & 0xffffu);
            q.r0 = (int)(kr >> 16);
            return q;
          };
          auto vetoed = [&](int p) -> bool { return ((uint32_t)__builtin_amdgcn_readlane(vpk, p) >> 26) & 1u; };

          /* ---- exact integer count sums of every drawn proposal over own taxa, per wave */
          int *pw = part + (bpar * 16) * NWV * 8;
          const bool pack = N < 512;   /* one taxon per thread: per-wave sums fit 16-bit fields */
          /* own taxon's limits and hard-site bits, fixed for the batch (one taxon per thread) */
          /* register-walk kernels: M <= TB (sr_regwalk); 1024-thread split halves hold <= TB taxa (compile-time) */
          const bool one = NWM > 0 || (SP && TB == 1024) || (SP && ohi - olo <= TB) || M <= TXS;
          int a1 = 0, b1 = 0;
          const HM hb1 = hbc;
          /* every thread owns a taxon when the shape is compiled in and fills the block (the bench kernel): the
             ownership test is then a constant, not an exec mask re-set around every slot */
          constexpr bool ALLOWN = SR_OWN_CONST && !SP && !PR && SR_FM > 0 && SR_FM >= TB;
          const bool own = ALLOWN || mt < ohi;
          if (one && own) { a1 = sab[mt]; b1 = sab[M + mt]; }
          FST(13);
#if defined(SR_STAMP_DRAWS)
          STAMP(5);
#elif defined(SR_STAMP_GIBBS)
          STAMP(6);
#else
          STAMP(3);
#endif
          if constexpr (PR) {
            /* pair kernels: the proposals in slot pairs of one code path (kinds pi1, pi2 / swap,
               pi3); the even lane of a taxon evaluates the pair's first proposal, the odd lane the
               second, and the per-wave sums are kept per lane parity (the two proposals' sums) */
            constexpr int SPA[9] = {1, 2, 3, 7, 8, 9, 13, 14, 15};
            constexpr int SPB[9] = {4, 5, 6, 10, 11, 12, -1, 0, -1};
            constexpr uint64_t EV = 0x5555555555555555ull, OD = 0xAAAAAAAAAAAAAAAAull;
#pragma unroll
            for (int sp = 0; sp < 9; ++sp) {   /* terms and their sums per slot pair (no per-slot arrays:
                                                  the register budget is 128 at four waves per SIMD) */
              const int pa = SPA[sp], pb = SPB[sp];
              const bool va = pa >= p0 && pa < pend && !vetoed(pa);
              const bool vb = pb >= 0 && pb >= p0 && pb < pend && !vetoed(pb >= 0 ? pb : 0);
              if (va || vb) {
                const Prop qa = load_prop(pa), qb = load_prop(pb >= 0 ? pb : pa);
                Prop q;
                q.i = hf ? qb.i : qa.i; q.j = hf ? qb.j : qa.j; q.ii = hf ? qb.ii : qa.ii; q.jj = hf ? qb.jj : qa.jj;
                q.inc1 = hf ? qb.inc1 : qa.inc1; q.inc2 = hf ? qb.inc2 : qa.inc2;
                q.Kn = hf ? qb.Kn : qa.Kn; q.r0 = hf ? qb.r0 : qa.r0;
                int d0 = 0, d1 = 0;
                if ((hf ? vb : va) && tx < M)
                  taxon_dt(prop_kind(pa), q, a1, b1, P + tx, pre + tx, M, hb1, hcnt, nhall, d0, d1, hbx, N, PS);
                int Xa0, Xa1, Ya, Xb0, Xb1, Yb;
                if (prop_kind(pa) == PK_PI1) {   /* dt in {-1, 0, 1}, dt0 dt1 = 0: ballot counts per parity */
                  const uint64_t p0m = __ballot(d0 > 0), n0m = __ballot(d0 < 0);
                  const uint64_t p1m = __ballot(d1 > 0), n1m = __ballot(d1 < 0);
                  Xa0 = (int)__popcll(p0m & EV) - (int)__popcll(n0m & EV); Xb0 = (int)__popcll(p0m & OD) - (int)__popcll(n0m & OD);
                  Xa1 = (int)__popcll(p1m & EV) - (int)__popcll(n1m & EV); Xb1 = (int)__popcll(p1m & OD) - (int)__popcll(n1m & OD);
                  Ya = (int)(__popcll((p0m | n0m) & EV) + __popcll((p1m | n1m) & EV));
                  Yb = (int)(__popcll((p0m | n0m) & OD) + __popcll((p1m | n1m) & OD));
                } else {   /* 16-bit field per parity: 32 lanes x (dt + N) < 2^16 for N < 1024 */
                  const int sh = 16 * hf;
                  const uint32_t u0 = (uint32_t)wave_sum_i32((int)((uint32_t)(d0 + N) << sh));
                  const uint32_t u1 = (uint32_t)wave_sum_i32((int)((uint32_t)(d1 + N) << sh));
                  const uint32_t u2 = (uint32_t)wave_sum_i32((int)((uint32_t)(abs(d0) + abs(d1)) << sh));
                  Xa0 = (int)(u0 & 0xffffu) - 32 * N; Xb0 = (int)(u0 >> 16) - 32 * N;
                  Xa1 = (int)(u1 & 0xffffu) - 32 * N; Xb1 = (int)(u1 >> 16) - 32 * N;
                  Ya = (int)(u2 & 0xffffu); Yb = (int)(u2 >> 16);
                }
                if (lane == 0 && va) { int *o = pw + (pa * NWV + wave) * 8; o[0] = Xa0; o[1] = Xa1; o[2] = Ya; o[3] = 0; }
                if (lane == 1 && vb) { int *o = pw + (pb * NWV + wave) * 8; o[0] = Xb0; o[1] = Xb1; o[2] = Yb; o[3] = 0; }
              }
            }
            FST(3);
            STAMP_K(PK_PI3);
          } else if (one) {
            /* one taxon per thread: all 16 proposal slots unrolled; slot s has the compile-time
               kind prop_kind(s), so each copy holds one kind's code and the slots' loads, ALU
               and reductions are independent */
            int d0s[16], d1s[16];
            /* the sweep's main batch (proposals 1..15 all drawn): every slot unconditionally, vetoed slots and
               lanes without a taxon masked afterwards, so no branch separates the slots' reads (a lane without a
               taxon reads the half's last column: in range in LDS and in HBM) */
            const bool full = SR_FULL_BATCH && p0 == 1 && pend == 16;
            if (full) {
              d0s[0] = 0; d1s[0] = 0;
              const int mtc = min(mt, ohi - 1);
#pragma unroll
              for (int sI = 1; sI < 16; ++sI) {
                const Prop q = load_prop(sI);
                int dt0 = 0, dt1 = 0;
                taxon_dt(prop_kind(sI), q, a1, b1, P + mtc, pre + mtc, M, hb1, hcnt, nhall, dt0, dt1, hbx, N, PS);
                const bool use = mt < ohi && !vetoed(sI);
                d0s[sI] = use ? dt0 : 0; d1s[sI] = use ? dt1 : 0;
              }
            } else {
#pragma unroll
            for (int sI = 0; sI < 16; ++sI) {
              d0s[sI] = 0; d1s[sI] = 0;
              if (sI >= p0 && sI < pend && !vetoed(sI)) {
                const Prop q = load_prop(sI);
                int dt0 = 0, dt1 = 0;
                if (own) taxon_dt(prop_kind(sI), q, a1, b1, P + mt, pre + mt, M, hb1, hcnt, nhall, dt0, dt1, hbx, N, PS);
                d0s[sI] = dt0; d1s[sI] = dt1;
              }
            }
            if (SR_DOUBLE == 1) {
              const int z = sr_opaque_zero();
#pragma unroll
              for (int sI = 0; sI < 16; ++sI) {
                if (sI >= p0 && sI < pend && !vetoed(sI)) {
                  const Prop q = load_prop(sI);
                  int dt0 = 0, dt1 = 0;
                  if (mt < ohi) taxon_dt(prop_kind(sI), q, a1 + z, b1, P + mt, pre + mt, M, hb1, hcnt, nhall, dt0, dt1, hbx, N, PS);
                  d0s[sI] |= dt0 & z; d1s[sI] |= dt1 & z;
                }
              }
            }
            }
            FST(3);
            if (SR_TSUMS && !GM && pack && pend - p0 >= SR_TSUMS) {   /* (GM: see below) */
              /* all 16 slots' sums of one wave in one transposed reduction (wave_sum32_t): values 0-15 the packed
                 X = (dt0 + N) | (dt1 + N) << 16, values 16-31 the nonzero counts (dt0 | dt1 != 0) | (dt0 != 0) << 16;
                 lanes 0-31 then hold one (list, slot) total each and write it (slots outside the batch: zeros,
                 never read) */
              uint32_t u[32];
#pragma unroll
              for (int sI = 0; sI < 16; ++sI) {
                u[sI] = (uint32_t)(d0s[sI] + N) | ((uint32_t)(d1s[sI] + N) << 16);
                u[16 + sI] = (uint32_t)((d0s[sI] | d1s[sI]) != 0) | ((uint32_t)(d0s[sI] != 0) << 16);
              }
              uint32_t v = wave_sum32_t(u, lane);
              if (SR_DOUBLE == 2) {
                const uint32_t z = (uint32_t)sr_opaque_zero();
#pragma unroll
                for (int sI = 0; sI < 16; ++sI) {
                  u[sI] = (uint32_t)(d0s[sI] + N) | ((uint32_t)(d1s[sI] + N) << 16) | z;
                  u[16 + sI] = ((uint32_t)((d0s[sI] | d1s[sI]) != 0) | ((uint32_t)(d0s[sI] != 0) << 16)) + z;
                }
                v |= wave_sum32_t(u, lane) & z;
              }
              const int sl = (((lane >> 1) & 1) << 3) | (((lane >> 2) & 1) << 2) | (((lane >> 3) & 1) << 1) | ((lane >> 4) & 1);
              const uint32_t pk = (uint32_t)__builtin_amdgcn_ds_bpermute(sl << 2, vpk);   /* slot sl's record */
              if (lane < 32) {
                int w0, w1;
                if (!(lane & 1)) { w0 = (int)(v & 0xffffu) - 64 * N; w1 = (int)(v >> 16) - 64 * N; }
                else {
                  const int any = (int)(v & 0xffffu), c0 = (int)(v >> 16);
                  const int pi = (int)(pk & 4095u), pj = (int)((pk >> 12) & 4095u);
                  /* pi1: exact nonzero counts (dt0 dt1 = 0); the reversals: the bound of the per-slot path */
                  const bool p1 = sl > 0 && (sl - 1) % 3 == 0;
                  w0 = p1 ? c0 : any * 2 * (max(pi, pj) - min(pi, pj) + 1);
                  w1 = p1 ? any - c0 : w0;
                }
                int *o = pw + (sl * NWV + wave) * 8 + 2 * (lane & 1);
                o[0] = w0; o[1] = w1;
              }
            } else if (SR_TSUMS && !pack && !GM && pend - p0 >= SR_TSUMS) {
              /* N >= 512 (the packed fields would overflow): two transposed reductions of 32 plain sums each,
                 (X0, X1) and (|dt0|, |dt1|) -- the per-slot path's exact Y.  Not in the HBM-column kernels: at
                 1024 threads (128 VGPRs) the 32 live sums spill and config 5 ran 5 % slower (r05f) */
              uint32_t u[32];
#pragma unroll
              for (int sI = 0; sI < 16; ++sI) { u[sI] = (uint32_t)d0s[sI]; u[16 + sI] = (uint32_t)d1s[sI]; }
              const int vx = (int)wave_sum32_t(u, lane);
#pragma unroll
              for (int sI = 0; sI < 16; ++sI) { u[sI] = (uint32_t)abs(d0s[sI]); u[16 + sI] = (uint32_t)abs(d1s[sI]); }
              const int vy = (int)wave_sum32_t(u, lane);
              const int sl = (((lane >> 1) & 1) << 3) | (((lane >> 2) & 1) << 2) | (((lane >> 3) & 1) << 1) | ((lane >> 4) & 1);
              if (lane < 32) {
                int *o = pw + (sl * NWV + wave) * 8 + (lane & 1);
                o[0] = vx; o[2] = vy;
              }
            } else {
#pragma unroll
            for (int sI = 0; sI < 16; ++sI) {
              if (full ? sI >= 1 : (sI >= p0 && sI < pend && !vetoed(sI))) {   /* (full: vetoed sums unread) */
                int X0, X1, Y0, Y1;
                if (prop_kind(sI) == PK_PI1) {   /* pi1: dt in {-1, 0, 1} and dt0 dt1 = 0: every sum is a ballot count */
                  const int cp0 = (int)__popcll(__ballot(d0s[sI] > 0)), cn0 = (int)__popcll(__ballot(d0s[sI] < 0));
                  const int cp1 = (int)__popcll(__ballot(d1s[sI] > 0)), cn1 = (int)__popcll(__ballot(d1s[sI] < 0));
                  X0 = cp0 - cn0; X1 = cp1 - cn1; Y0 = cp0 + cn0; Y1 = cp1 + cn1;
                } else if (pack) {   /* per-wave sums of (dt + N) fit 16-bit fields (N < 512) */
                  const uint32_t u1 = (uint32_t)wave_sum_i32((int)((uint32_t)(d0s[sI] + N) | ((uint32_t)(d1s[sI] + N) << 16)));
                  X0 = (int)(u1 & 0xffffu) - 64 * N; X1 = (int)(u1 >> 16) - 64 * N;
#ifdef SR_EXACT_Y
                  const uint32_t u2 = (uint32_t)wave_sum_i32((int)((uint32_t)abs(d0s[sI]) | ((uint32_t)abs(d1s[sI]) << 16)));
                  Y0 = (int)(u2 & 0xffffu); Y1 = (int)(u2 >> 16);
#else
                  /* the error bound needs only upper bounds of sum |dt0| and sum |dt1|: a reversal of
                     [ii, jj] changes a taxon's alive cells inside it only, |dt0| + |dt1| <= 2 (jj - ii + 1),
                     times the taxa with a nonzero change (one ballot instead of a second reduction) */
                  const Prop qb = load_prop(sI);
                  Y0 = Y1 = (int)__popcll(__ballot((d0s[sI] | d1s[sI]) != 0)) * 2 * (qb.jj - qb.ii + 1);
#endif
                } else {
                  X0 = wave_sum_i32(d0s[sI]); X1 = wave_sum_i32(d1s[sI]);
                  Y0 = wave_sum_i32(abs(d0s[sI])); Y1 = wave_sum_i32(abs(d1s[sI]));
                }
                if (lane == 0) {
                  int *o = pw + (sI * NWV + wave) * 8;
                  o[0] = X0; o[1] = X1; o[2] = Y0; o[3] = Y1;
                }
              }
            }
            }
            STAMP_K(PK_PI3);
          } else {
            /* several taxa per thread (M > TB; the HBM-column kernels): per taxon, every proposal slot
               unrolled (compile-time kinds) so that the taxon's state and column reads of all slots are
               in flight together -- one memory round trip per taxon, not one per proposal and taxon;
               per-slot sums kept in registers across the taxa */
            int x0s[16], x1s[16], ys[16];
            bool anyp3 = false;
#pragma unroll
            for (int sI = 0; sI < 16; ++sI) {
              x0s[sI] = 0; x1s[sI] = 0; ys[sI] = 0;
              if (prop_kind(sI) == PK_PI3) anyp3 |= sI >= p0 && sI < pend && !vetoed(sI);
            }
            for (int m0 = (SP ? olo : 0) + wave * 64; m0 < (SP ? ohi : M); m0 += TB) {   /* SP: own taxa */
              const int m = m0 + lane;
              const bool mv = m < (SP ? ohi : M);
              const int a = mv ? sab[m] : 0, b = mv ? sab[M + m] : 0;
              const HM hb = (anyp3 && mv) ? hard_bits_col<HM>(P + m, M, hl, nh) : (HM)0;
#pragma unroll
              for (int sI = 0; sI < 16; ++sI) {
                if (sI >= p0 && sI < pend && !vetoed(sI)) {
                  const Prop q = load_prop(sI);
                  int dt0 = 0, dt1 = 0;
                  if (mv) taxon_dt(prop_kind(sI), q, a, b, P + m, pre + m, M, hb, hcnt, nhall, dt0, dt1, hbx, N, PS);
                  x0s[sI] += dt0; x1s[sI] += dt1; ys[sI] += abs(dt0) + abs(dt1);
                }
              }
            }
#pragma unroll
            for (int sI = 0; sI < 16; ++sI) {
              if (sI >= p0 && sI < pend && !vetoed(sI)) {
                /* Y0 = Y1 = sum (|dt0| + |dt1|): upper bounds of both (the decision's error bound) */
                const int X0 = wave_sum_i32(x0s[sI]), X1 = wave_sum_i32(x1s[sI]), Y = wave_sum_i32(ys[sI]);
                if (lane == 0) {
                  int *o = pw + (sI * NWV + wave) * 8;
                  o[0] = X0; o[1] = X1; o[2] = Y; o[3] = Y;
                }
              }
            }
            STAMP_K(PK_PI3);
          }
          FST(4);
          SR_SYNC();
          if constexpr (SP) {   /* this half's sums of the batch's proposals (lane p of wave 0), exchanged */
            if (wave == 0 && lane >= p0 && lane < pend && lane < 16 && !((vpk >> 26) & 1)) {
              int X0 = 0, X1 = 0, Y0 = 0, Y1 = 0;
              for (int w = 0; w < NWV; ++w) {
                const int *o = pw + (lane * NWV + w) * 8;
                X0 += o[0]; X1 += o[1]; Y0 += o[2]; Y1 += o[3];
              }
              int *xp = xb + 16 + ((bpar * 2 + half) * 16 + lane) * 4;
              xst(xp, X0); xst(xp + 1, X1); xst(xp + 2, Y0); xst(xp + 3, Y1);
            }
            xsync();
          }
          STAMP_E(5);
          FST(5);

          /* ---- lane-parallel certified decisions (lane p decides proposal p; pc_classify / pc_resolve).
             cls: 0 rejected, 1 accepted, 2 needs the exact delta or the exact log. */
          const double aC = __builtin_fabs(K.cc) + __builtin_fabs(K.d), aD = __builtin_fabs(K.dd) + __builtin_fabs(K.c);
          double Sp = 0.0, Ebp = 0.0;
          int cls = 0, Knz = 0;
          uint32_t uwp = 1;
          {
            const int p = lane;
            if (p >= p0 && p < pend) {
              if (!((vpk >> 26) & 1)) {
                int X0 = 0, X1 = 0, Y0 = 0, Y1 = 0;
#pragma unroll
                for (int w = 0; w < NWV; ++w) {
                  const int *o = pw + (p * NWV + w) * 8;
                  X0 += o[0]; X1 += o[1]; Y0 += o[2]; Y1 += o[3];
                }
                if constexpr (SP) {   /* + the other half's */
                  const int *yp = xb + 16 + ((bpar * 2 + (half ^ 1)) * 16 + p) * 4;
                  X0 += xld(yp); X1 += xld(yp + 1); Y0 += xld(yp + 2); Y1 += xld(yp + 3);
                }
                uwp = (uint32_t)vuw;
                cls = pc_classify(X0, X1, Y0, Y1, K, aC, aD, PR, uwp, Sp, Ebp, Knz);
#ifdef SR_FORCE_EXACT   /* test build: every decision by the exact sequential delta */
                cls = (Knz == 0) ? 1 : 2;
                Ebp = __builtin_inf();
#else
                if (MCD) {   /* manycd: per-taxon coefficients, the exact sequential delta decides */
                  cls = (Knz == 0) ? 1 : 2;
                  Ebp = __builtin_inf();
                }
#endif
              }
            }
          }
          uint64_t pend_mask = __ballot(cls != 0);
          pend_mask = __builtin_amdgcn_readfirstlane((uint32_t)pend_mask) | ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(pend_mask >> 32)) << 32);
          bpar ^= 1;
          int acc_p = -1, used = 0;
          bool udrawn = false;
          double delta = 0.0;
          while (pend_mask) {
            const int p = __builtin_ctzll(pend_mask);
            pend_mask &= pend_mask - 1;
            const int kind = prop_kind(p);
            const Prop q = load_prop(p);
            const double S = readlane_f64(Sp, p), Eb = readlane_f64(Ebp, p);
            const int c0 = __builtin_amdgcn_readlane(cls, p), kz = __builtin_amdgcn_readlane(Knz, p);
            const double u = (double)(uint32_t)__builtin_amdgcn_readlane((int)uwp, p) / 4294967296.0;
            bool accept, have_exact;
            double dl;
            const bool decided = pc_resolve(S, Eb, c0, kz, u, tb, accept, udrawn, have_exact, dl);
            if (!decided || (accept && want_logl && !have_exact)) {   /* the exact sequential delta */
              if constexpr (SP)
                dl = sr_exact_delta<PR, GM, SP>(kind, q, K, sab, P, pre, M, N, KTC, olo, ohi, hl, nh, hcnt, nhall, hbx,
                                                cbuf + xpar * KTC * sr_chunk(PR), xb + 272 + xpar * KTC, xs, lane, wave,
                                                TB, xsync, nullptr, nullptr, PS);
              else   /* (no exchange: the one-workgroup kernels never see the split machinery) */
                dl = sr_exact_delta<PR, GM, SP>(kind, q, K, sab, P, pre, M, N, KTC, 0, M, hl, nh, hcnt, nhall, hbx,
                                                cbuf + xpar * KTC * sr_chunk(PR), ccnt + xpar * KTC, xs, lane, wave, TB,
                                                [] {}, cv, cx);
              xpar ^= 1;
              if (!decided) {
                if (tid == 0) misc[MS_NEXACT]++;
                if (dl >= 0.) { accept = true; udrawn = false; }
                else { udrawn = true; accept = dl > sr_log_m(u, &tb); }
              }
            }
            if (!accept) continue;
            delta = dl;
            acc_p = p;
            used = udrawn ? __builtin_amdgcn_readlane(voff, p) : __builtin_amdgcn_readlane(vnd, p);
            break;
          }
#ifdef SR_STAMP_DECIDE
          STAMP(6);
#else
          STAMP(7);
#endif
          FST(6);
          if (acc_p < 0) {   /* all of p0..pend-1 rejected or vetoed, as hypothesised */
            rng_skip(R, (uint32_t)__builtin_amdgcn_readlane(voff, pend - 1));
            p0 = pend;
            continue;
          }
          rng_skip(R, (uint32_t)used);
          p0 = acc_p + 1;

          /* ---- apply the accepted proposal acc_p */
          const int kind = prop_kind(acc_p);
          const Prop q = load_prop(acc_p);
          const int i = q.i, j = q.j, ii = q.ii, jj = q.jj, inc1 = q.inc1, inc2 = q.inc2, Kn = q.Kn;
          if (tid == 0) misc[MS_ACC + (kind == PK_PI1 ? 3 : kind == PK_PI2 ? 4 : kind == PK_SWAP ? 5 : 6)]++;
          loglik += delta;
          const int16_t *nhp = nhall + q.r0;   /* pi3: the non-hard positions of [i, j] in order */
          for (int m = (PR && hf) ? M : olo + tx; m < ohi; m += TXS) {   /* PR: the even lane of each pair; SP: own taxa */
            uint32_t *Pm = P + m;
            uint16_t *prem = pre + m;
            const int a = sab[m], b = sab[M + m];
            int dt0, dt1;
            taxon_dt(kind, q, a, b, Pm, prem, M, kind == PK_PI3 ? hard_bits_col<HM>(Pm, M, hl, nh) : (HM)0, hcnt, nhall, dt0, dt1,
                     hbx, N, PS);
            /* every read of the taxon's state before its first write (the compiler cannot tell the LDS / HBM
               arrays apart, so a read after a write waits for it: one round trip instead of one per access) */
            const int k0 = scnt[m], k1 = scnt[M + m], k2 = scnt[2 * M + m], k3 = scnt[3 * M + m];
            const int lo = min(i, j), hi = max(i, j), wl = lo >> 5, wh = hi >> 5;
            /* pi1 over at most 8 words (always at N <= 256): the words [wl - 1, wh + 1], the moved bit and the
               prefix below word wl read now; the shifted words and their prefix entries computed in registers */
            const bool reg1 = SR_APPLY_REG && (!GM || SR_GM_APPLY_REG) && kind == PK_PI1 && wh - wl < 8;   /* (GM: SR_GM_APPLY_REG) */
            uint32_t wv[10];
            uint32_t vb = 0u;
            int sbase = 0;
            if (reg1) {
#pragma unroll
              for (int t = 0; t < 10; ++t) {
                const int w = wl - 1 + t;
                wv[t] = (w >= 0 && w < NW && w <= wh + 1) ? Pm[w * M] : 0u;
              }
              vb = (Pm[(i >> 5) * M] >> (i & 31)) & 1u;
              sbase = prem[wl * PS];
            }
            scnt[m] = k0 + dt0; scnt[M + m] = k1 - dt0; scnt[2 * M + m] = k2 + dt1; scnt[3 * M + m] = k3 - dt1;
            int na_ = a, nb_ = b;   /* HBM columns: the new limits, stored below when they change */
            auto set_a = [&](int v) { if constexpr (GM) na_ = v; else sab[m] = v; };
            auto set_b = [&](int v) { if constexpr (GM) nb_ = v; else sab[M + m] = v; };
            if (reg1) {                                            /* mcmc.c:1266-1297 */
              if (i < j) {
                if (ii < a && a <= jj + 1) set_a(a - 1);
                if (ii < b && b <= jj + 1) set_b(b - 1);
              } else {
                if (ii <= a && a <= jj) set_a(a + 1);
                if (ii <= b && b <= jj) set_b(b + 1);
              }
              int sacc = sbase;
#pragma unroll
              for (int t = 1; t < 10; ++t) {
                const int w = wl - 1 + t;   /* words wl .. wh */
                if (w <= wh) {
                  const uint32_t old = wv[t];
                  const uint32_t sh = (i < j) ? ((old >> 1) | (wv[t + 1 < 10 ? t + 1 : 9] << 31)) : ((old << 1) | (wv[t - 1] >> 31));
                  const uint32_t m1 = (i < j) ? range_mask(w, i, j - 1) : range_mask(w, j + 1, i);
                  uint32_t nw = (old & ~m1) | (sh & m1);
                  if ((j >> 5) == w) nw = (nw & ~(1u << (j & 31))) | (vb << (j & 31));
                  Pm[w * M] = nw;
                  if (w < wh) { sacc += __popc(nw); prem[(w + 1) * PS] = (uint16_t)sacc; }   /* prefix entries (lo/32, hi/32] */
                }
              }
            } else {
            if (kind == PK_PI1) {                                  /* mcmc.c:1266-1297 */
              /* the shifted words read 8 at a time before they are rewritten (one memory round trip
                 per 8 words: the HBM-column kernels) */
              if (i < j) {
                if (ii < a && a <= jj + 1) set_a(a - 1);
                if (ii < b && b <= jj + 1) set_b(b - 1);
                const uint32_t vb = (Pm[(i >> 5) * M] >> (i & 31)) & 1u;
                for (int w0 = i >> 5; w0 <= (j >> 5); w0 += 8) {
                  uint32_t wv[9];
#pragma unroll
                  for (int t = 0; t < 9; ++t) wv[t] = (w0 + t <= (j >> 5) + 1 && w0 + t < NW) ? Pm[(w0 + t) * M] : 0u;
#pragma unroll
                  for (int t = 0; t < 8; ++t) {
                    const int w = w0 + t;
                    if (w <= (j >> 5)) {
                      const uint32_t old = wv[t], nxt = wv[t + 1];
                      const uint32_t sh = (old >> 1) | (nxt << 31);
                      const uint32_t m1 = range_mask(w, i, j - 1);
                      uint32_t nw = (old & ~m1) | (sh & m1);
                      if ((j >> 5) == w) nw = (nw & ~(1u << (j & 31))) | (vb << (j & 31));
                      Pm[w * M] = nw;
                    }
                  }
                }
              } else {
                if (ii <= a && a <= jj) set_a(a + 1);
                if (ii <= b && b <= jj) set_b(b + 1);
                const uint32_t vb = (Pm[(i >> 5) * M] >> (i & 31)) & 1u;
                for (int w0 = i >> 5; w0 >= (j >> 5); w0 -= 8) {
                  uint32_t wv[9];   /* wv[t] = word w0 - t */
#pragma unroll
                  for (int t = 0; t < 9; ++t) wv[t] = (w0 - t >= (j >> 5) - 1 && w0 - t >= 0) ? Pm[(w0 - t) * M] : 0u;
#pragma unroll
                  for (int t = 0; t < 8; ++t) {
                    const int w = w0 - t;
                    if (w >= (j >> 5)) {
                      const uint32_t old = wv[t], prv = wv[t + 1];
                      const uint32_t sh = (old << 1) | (prv >> 31);
                      const uint32_t m1 = range_mask(w, j + 1, i);
                      uint32_t nw = (old & ~m1) | (sh & m1);
                      if ((j >> 5) == w) nw = (nw & ~(1u << (j & 31))) | (vb << (j & 31));
                      Pm[w * M] = nw;
                    }
                  }
                }
              }
            } else {                                               /* mcmc.c:1446-1474, 1641-1670 */
              const int ain = ininterval(a, i, j + 1, inc1, inc2);
              const int bin = ininterval(b, i, j + 1, inc1, inc2);
              if (ain && !bin) set_a(i + j + 1 - a);
              else if (!ain && bin) set_b(i + j + 1 - b);
              else if (ain && bin) { set_b(i + j + 1 - a); set_a(i + j + 1 - b); }
              if (kind != PK_PI3) {
                for (int n = i; n < i + j - n; ++n) {
                  const int p2 = i + j - n;
                  const uint32_t b1 = (Pm[(n >> 5) * M] >> (n & 31)) & 1u, b2 = (Pm[(p2 >> 5) * M] >> (p2 & 31)) & 1u;
                  if (b1 != b2) { Pm[(n >> 5) * M] ^= (1u << (n & 31)); Pm[(p2 >> 5) * M] ^= (1u << (p2 & 31)); }
                }
              } else {
                for (int r = 0; r < Kn - 1 - r; ++r) {
                  const int n = nhp[r], p2 = nhp[Kn - 1 - r];
                  const uint32_t b1 = (Pm[(n >> 5) * M] >> (n & 31)) & 1u, b2 = (Pm[(p2 >> 5) * M] >> (p2 & 31)) & 1u;
                  if (b1 != b2) { Pm[(n >> 5) * M] ^= (1u << (n & 31)); Pm[(p2 >> 5) * M] ^= (1u << (p2 & 31)); }
                }
              }
            }
            {   /* the move permutes positions [lo, hi] only: prefix entries (lo/32, hi/32] change */
              const int rlo = wl + 1, rhi = wh;
              int sacc = prem[(rlo - 1) * PS];
              for (int r0 = rlo; r0 <= rhi; r0 += 8) {
                uint32_t wv[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) wv[t] = (r0 + t <= rhi) ? Pm[(r0 + t - 1) * M] : 0u;
#pragma unroll
                for (int t = 0; t < 8; ++t)
                  if (r0 + t <= rhi) { sacc += __popc(wv[t]); prem[(r0 + t) * PS] = (uint16_t)sacc; }
              }
            }
            }
            if constexpr (GM) {
              if (na_ != a) sab[m] = na_;
              if (nb_ != b) sab[M + m] = nb_;
            }
          }
          FST(7);
          /* rpi (double-buffered full permutation, read only at save time) and hard positions */
          bool hmoved = false;   /* wave-uniform */
          {
            const int32_t *ro = rcur ? rpiB : rpiA;
            int32_t *rn = rcur ? rpiA : rpiB;
            if (kind == PK_PI1) {
              for (int n = tid; n < N; n += TB) {
                int src = n;
                if (i < j) { if (n >= i && n < j) src = n + 1; else if (n == j) src = i; }
                else { if (n > j && n <= i) src = n - 1; else if (n == j) src = i; }
                rn[n] = ro[src];
              }
              for (int k0 = 0; k0 < nh; k0 += 64) {   /* one hard site per lane (several waves of them: > 64) */
                const int k = k0 + lane;
                const int h = (k < nh) ? hp[k] : -1;
                int hn = h;
                if (h == i) hn = j;
                else if (i < j && h > i && h <= j) hn = h - 1;
                else if (i > j && h >= j && h < i) hn = h + 1;
                hmoved = hmoved || __ballot(k < nh && hn != h) != 0;
                if (k < nh) hp[k] = hn;
              }
            } else if (kind != PK_PI3) {
              for (int n = tid; n < N; n += TB) rn[n] = ro[(n >= i && n <= j) ? (i + j - n) : n];
              for (int k0 = 0; k0 < nh; k0 += 64) {
                const int k = k0 + lane;
                const int h = (k < nh) ? hp[k] : -1;
                const bool mv = k < nh && h >= i && h <= j && i + j - h != h;
                hmoved = hmoved || __ballot(mv) != 0;
                if (mv) hp[k] = i + j - h;
              }
            } else {
              for (int n = tid; n < N; n += TB)
                if (n < i || n > j || hcnt[n + 1] != hcnt[n]) rn[n] = ro[n];
              for (int r = tid; r < Kn; r += TB) rn[nhp[r]] = ro[nhp[Kn - 1 - r]];
            }
            rcur ^= 1;
          }
          FST(10);
          /* the hard tables only when a hard site moved (the columns' hard-site bits never change) */
          if (hmoved) {   /* (block-uniform: every wave holds the same hard positions) */
            if constexpr (SHT) SR_SYNC(); else wsync();   /* SHT: every wave is past its reads of the shared tables */
            build_hard_tables(hp, nh, N, NW, hbw, hcnt, nhall, lane, !SHT || wave == 0);
            if constexpr (SHT) SR_SYNC();                 /* ... and the next batch reads the new ones */
            if (SR_DOUBLE == 8 && !SHT) { wsync(); build_hard_tables(hp, nh, N, NW, hbw, hcnt, nhall, lane); }
            tvalid = false;
            if (SR_COOP_TABLES > 1 && p0 < 16) {
              /* the proposal tables depend on the hard positions: refilled here by all threads at the next
                 batch's start (every wave is past this batch's table reads: the terms barrier), one barrier
                 instead of each wave refilling its own copy */
              rng_ensure(R, 133, tid, TB);
              tblk = R.blk;
              toff = R.off;
              const uint32_t sbase = (tblk & (SR_RING - 1)) * SR_MT_N + toff;
              const int savail = min((int)((R.gen - tblk) * SR_MT_N - toff), 128);
              for (int k = tid; k < 3 * 128; k += TB)
                ptab_fill(ptab, ring, sbase, savail, k & 127, k >> 7, N, nh, hcnt, nhall, mdN, mdN1, md2, mdH, mdH1);
              SR_SYNC();
              tvalid = true;
            }
          }
          FST(9);
          wsync();
          STAMP(7);
        } /* batches */
      }
      STAMP(7);
      FST(0);
      SR_SYNC();
      FST(11);
      }
    } /* sweeps */

    /* ---------------- saved sample (mcmc_save_chain, mcmc.c:69-92) */
    if (A.save) {
      const KArgs &B = kargs_late(A);
      const int slot = B.rec_base + call;
      const int W = 2 * M + N;
      int16_t *rec = B.rec_abpi + ((size_t)chain * B.rec_cap + slot) * W;
      if constexpr (SP) {   /* own taxa; the permutation and c, d, loglik from half 0 */
        for (int m = olo + tid; m < ohi; m += TB) { rec[m] = (int16_t)sab[m]; rec[M + m] = (int16_t)sab[M + m]; }
      } else {
        for (int m = tid; m < 2 * M; m += TB) rec[m] = (int16_t)sab[m];
      }
      const int32_t *rc = rcur ? rpiB : rpiA;
      if (!SP || half == 0)
        for (int n = tid; n < N; n += TB) rec[2 * M + rc[n]] = (int16_t)n;
      if (tid == 0 && (!SP || half == 0)) {
        double *rd = B.rec_cdl + ((size_t)chain * B.rec_cap + slot) * 3;
        rd[0] = c; rd[1] = d; rd[2] = loglik;
      }
      if constexpr (MCD) {   /* every taxon's c, d (mcmc.c:86-90) */
        double *rv = B.rec_cdv + ((size_t)chain * B.rec_cap + slot) * 2 * M;
        for (int m = tid; m < 2 * M; m += TB) rv[m] = cv[m];
      }
    }
  } /* calls */

  /* ---------------- store state */
  STAMP(7);
  STAMP_STORE(A.dbg);
#ifdef SR_STAMPS
  if (tid == 0) { A.dbg[blockIdx.x * 17 * 8 + 0] += misc[MS_NEXACT]; for (int q_ = 0; q_ < 4; ++q_) A.dbg[blockIdx.x * 17 * 8 + 1 + q_] += misc[MS_FBK + q_];
                  for (int q_ = 0; q_ < 3; ++q_) A.dbg[blockIdx.x * 17 * 8 + 5 + q_] += misc[40 + q_];
#if !defined(SR_STAMP_FINE) && !defined(SR_STAMP_GIBBS)
                  if (TB <= 512) A.dbg[(blockIdx.x * 17 + 9) * 8 + 0] += misc[43];   /* (row 9: no wave's stamps) */
#endif
#if defined(SR_STAMP_GIBBS) || defined(SR_STAMP_FINE)
                  for (int q_ = 0; q_ < 3; ++q_) A.dbg[blockIdx.x * 17 * 8 + 5 + q_] = misc[MS_FBK + 26 + q_];
                  A.dbg[blockIdx.x * 17 * 8 + 4] = misc[MS_FBK + 29];
#endif
                }
#endif
  __syncthreads();
  const KArgs &B = kargs_late(A);
  uint32_t *oP = B.P + (size_t)chain * NW * M;
  if (!GM) for (int i = tid; i < NW * M; i += TB) oP[i] = P[i];
  const int32_t *rc = rcur ? rpiB : rpiA;
  int32_t *orpi = B.rpi + (size_t)chain * N;
  uint32_t *omt = B.mt + (size_t)chain * SR_RING * SR_MT_N;
  if (!SP || half == 0) {   /* SP: block-uniform state, identical in both halves */
    for (int i = tid; i < N; i += TB) orpi[i] = rc[i];
    for (int i = tid; i < SR_RING * SR_MT_N; i += TB) omt[i] = ring[i];
  }
  int32_t *oab = B.ab + (size_t)chain * 2 * M;
  if (!GM) for (int i = tid; i < 2 * M; i += TB) oab[i] = sab[i];
  int32_t *ocnt = B.cnt + (size_t)chain * 4 * M;
  if (!GM) for (int i = tid; i < 4 * M; i += TB) ocnt[i] = scnt[i];
  if (tid == 0) {
    uint64_t *acc = B.acc + (size_t)chain * SR_NACC;
    if (!SP || half == 0) {
      for (int k = 0; k < nh; ++k) B.hp[(size_t)chain * NHC + k] = hp[k];
      B.cdl[(size_t)chain * 4 + 0] = c;
      B.cdl[(size_t)chain * 4 + 1] = d;
      B.cdl[(size_t)chain * 4 + 2] = loglik;
      B.rng[(size_t)chain * 2 + 0] = (uint64_t)R.blk * SR_MT_N + R.off;
      B.rng[(size_t)chain * 2 + 1] = R.gen;
      for (int k = 0; k < 7; ++k)
        if (k != 2) acc[k] += misc[MS_ACC + k];
      acc[7] += misc[MS_NEXACT];
      acc[9] += misc[MS_CDSEQ];
    }
    /* the Gibbs counters (a / b changes, exact-walk fallbacks) are per half under SP: atomics */
    if constexpr (SP) {
      atomicAdd((unsigned long long *)acc + 2, (unsigned long long)(misc[MS_ACC + 2] + misc[MS_CAB]));
      atomicAdd((unsigned long long *)acc + 8, (unsigned long long)misc[MS_FBK]);
    } else {
      acc[2] += misc[MS_ACC + 2] + misc[MS_CAB];
      acc[8] += misc[MS_FBK];
    }
  }
}

#ifdef SR_JIT
/* the shape-specialised build (sr_spec.c): this one instantiation, specialised by SR_FN / SR_FM / SR_FH, and
   its ABI record, which the loader compares with its own before launching (srk_spec_load) */
template __global__ void sr_sweep_kernel<SR_JIT_TB, SR_JIT_NWM, false>(KArgs);
__constant__ unsigned long long sr_spec_abi[4] = {
    sizeof(KArgs), (unsigned long long)SR_JIT_TB | ((unsigned long long)SR_JIT_NWM << 16),
    (unsigned long long)SR_FN | ((unsigned long long)SR_FM << 16) | ((unsigned long long)(SR_FH & 0xffff) << 32),
    (unsigned long long)sr_layout(SR_FN, SR_FM, (SR_FN + 31) / 32, SR_JIT_TB, false, false, SR_FH).total};
#else
/* ================================================================ session layer */
#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "seriation: HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return -5; } } while (0)


struct srk_dev {
  int device, N, M, NW, nh, nchains, TB, TPT, rec_cap, gm, pr, sp, grid, coop;
  int lck;                 /* split kernels: Gibbs checkpoints in LDS (LK kernels) */
  int mcd;                 /* manycd: per-taxon c, d (MCD kernels) */
  int jit;                 /* the launch uses the shape-specialised kernel (srk_spec_load) */
  int jemb;                /* ... and its code object is the one embedded in the library */
  double *dsum;            /* srk_exp_data's per-chain sums (device) */
  hipModule_t mod;
  hipFunction_t jfn;
  size_t lds;
  hipStream_t stream;
  int own_stream;
  hipEvent_t ev0, ev1;
  int have_events;
  KArgs args;
  void *bufs[24];
  int nbufs;
};

typedef void (*sr_kfn)(KArgs);

/* NWM: walks of <= 9 / 17 words (N + 1 entries: N <= 287 / 543) use the register-resident
 * Gibbs draw, longer ones the LDS walk.  gm: the HBM-column variant (sr_layout) */
/* the pair kernel (two lanes per taxon, 1024 threads): walks of <= 9 words (N <= 287) and 257..512
 * taxa with columns in LDS.  Opt-in (SR_KERNEL=pair in the environment): bit-exact, but 1.67x slower
 * than the one-thread-per-taxon kernel on the bench workload (profiles/r03c_ab_pair.json: 24.6 vs
 * 14.7 ms per launch) -- its per-wave instruction count fell only 13 % (4.3 k vs 5.0 k VALU per
 * wave per sweep: most of a wave's work is per proposal and per sweep, not per taxon, and all 16
 * waves repeat it), the 128-VGPR budget spills 171 registers, and waves park 60 % of their cycles
 * (r03d SQ passes). */
static bool sr_pair_ok(int N, int M)
{
  const char *e = getenv("SR_KERNEL");
  if (!e || strcmp(e, "pair") != 0) return false;
  return sr_nwm(N) == 9 && M > 256 && M <= 512;
}

static sr_kfn sr_pick_kernel(int TB, int N, int M, bool gm, bool pr, int nh, bool sp = false, bool mcd = false,
                             bool lk = false)
{
  if (mcd) {   /* manycd: the generic one-workgroup kernels at 1024 threads */
    if (TB != 1024 || pr || sp) return nullptr;
    return gm ? (sr_kfn)sr_sweep_kernel<1024, 0, true, false, false, true>
              : (sr_kfn)sr_sweep_kernel<1024, 0, false, false, false, true>;
  }
  if (pr) return (TB == 1024 && !gm) ? (sr_kfn)sr_sweep_kernel<1024, 9, false, true> : nullptr;
#ifndef SR_STAMPS
  if (sp) {   /* LK: checkpoints in LDS (where the layout fits them), else in HBM scratch */
    if (!gm) return nullptr;
    if (TB == 1024) return lk ? (sr_kfn)sr_sweep_kernel<1024, 0, true, false, true, false, true>
                              : (sr_kfn)sr_sweep_kernel<1024, 0, true, false, true>;
    if (TB == 512) return lk ? (sr_kfn)sr_sweep_kernel<512, 0, true, false, true, false, true>
                             : (sr_kfn)sr_sweep_kernel<512, 0, true, false, true>;
    return nullptr;
  }
#else
  if (sp) return nullptr;   /* (stamp builds index their counters by block) */
#endif
#ifdef SR_PAIR_ONLY   /* register-pressure experiments: compile the pair kernel alone */
  return nullptr;
#endif
  if (gm) {
    if (TB == 256) return (sr_kfn)sr_sweep_kernel<256, 0, true>;
    if (TB == 512) return (sr_kfn)sr_sweep_kernel<512, 0, true>;
    if (TB == 1024) return (sr_kfn)sr_sweep_kernel<1024, 0, true>;
    return nullptr;
  }
  const int nwm = sr_regwalk(N, M, TB, false, nh) ? sr_nwm(N) : 0;
  if (TB == 256) return nwm == 9 ? (sr_kfn)sr_sweep_kernel<256, 9, false> : nwm == 17 ? (sr_kfn)sr_sweep_kernel<256, 17, false> : (sr_kfn)sr_sweep_kernel<256, 0, false>;
  if (TB == 512) return nwm == 9 ? (sr_kfn)sr_sweep_kernel<512, 9, false> : nwm == 17 ? (sr_kfn)sr_sweep_kernel<512, 17, false> : (sr_kfn)sr_sweep_kernel<512, 0, false>;
  if (TB == 1024) return (sr_kfn)sr_sweep_kernel<1024, 0, false>;
  return nullptr;
}

/* ---- the kernel a session runs ----------------------------------------------------------------
 * Block size, variant (LDS columns / HBM columns / pair kernel) and LDS bytes from the shape alone (no
 * HIP call): srk_create launches this plan, srk_plan / sr_specialize report it without a GPU. */
struct srk_kplan { int TB, pr, gm, mcd; size_t lds; };

static int plan_kernel(int N, int M, int nh, int block_threads, int gm_force, int mcd, srk_kplan *kp)
{
  if (nh > N || N > 4095 || M > SR_MMAX) return -6;
  const int NW = (N + 31) / 32;
  int TB = block_threads;
  if (mcd) {   /* manycd: 1024 threads (one or more taxa per thread) */
    if (TB > 0 && TB != 1024) return -6;
    TB = 1024;
  }
  /* the pair kernel where it was asked for (two lanes per taxon, 1024 threads), else one thread per
     taxon in the smallest block of 256..1024 threads that covers M */
  int pr = (TB <= 0 && !mcd && gm_force != 1 && nh <= 32 && sr_pair_ok(N, M)) ? 1 : 0;
  if (pr) TB = 1024;
  if (TB <= 0) { TB = 256; while (TB < M && TB < 1024) TB *= 2; }
  /* columns in LDS when the whole layout fits, else the HBM-column variant */
  int gm = 0;
  Lay L = sr_layout(N, M, NW, TB, false, pr != 0, nh);
  if (L.total > 160 * 1024 && block_threads <= 0 && !mcd && !pr && gm_force != 1 && TB == 1024 && M <= 1024) {
    /* mid-size shapes (513-1024 taxa, N up to ~320): the 1024-thread LDS layout does not fit, a 512-thread one (two
       taxa per thread) does -- LDS columns there beat HBM columns at 1024 threads by 11-30 % (256 x 600, 200 x 800,
       128 x 1000: profiles/r06c_ab_planner.json, same box, parity legs green) */
    const Lay L2 = sr_layout(N, M, NW, 512, false, false, nh);
    if (L2.total <= 160 * 1024 && sr_pick_kernel(512, N, M, false, false, nh, false, false)) { TB = 512; L = L2; }
  }
  if (L.total > 160 * 1024) { gm = 1; L = sr_layout(N, M, NW, TB, true, false, nh); }
  if (gm_force >= 0 && gm_force != gm) {   /* explicit variant request (tests) */
    gm = gm_force;
    L = sr_layout(N, M, NW, TB, gm != 0, pr != 0, nh);
  }
  if (gm) pr = 0;
  if (!sr_pick_kernel(TB, N, M, gm != 0, pr != 0, nh, false, mcd != 0) || L.total > 160 * 1024) return -6;
  kp->TB = TB; kp->pr = pr; kp->gm = gm; kp->mcd = mcd; kp->lds = L.total;
  return 0;
}

/* the specialised kernel's shape: LDS-column sessions of the one-thread-per-taxon kernels (the HBM-column
   split kernel measured 4.4 % slower specialised, profiles/r03z6_ab_jit.json; the pair kernel is opt-in) */
static bool spec_shape_of(int N, int M, int nh, const srk_kplan &kp, sr_spec_shape *s)
{
  if (kp.gm || kp.pr || kp.mcd) return false;
  s->TB = kp.TB;
  s->NWM = sr_regwalk(N, M, kp.TB, false, nh) ? sr_nwm(N) : 0;
  s->N = N; s->M = M; s->NH = nh;
#ifdef SR_FORCE_EXACT
  s->force = 1;
#else
  s->force = 0;
#endif
  return true;
}

extern "C" int srk_plan(int N, int M, int nh, int block_threads, int gm_force, int manycd, sr_spec_shape *shape)
{
  srk_kplan kp;
  if (int e = plan_kernel(N, M, nh, block_threads, gm_force, manycd, &kp)) return e;
  return spec_shape_of(N, M, nh, kp, shape) ? 1 : 0;
}

/* ---- shape-specialised kernels (the default for LDS-column sessions; sr_spec.c) -----------------
 * The generic kernels take N, M and the hard-site count from their launch arguments; at 256 VGPRs and
 * two waves per SIMD the bench kernel then holds layout offsets, strides, loop bounds and the five
 * uniform_int divisors' magic numbers in ~590 spilled SGPRs.  The session's kernel compiled with them
 * fixed (sr_spec.c: from the source snapshot the library was built from, cached) spills ~170.  Same
 * source and -ffp-contract=off: the same arithmetic in the same order, bit-identical results
 * (tests/test_gpu_jit.py, and every GPU parity test runs it by default).  The code object's ABI record
 * (sizeof KArgs, block, walk words, shape, LDS bytes) must equal this library's, else it is not used.
 * Any failure leaves the generic HIP kernel in place, with one stderr line per reason; there is no CPU
 * path either way. */
/* where a session's specialised code object comes from, resolved before any HIP call of srk_create (a compile,
   when one is needed, happens here and says so on stderr): embedded in the library (the shapes of
   csrc/sr_embed_shapes.txt), else the cache, else compiled into it.  0 = found (img != NULL: embedded, else
   path), -1 = the session runs no specialised kernel, else the sr_spec.c reason (already reported). */
struct srk_spec_src { sr_spec_shape s; const void *img; size_t bytes; char path[4608]; };

static int srk_spec_resolve(int N, int M, int nh, const srk_kplan &kp, srk_spec_src *src)
{
#if defined(SR_STAMPS)
  (void)N; (void)M; (void)nh; (void)kp; (void)src;
  return -1;   /* (stamp builds: generic kernels only) */
#else
  if (!spec_shape_of(N, M, nh, kp, &src->s)) return -1;
  src->img = sr_spec_embedded(&src->s, &src->bytes);
  src->path[0] = 0;
  if (src->img) return 0;
  /* SR_JIT=cache: a deployment that never spawns the compiler from a session -- embedded or cached (sr_specialize
     ahead of time) objects only, else the generic kernel */
  const char *jm = getenv("SR_JIT");
  int rc;
  if (jm && !strcmp(jm, "cache")) {
    rc = sr_spec_path(&src->s, src->path, sizeof src->path);
    if (!rc && access(src->path, R_OK) != 0) rc = SR_SPEC_ENOJIT;
  } else {
    rc = sr_spec_object(&src->s, src->path, sizeof src->path, 1);
  }
  if (rc) sr_spec_note(rc, rc == SR_SPEC_ECC ? src->path : nullptr);
  return rc;
#endif
}

static int srk_spec_load(srk_dev *d, const srk_spec_src *src)
{
  const sr_spec_shape &s = src->s;
  char log[4700];
  char name[128];
  snprintf(name, sizeof name, "_Z15sr_sweep_kernelILi%dELi%dELb0ELb0ELb0ELb0ELb0EEv5KArgs", s.TB, s.NWM);
  unsigned long long abi[4] = {0, 0, 0, 0};
  const unsigned long long want[4] = {
      sizeof(KArgs), (unsigned long long)s.TB | ((unsigned long long)s.NWM << 16),
      (unsigned long long)s.N | ((unsigned long long)s.M << 16) | ((unsigned long long)(s.NH & 0xffff) << 32),
      (unsigned long long)d->lds};
  hipDeviceptr_t ga = nullptr;
  size_t gbytes = 0;
  const char *what = nullptr;
  const hipError_t le = src->img ? hipModuleLoadData(&d->mod, src->img) : hipModuleLoad(&d->mod, src->path);
  if (le != hipSuccess) { d->mod = nullptr; what = src->img ? "hipModuleLoadData" : "hipModuleLoad"; }
  else if (hipModuleGetFunction(&d->jfn, d->mod, name) != hipSuccess) what = "hipModuleGetFunction";
  else if (hipModuleGetGlobal(&ga, &gbytes, d->mod, "sr_spec_abi") != hipSuccess || gbytes != sizeof abi ||
           hipMemcpyDtoH(abi, ga, sizeof abi) != hipSuccess) what = "no ABI record";
  else if (memcmp(abi, want, sizeof abi) != 0) what = "ABI record differs";
  if (what) {
    (void)hipGetLastError();   /* the failed module call's error must not surface at the first generic launch */
    snprintf(log, sizeof log, "%s (%s)", src->img ? "embedded code object" : src->path, what);
    sr_spec_note(SR_SPEC_ELOAD, log);
    if (d->mod) (void)hipModuleUnload(d->mod);
    d->mod = nullptr; d->jfn = nullptr;
    return SR_SPEC_ELOAD;
  }
  d->jit = 1;
  d->jemb = src->img != nullptr;
  return 0;
}

/* public (include/seriation.h): fill the specialised-kernel cache for a dataset without a GPU */
extern "C" int sr_specialize(const sr_dataset *ds, const sr_run_opts *opts)
{
  if (!ds || ds->N <= 0 || ds->M <= 0 || ds->nh < 0) return SR_EINVAL;
  sr_run_opts o;
  if (opts) o = *opts;
  else sr_default_opts(&o);
  if (o.flags & SR_F_GENERIC_KERNEL) return 0;
  const int gm_force = (o.flags & SR_F_HBM_COLUMNS) ? 1 : ((o.flags & SR_F_LDS_COLUMNS) ? 0 : -1);
  sr_spec_shape s;
  const int r = srk_plan(ds->N, ds->M, ds->nh, o.block_threads, gm_force, o.manycd != 0, &s);
  if (r <= 0) return r < 0 ? SR_EUNSUPPORTED : 0;
#if defined(SR_STAMPS)
  return 0;
#else
  size_t bytes = 0;
  if (sr_spec_embedded(&s, &bytes)) return 1;   /* linked into the library: nothing to prepare */
  char path[4608];
  const int rc = sr_spec_object(&s, path, sizeof path, 0);
  if (rc) {
    sr_spec_note(rc, rc == SR_SPEC_ECC ? path : nullptr);
    return SR_EIO;
  }
  return 1;
#endif
}

/* test hook: the cache path of the specialised kernel a session of this shape would load (0), else the
   sr_spec.c reason or 1 when the session would run no specialised kernel */
extern "C" int sr_spec_cache_path(int N, int M, int nh, int block_threads, char *path, size_t len)
{
  sr_spec_shape s;
  const int r = srk_plan(N, M, nh, block_threads, -1, 0, &s);
  if (r <= 0) return 1;
  return sr_spec_path(&s, path, len);
}

extern "C" int srk_device_count(void)
{
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

template <typename T>
static int dev_alloc_copy(srk_dev *d, T **dst, const T *src, size_t n)
{
  void *p = nullptr;
  HIPCHK(hipMalloc(&p, n * sizeof(T) + 16));
  d->bufs[d->nbufs++] = p;
  if (src) HIPCHK(hipMemcpy(p, src, n * sizeof(T), hipMemcpyHostToDevice));
  else HIPCHK(hipMemset(p, 0, n * sizeof(T)));
  *dst = (T *)p;
  return 0;
}

extern "C" int srk_create(const sr_state_host *st, int device, int block_threads, int rec_cap_calls, int gm_force,
                          const uint32_t *pkey, int spec, srk_dev **out)
{
  srk_kplan kp;
  if (plan_kernel(st->N, st->M, st->nh, block_threads, gm_force, st->manycd, &kp)) return -6;
  /* the specialised code object first: any compile happens before the device is touched */
  srk_spec_src *ssrc = spec ? new srk_spec_src() : nullptr;
  const int sres = ssrc ? srk_spec_resolve(st->N, st->M, st->nh, kp, ssrc) : -1;
  struct Free { srk_spec_src *p; ~Free() { delete p; } } ssrc_free{ssrc};
  int ndev = srk_device_count();
  if (ndev <= 0 || device < 0 || device >= ndev) return -5;
  HIPCHK(hipSetDevice(device));
  srk_dev *d = new srk_dev();
  d->device = device; d->N = st->N; d->M = st->M; d->NW = st->NW; d->nh = st->nh; d->nchains = st->nchains;
  const int TB = kp.TB;
  d->TB = TB; d->TPT = 1; d->pr = kp.pr; d->gm = kp.gm; d->mcd = kp.mcd; d->lds = kp.lds;
  /* split chains (two co-resident workgroups per chain, one taxon per thread): HBM columns at 1024
     threads when the taxa exceed one block but each half fits it, and the whole grid (16 blocks per
     8 chains) is co-resident -- launched cooperatively.  SR_SPLIT=0 disables it, SR_SPLIT=1 also
     splits chains of <= 1024 taxa (tests). */
  d->sp = 0; d->grid = st->nchains;
  {
    const char *e = getenv("SR_SPLIT");
    const int want = e ? atoi(e) : -1;
    const int Mh = sr_sp_half(st->M);
    /* the split kernels' own layout: Gibbs checkpoints in LDS where they fit (SR_SP_LCK; up to N ~ 1300 at 1024
       threads), else in HBM scratch (round 4's form; any N) */
    const size_t lds_lk = sr_layout(st->N, st->M, st->NW, TB, true, false, st->nh, true).total;
    const bool lk = SR_SP_LCK && lds_lk <= 160 * 1024;
    const size_t lds_sp = lk ? lds_lk : sr_layout(st->N, st->M, st->NW, TB, true, false, st->nh, false).total;
    sr_kfn ks = sr_pick_kernel(TB, st->N, st->M, true, false, st->nh, true, false, lk);
    if (lds_sp > 160 * 1024) ks = nullptr;
    /* SR_SPLIT=2 (experiment, opt-in only): 512-thread halves of up to two blocks' taxa, several taxa per
       thread (256 VGPRs, 8 waves per CU; measured slower) -- never chosen without it */
    if (want != 0 && !d->mcd && d->gm && ks && ((TB == 1024 && Mh <= TB) || (want == 2 && TB == 512 && Mh <= 2 * TB)) &&
        st->M > 128 &&
        (st->M > TB || want >= 1)) {
      int cus = 0, occ = 0, coop = 0;
      const int grid = 16 * ((st->nchains + 7) / 8);
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
          hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, device) == hipSuccess && coop &&
          hipFuncSetAttribute((const void *)ks, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_sp) == hipSuccess &&
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void *)ks, TB, lds_sp) == hipSuccess &&
          grid <= occ * cus) {
        d->sp = 1;
        d->lck = lk ? 1 : 0;
        d->grid = grid;
        d->lds = lds_sp;
        /* SR_COOP=0: an ordinary launch of the same grid (rocprofv3's kernel tracer crashes at
           process exit after cooperative launches; on an otherwise idle GPU the grid is resident
           anyway, and a wait that times out fails the session instead of hanging) */
        const char *ce = getenv("SR_COOP");
        d->coop = (ce && atoi(ce) == 0) ? 0 : 1;
      }
    }
  }
  d->rec_cap = rec_cap_calls > 0 ? rec_cap_calls : 1;
  const size_t C = st->nchains;
  KArgs &A = d->args;
  memset(&A, 0, sizeof(A));
  A.N = st->N; A.M = st->M; A.NW = st->NW; A.nh = st->nh; A.nchains = st->nchains; A.rec_cap = d->rec_cap;
  int rc = 0;
  rc |= dev_alloc_copy(d, &A.P, st->P, C * st->NW * st->M);
  rc |= dev_alloc_copy(d, &A.rpi, st->rpi, C * st->N);
  rc |= dev_alloc_copy(d, &A.hp, st->hp, C * SR_NHCAP(st->nh));
  rc |= dev_alloc_copy(d, &A.ab, st->ab, C * 2 * st->M);
  rc |= dev_alloc_copy(d, &A.cnt, st->cnt, C * 4 * st->M);
  rc |= dev_alloc_copy(d, &A.cdl, st->cdl, C * 4);
  rc |= dev_alloc_copy(d, &A.mt, st->mt, C * SR_RING * SR_MT_N);
  rc |= dev_alloc_copy(d, &A.rng, st->rng, C * 2);
  rc |= dev_alloc_copy(d, &A.acc, st->acc, C * SR_NACC);
  rc |= dev_alloc_copy(d, &A.rec_abpi, (const int16_t *)nullptr, C * d->rec_cap * (2 * st->M + st->N));
  rc |= dev_alloc_copy(d, &A.rec_cdl, (const double *)nullptr, C * d->rec_cap * 3);
  rc |= dev_alloc_copy(d, &A.dbg, (const unsigned long long *)nullptr, C * 17 * 8);
  if (pkey) rc |= dev_alloc_copy(d, &A.pkey, pkey, C * 2);
  if (d->gm) {
    rc |= dev_alloc_copy(d, &A.gpre, (const uint16_t *)nullptr, C * sr_gm_pre(st->M, st->NW));
    using CKT = typename std::conditional<SR_CK32 != 0, float, double>::type;
    CKT *gck = nullptr;
    /* (split kernels with their checkpoints in LDS: no HBM scratch) */
    rc |= dev_alloc_copy(d, &gck, (const CKT *)nullptr,
                         C * (d->sp ? ((d->lck && !SR_SP_LPRE) ? 0 : sr_sp_ck(st->N, TB)) : sr_gm_ck(st->N, st->M, TB)));
    A.gck = gck;
    rc |= dev_alloc_copy(d, &A.glbuf, (const double *)nullptr, C * st->M);
    rc |= dev_alloc_copy(d, &A.gcbuf, (const double *)nullptr, C * sr_gm_cbuf(st->M));
  }
  if (d->mcd) {
    rc |= dev_alloc_copy(d, &A.cdv, (const double *)st->cdv, C * 2 * st->M);
    rc |= dev_alloc_copy(d, &A.cdx, (const double *)nullptr, C * 2 * st->M);
    rc |= dev_alloc_copy(d, &A.rec_cdv, (const double *)nullptr, C * d->rec_cap * 2 * st->M);
  }
  if (d->sp) {
    rc |= dev_alloc_copy(d, &A.xflag, (const int *)nullptr, C * 2);
    rc |= dev_alloc_copy(d, &A.xbuf, (const int *)nullptr, C * sr_sp_xb(st->M));
    rc |= dev_alloc_copy(d, &A.xerr, (const int *)nullptr, 1);
  }
  if (rc) { srk_destroy(d); return -5; }
  sr_kfn k = sr_pick_kernel(TB, st->N, st->M, d->gm != 0, d->pr != 0, st->nh, d->sp != 0, d->mcd != 0, d->lck != 0);
  if (hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)d->lds) != hipSuccess) {
    srk_destroy(d);
    return -5;
  }
  if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) { srk_destroy(d); return -5; }
  d->own_stream = 1;
  if (hipEventCreate(&d->ev0) == hipSuccess && hipEventCreate(&d->ev1) == hipSuccess) d->have_events = 1;
  if (sres == 0) (void)srk_spec_load(d, ssrc);
  *out = d;
  return 0;
}

extern "C" int srk_set_stream(srk_dev *d, void *stream)
{
  HIPCHK(hipSetDevice(d->device));
  /* work already queued on the old stream reads and writes the chain state the next launch
     uses: drain it before switching, so the launch order is the call order */
  HIPCHK(hipStreamSynchronize(d->stream));
  if (d->own_stream) { (void)hipStreamDestroy(d->stream); d->own_stream = 0; }
  d->stream = (hipStream_t)stream;
  return 0;
}

extern "C" int srk_run(srk_dev *d, int calls, int spc, int save, int rec_base)
{
  if (calls <= 0) return 0;
  if (save && rec_base + calls > d->rec_cap) return -1;
  HIPCHK(hipSetDevice(d->device));
  KArgs A = d->args;
  A.calls = calls; A.spc = spc; A.save = save; A.rec_base = rec_base;
  sr_kfn k = sr_pick_kernel(d->TB, d->N, d->M, d->gm != 0, d->pr != 0, d->nh, d->sp != 0, d->mcd != 0, d->lck != 0);
  if (d->sp) HIPCHK(hipMemsetAsync(A.xflag, 0, (size_t)d->nchains * 2 * sizeof(int), d->stream));   /* exchange sequence restarts */
  if (d->have_events) HIPCHK(hipEventRecord(d->ev0, d->stream));
  if (d->jit) {   /* the run-time specialised kernel (same arguments; LDS columns: one workgroup per chain) */
    void *kp[] = {&A};
    HIPCHK(hipModuleLaunchKernel(d->jfn, (unsigned)d->nchains, 1, 1, d->TB, 1, 1, (unsigned)d->lds, d->stream, kp, nullptr));
  } else if (d->sp && d->coop) {   /* both halves of every chain must be resident together */
    void *kargs[] = {&A};
    HIPCHK(hipLaunchCooperativeKernel((const void *)k, dim3(d->grid), dim3(d->TB), kargs, (unsigned)d->lds, d->stream));
  } else if (d->sp) {
    hipLaunchKernelGGL(k, dim3(d->grid), dim3(d->TB), d->lds, d->stream, A);
  } else {
    hipLaunchKernelGGL(k, dim3(d->nchains), dim3(d->TB), d->lds, d->stream, A);
  }
  HIPCHK(hipGetLastError());
  if (d->have_events) HIPCHK(hipEventRecord(d->ev1, d->stream));
  return 0;
}

/* split chains: a half that waited past its deadline (the other half not resident) left garbage */
static int sp_check(srk_dev *d)
{
  if (!d->sp) return 0;
  int e = 0;
  HIPCHK(hipMemcpy(&e, d->args.xerr, sizeof(int), hipMemcpyDeviceToHost));
  if (e) { fprintf(stderr, "seriation: split-chain exchange timed out (halves not co-resident)\n"); return -5; }
  return 0;
}

extern "C" int srk_sync(srk_dev *d)
{
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipStreamSynchronize(d->stream));
  return sp_check(d);
}

extern "C" double srk_last_ms(srk_dev *d)
{
  if (!d->have_events) return -1.0;
  float ms = -1.0f;
  if (hipEventSynchronize(d->ev1) != hipSuccess) return -1.0;
  if (hipEventElapsedTime(&ms, d->ev0, d->ev1) != hipSuccess) return -1.0;
  return (double)ms;
}

extern "C" int srk_block_threads(const srk_dev *d) { return d->TB; }
extern "C" int srk_variant(const srk_dev *d) { return d->gm ? (d->sp ? 3 : 1) : (d->pr ? 2 : 0); }
extern "C" int srk_specialized(const srk_dev *d) { return d->jit ? (d->jemb ? 2 : 1) : 0; }   /* 2: embedded */

extern "C" int srk_fetch_dbg(srk_dev *d, unsigned long long *out)
{
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipStreamSynchronize(d->stream));
  HIPCHK(hipMemcpy(out, d->args.dbg, (size_t)d->nchains * 17 * 8 * 8, hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int srk_fetch_records(srk_dev *d, int first, int count, int16_t *ab_pi, double *cdl)
{
  if (first < 0 || count < 0 || first + count > d->rec_cap) return -1;
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipStreamSynchronize(d->stream));
  if (int e = sp_check(d)) return e;
  if (count == 0) return 0;
  const size_t W = 2 * (size_t)d->M + d->N;
  /* chain c's rows [first, first + count) of its rec_cap-row slab; one copy when they are the whole slab */
  const bool whole = (first == 0 && count == d->rec_cap);
  for (int c = 0; c < (whole ? 1 : d->nchains); ++c) {
    const size_t rows = whole ? (size_t)d->nchains * count : (size_t)count;
    if (ab_pi)
      HIPCHK(hipMemcpy(ab_pi + (size_t)c * count * W, d->args.rec_abpi + ((size_t)c * d->rec_cap + first) * W,
                       rows * W * sizeof(int16_t), hipMemcpyDeviceToHost));
    if (cdl)
      HIPCHK(hipMemcpy(cdl + (size_t)c * count * 3, d->args.rec_cdl + ((size_t)c * d->rec_cap + first) * 3,
                       rows * 3 * sizeof(double), hipMemcpyDeviceToHost));
  }
  return 0;
}

/* compute_exp_data's sums (mcmc.c:53-58) over record rows [first, first + count) of every chain:
   ls = sum of -loglik, cs = sum of exp(c), ds = sum of exp(d), in row order.  One block per chain: the
   exps of a chunk of rows in parallel into LDS (sr_exp_m is glibc's exp bit for bit), then thread 0
   adds the chunk in row order (the reference's sequential sums).  Only 3 doubles per chain leave the
   GPU (the row data stay in HBM). */
#define SR_XD_CHUNK 1024
__global__ __launch_bounds__(256) void sr_exp_data_kernel(const double *rec_cdl, int rec_cap, int first, int count,
                                                          double *out)
{
  __shared__ double tabs[512];
  __shared__ double ce[SR_XD_CHUNK], de[SR_XD_CHUNK], le[SR_XD_CHUNK];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    ((uint64_t *)tabs)[i] = c_exp_tab[i];
    tabs[256 + i] = c_log_tab[i];
  }
  sr_mtab tb;
  tb.exp_tab = (const uint64_t *)tabs; tb.log_tab = tabs + 256;
  const int c = blockIdx.x;
  const double *r = rec_cdl + ((size_t)c * rec_cap + first) * 3;
  double ls = 0., cs = 0., ds = 0.;
  for (int t0 = 0; t0 < count; t0 += SR_XD_CHUNK) {
    const int n = min(SR_XD_CHUNK, count - t0);
    __syncthreads();   /* tables loaded / the previous chunk summed */
    for (int t = threadIdx.x; t < n; t += blockDim.x) {
      const double *rr = r + 3 * (size_t)(t0 + t);
      ce[t] = sr_exp_m(rr[0], &tb);
      de[t] = sr_exp_m(rr[1], &tb);
      le[t] = rr[2];
    }
    __syncthreads();
    if (threadIdx.x == 0)
      for (int t = 0; t < n; ++t) { ls += -(le[t]); cs += ce[t]; ds += de[t]; }
  }
  if (threadIdx.x == 0) { out[3 * c] = ls; out[3 * c + 1] = cs; out[3 * c + 2] = ds; }
}

extern "C" int srk_exp_data(srk_dev *d, int first, int count, double *sums)
{
  if (first < 0 || count < 0 || first + count > d->rec_cap) return -1;
  HIPCHK(hipSetDevice(d->device));
  if (!d->dsum) {
    void *p = nullptr;
    HIPCHK(hipMalloc(&p, (size_t)d->nchains * 3 * sizeof(double)));
    d->bufs[d->nbufs++] = p;
    d->dsum = (double *)p;
  }
  hipLaunchKernelGGL(sr_exp_data_kernel, dim3(d->nchains), dim3(256), 0, d->stream, d->args.rec_cdl, d->rec_cap, first, count,
                     d->dsum);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(sums, d->dsum, (size_t)d->nchains * 3 * sizeof(double), hipMemcpyDeviceToHost, d->stream));
  HIPCHK(hipStreamSynchronize(d->stream));
  return sp_check(d);
}

/* one chain's rows [first, first + count) of its record slab */
extern "C" int srk_fetch_chain_records(srk_dev *d, int chain, int first, int count, int16_t *ab_pi, double *cdl)
{
  if (chain < 0 || chain >= d->nchains || first < 0 || count < 0 || first + count > d->rec_cap) return -1;
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipStreamSynchronize(d->stream));
  if (int e = sp_check(d)) return e;
  if (count == 0) return 0;
  const size_t W = 2 * (size_t)d->M + d->N, row = (size_t)chain * d->rec_cap + first;
  if (ab_pi) HIPCHK(hipMemcpy(ab_pi, d->args.rec_abpi + row * W, (size_t)count * W * sizeof(int16_t), hipMemcpyDeviceToHost));
  if (cdl) HIPCHK(hipMemcpy(cdl, d->args.rec_cdl + row * 3, (size_t)count * 3 * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int srk_copy_chain_records(srk_dev *d, int chain, int first, int count, int16_t *ab_pi, double *cdl)
{
  if (chain < 0 || chain >= d->nchains || first < 0 || count < 0 || first + count > d->rec_cap) return -1;
  if (count == 0) return 0;
  HIPCHK(hipSetDevice(d->device));
  const size_t W = 2 * (size_t)d->M + d->N, row = (size_t)chain * d->rec_cap + first;
  if (ab_pi)
    HIPCHK(hipMemcpyAsync(ab_pi, d->args.rec_abpi + row * W, (size_t)count * W * sizeof(int16_t), hipMemcpyDeviceToDevice,
                          d->stream));
  if (cdl)
    HIPCHK(hipMemcpyAsync(cdl, d->args.rec_cdl + row * 3, (size_t)count * 3 * sizeof(double), hipMemcpyDeviceToDevice,
                          d->stream));
  return 0;
}

/* Sampling with the host work overlapped: launch j (k_j calls, records into half j&1 of the record
 * buffer) is followed on the stream by an async copy of its records into pinned host half j&1; the
 * host then waits only for launch j-1's copy and hands it to `consume` while launch j runs.  Needs
 * rec_cap >= 2 * cpl.  consume(ctx, first_call, count, ab_pi [nchains][count][2M+N], cdl
 * [nchains][count][3]) returns nonzero to stop. */
extern "C" int srk_run_pipelined(srk_dev *d, int total_calls, int cpl, int spc,
                                 int (*consume)(void *, int, int, const int16_t *, const double *, const double *), void *ctx)
{
  if (total_calls <= 0) return 0;
  if (cpl <= 0 || 2 * cpl > d->rec_cap) return -1;
  HIPCHK(hipSetDevice(d->device));
  const size_t W = 2 * (size_t)d->M + d->N, C = d->nchains;
  int16_t *hab[2] = {nullptr, nullptr};
  double *hcd[2] = {nullptr, nullptr};
  double *hcv[2] = {nullptr, nullptr};   /* manycd: per-taxon c, d rows */
  const size_t R2 = 2 * (size_t)d->M;
  hipEvent_t ev[2] = {nullptr, nullptr};
  int cnt[2] = {0, 0}, first[2] = {0, 0};
  int rc = 0;
  for (int h = 0; h < 2 && !rc; ++h) {
    if (hipHostMalloc((void **)&hab[h], C * cpl * W * sizeof(int16_t), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&hcd[h], C * cpl * 3 * sizeof(double), hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&ev[h], hipEventDisableTiming) != hipSuccess ||
        (d->mcd && hipHostMalloc((void **)&hcv[h], C * cpl * R2 * sizeof(double), hipHostMallocDefault) != hipSuccess))
      rc = -5;
  }
  int done = 0, j = 0;
  while (!rc && done < total_calls) {
    const int h = j & 1, k = (total_calls - done < cpl) ? total_calls - done : cpl;
    rc = srk_run(d, k, spc, 1, h * cpl);
    if (rc) break;
    /* strided: chain c's k records at [c][h*cpl .. h*cpl+k) -> pinned [c][0..k) */
    if (hipMemcpy2DAsync(hab[h], k * W * sizeof(int16_t), d->args.rec_abpi + (size_t)h * cpl * W,
                         d->rec_cap * W * sizeof(int16_t), k * W * sizeof(int16_t), C, hipMemcpyDeviceToHost,
                         d->stream) != hipSuccess ||
        hipMemcpy2DAsync(hcd[h], k * 3 * sizeof(double), d->args.rec_cdl + (size_t)h * cpl * 3,
                         d->rec_cap * 3 * sizeof(double), k * 3 * sizeof(double), C, hipMemcpyDeviceToHost,
                         d->stream) != hipSuccess ||
        (d->mcd && hipMemcpy2DAsync(hcv[h], k * R2 * sizeof(double), d->args.rec_cdv + (size_t)h * cpl * R2,
                                    d->rec_cap * R2 * sizeof(double), k * R2 * sizeof(double), C, hipMemcpyDeviceToHost,
                                    d->stream) != hipSuccess) ||
        hipEventRecord(ev[h], d->stream) != hipSuccess) { rc = -5; break; }
    cnt[h] = k; first[h] = done;
    if (j > 0) {   /* the previous launch's records, while this launch runs */
      const int p = h ^ 1;
      if (hipEventSynchronize(ev[p]) != hipSuccess) { rc = -5; break; }
      if (consume(ctx, first[p], cnt[p], hab[p], hcd[p], hcv[p])) { rc = -1; break; }
    }
    done += k;
    ++j;
  }
  if (!rc && j > 0) {
    const int p = (j - 1) & 1;
    if (hipEventSynchronize(ev[p]) != hipSuccess) rc = -5;
    else if (consume(ctx, first[p], cnt[p], hab[p], hcd[p], hcv[p])) rc = -1;
  }
  (void)hipStreamSynchronize(d->stream);
  if (!rc) rc = sp_check(d);
  for (int h = 0; h < 2; ++h) {
    if (hab[h]) (void)hipHostFree(hab[h]);
    if (hcd[h]) (void)hipHostFree(hcd[h]);
    if (hcv[h]) (void)hipHostFree(hcv[h]);
    if (ev[h]) (void)hipEventDestroy(ev[h]);
  }
  return rc;
}

extern "C" int srk_records_device(srk_dev *d, const int16_t **rec, int *rec_cap, int *device, void **stream)
{
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipStreamSynchronize(d->stream));
  if (int e = sp_check(d)) return e;
  *rec = d->args.rec_abpi;
  *rec_cap = d->rec_cap;
  *device = d->device;
  *stream = (void *)d->stream;
  return 0;
}

extern "C" int srk_download_state(srk_dev *d, sr_state_host *st)
{
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipStreamSynchronize(d->stream));
  if (int e = sp_check(d)) return e;
  const size_t C = d->nchains;
  const KArgs &A = d->args;
  if (st->P) HIPCHK(hipMemcpy(st->P, A.P, C * d->NW * d->M * 4, hipMemcpyDeviceToHost));
  if (st->rpi) HIPCHK(hipMemcpy(st->rpi, A.rpi, C * d->N * 4, hipMemcpyDeviceToHost));
  if (st->hp) HIPCHK(hipMemcpy(st->hp, A.hp, C * SR_NHCAP(d->nh) * 4, hipMemcpyDeviceToHost));
  if (st->ab) HIPCHK(hipMemcpy(st->ab, A.ab, C * 2 * d->M * 4, hipMemcpyDeviceToHost));
  if (st->cnt) HIPCHK(hipMemcpy(st->cnt, A.cnt, C * 4 * d->M * 4, hipMemcpyDeviceToHost));
  if (st->cdl) HIPCHK(hipMemcpy(st->cdl, A.cdl, C * 4 * 8, hipMemcpyDeviceToHost));
  if (st->mt) HIPCHK(hipMemcpy(st->mt, A.mt, C * SR_RING * SR_MT_N * 4, hipMemcpyDeviceToHost));
  if (st->rng) HIPCHK(hipMemcpy(st->rng, A.rng, C * 2 * 8, hipMemcpyDeviceToHost));
  if (st->acc) HIPCHK(hipMemcpy(st->acc, A.acc, C * SR_NACC * 8, hipMemcpyDeviceToHost));
  if (st->cdv && d->mcd) HIPCHK(hipMemcpy(st->cdv, A.cdv, C * 2 * d->M * 8, hipMemcpyDeviceToHost));
  return 0;
}

/* manycd: every chain's per-taxon c, d of record rows [first, first + count): cdv [nchains][count][2M] */
extern "C" int srk_fetch_cdv(srk_dev *d, int first, int count, double *cdv)
{
  if (!d->mcd || first < 0 || count < 0 || first + count > d->rec_cap) return -1;
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipStreamSynchronize(d->stream));
  if (count == 0) return 0;
  const size_t row = 2 * (size_t)d->M;
  HIPCHK(hipMemcpy2D(cdv, count * row * 8, d->args.rec_cdv + (size_t)first * row, d->rec_cap * row * 8, count * row * 8,
                     d->nchains, hipMemcpyDeviceToHost));
  return 0;
}

/* record rows [0, count) of every chain uploaded (a restored checkpoint's records: ab_pi [nchains][count][2M+N],
   cdl [nchains][count][3], manycd sessions' cdv [nchains][count][2M]) */
extern "C" int srk_upload_records(srk_dev *d, int count, const int16_t *ab_pi, const double *cdl, const double *cdv)
{
  if (count < 0 || count > d->rec_cap || (cdv && !d->mcd)) return -1;
  if (count == 0) return 0;
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipStreamSynchronize(d->stream));
  const size_t W = 2 * (size_t)d->M + d->N, R2 = 2 * (size_t)d->M;
  HIPCHK(hipMemcpy2D(d->args.rec_abpi, d->rec_cap * W * 2, ab_pi, count * W * 2, count * W * 2, d->nchains,
                     hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy2D(d->args.rec_cdl, d->rec_cap * 3 * 8, cdl, count * 3 * 8, count * 3 * 8, d->nchains,
                     hipMemcpyHostToDevice));
  if (cdv)
    HIPCHK(hipMemcpy2D(d->args.rec_cdv, d->rec_cap * R2 * 8, cdv, count * R2 * 8, count * R2 * 8, d->nchains,
                       hipMemcpyHostToDevice));
  return 0;
}

extern "C" void srk_destroy(srk_dev *d)
{
  if (!d) return;
  (void)hipSetDevice(d->device);
  if (d->stream) (void)hipStreamSynchronize(d->stream);
  for (int i = 0; i < d->nbufs; ++i) (void)hipFree(d->bufs[i]);
  if (d->have_events) { (void)hipEventDestroy(d->ev0); (void)hipEventDestroy(d->ev1); }
  if (d->own_stream && d->stream) (void)hipStreamDestroy(d->stream);
  if (d->mod) (void)hipModuleUnload(d->mod);
  delete d;
}

/* ================================================================ self-test hook */
/* Device copies of the deterministic exp/log, for the host<->device bit-parity test. */
__global__ void sr_math_selftest_kernel(const double *in, long n, double *oe, double *ol)
{
  __shared__ double tabs[512];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    ((uint64_t *)tabs)[i] = c_exp_tab[i];
    tabs[256 + i] = c_log_tab[i];
  }
  __syncthreads();
  sr_mtab tb;
  tb.exp_tab = (const uint64_t *)tabs; tb.log_tab = tabs + 256;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    oe[i] = sr_exp_m(in[i], &tb);
    ol[i] = sr_log_m(in[i], &tb);
  }
}

extern "C" __attribute__((visibility("default"))) int sr_device_selftest_math(int device, const double *in, long n,
                                                                             double *out_exp, double *out_log)
{
  if (n <= 0) return 0;
  HIPCHK(hipSetDevice(device));
  double *din = nullptr, *de = nullptr, *dl = nullptr;
  HIPCHK(hipMalloc(&din, n * 8));
  HIPCHK(hipMalloc(&de, n * 8));
  HIPCHK(hipMalloc(&dl, n * 8));
  HIPCHK(hipMemcpy(din, in, n * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(sr_math_selftest_kernel, dim3(1024), dim3(256), 0, 0, din, n, de, dl);
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out_exp, de, n * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(out_log, dl, n * 8, hipMemcpyDeviceToHost));
  (void)hipFree(din); (void)hipFree(de); (void)hipFree(dl);
  return 0;
}

/* ================================================================ certification self-tests (test hooks)
 * The bit-exactness of the sampler rests on two analytic error bounds that chain-level parity cannot probe
 * (a uniform u lands in the band where an understated bound would give a wrong answer about once in 1e13 draws):
 * the Gibbs picks' REL / ABS (draw_fast_s, draw_fast) and phase C's Eb (pc_classify / pc_resolve).  These hooks run
 * the product's own device functions on caller-chosen inputs -- u placed on and around the reference's exact CDF
 * boundaries, count sums whose reference delta sits at 0 or at log u -- and return what the function decided and
 * whether it fell back to the exact path (tests/test_gpu_cert.py checks every case against the oracle). */

/* One wave per block, one case per lane; block b's lanes share (c, d) = cd[2b], cd[2b + 1].  MODE 0 / 1:
 * draw_fast_s<9> / <17> (register walks, the LDS-column kernels up to N = 287 / 543), 2: draw_fast<false> (LDS
 * columns beyond), 3: draw_fast<true> (HBM columns: byte tables, grouped checkpoints, SR_QSPAN trims).  Case m: the
 * column's position-ordered bits P[w * M + m] (M = cases), its prefix table pre[w * M + m], walk direction rev[m]
 * (1: walk entry w = position N - 1 - w, the b-draw), current limit o[m] and walk end L[m] (entries 0..L), u[m].
 * out[5 m ..]: the pick and the count deltas dt0, df0, dt1, df1 at it; fb[m]: exact-walk fallbacks taken. */
template <int MODE>
__global__ void __launch_bounds__(64) sr_gibbs_selftest_kernel(const uint32_t *P, const uint16_t *pre, int N, int M,
                                                               const double *cd, const int *oo, const int *LL,
                                                               const int *rv, const double *uu, int *out,
                                                               unsigned long long *fb, double *cks)
{
  __shared__ double tabs[512];
  __shared__ double T4w[T4STRIDE];
  __shared__ double T8w[2 * 257];
  const int lane = threadIdx.x, m = blockIdx.x * 64 + lane;
  for (int i = lane; i < 256; i += 64) {
    ((uint64_t *)tabs)[i] = c_exp_tab[i];
    tabs[256 + i] = c_log_tab[i];
  }
  __syncthreads();
  sr_mtab tb;
  tb.exp_tab = (const uint64_t *)tabs; tb.log_tab = tabs + 256;
  CD K;   /* as the sweep kernel's phase A */
  K.c = cd[2 * blockIdx.x]; K.d = cd[2 * blockIdx.x + 1];
  K.cc = sr_log_m(1. - sr_exp_m(K.c, &tb), &tb);
  K.dd = sr_log_m(1. - sr_exp_m(K.d, &tb), &tb);
  K.ec = sr_exp_m(SR_LOGEPSILON, &tb);
  const double vA = (K.d - K.cc) * 1.4426950408889634;
  const double vB = (K.dd - K.c) * 1.4426950408889634;
  const double rA = sr_exp_m(K.cc - K.d, &tb), rB = sr_exp_m(K.c - K.dd, &tb);
  if (lane < 16) {
    double sc[5];
    const double pr = t4_row(lane, rA, rB, sc);
#pragma unroll
    for (int c = 0; c < 5; ++c) { T4w[2 * (c * 16 + lane)] = sc[c]; T4w[2 * (c * 16 + lane) + 1] = pr; }
  }
  for (int q = 0; q < 4; ++q) *reinterpret_cast<double2 *>(T8w + 2 * (lane + 64 * q)) = t8_entry(lane + 64 * q, rA, rB);
  if (lane == 0) *reinterpret_cast<double2 *>(T8w + 2 * 256) = make_double2(0.0, 1.0);
  __syncthreads();
  const int NW = (N + 31) >> 5;
  const uint32_t *Pm = P + m;
  const uint16_t *prem = pre + m;
  const int o = oo[m], L = LL[m];
  const bool rev = rv[m] != 0;
  const double u = uu[m];
  const int POo = rev ? (int)prem[NW * M] - col_pre(prem, Pm, M, N - o) : col_pre(prem, Pm, M, o);
  int d0 = 0, e0 = 0, d1 = 0, e1 = 0, res;
  if constexpr (MODE <= 1) {
    constexpr int NWM = MODE == 0 ? 9 : 17;
    uint32_t wk[NWM];
    load_fwd<NWM>(Pm, M, NW, wk);
    if (rev) {
      uint32_t rw[NWM];
      make_rev<NWM>(Pm, M, N, NW, wk, rw);
#pragma unroll
      for (int k = 0; k < NWM; ++k) wk[k] = rw[k];
    }
    res = draw_fast_s<NWM>(wk, Pm, M, N, rev, o, L, POo, u, K, tb, vA, vB, T4w, T8w, (uint64_t *)(fb + m), d0, e0, d1, e1);
  } else {
    res = draw_fast<MODE == 3>(Pm, prem, M, N, NW, rev, o, L, POo, u, K, tb, vA, vB, rA, rB, T4w, T8w, cks + m, M, 0,
                               (uint64_t *)(fb + m), d0, e0, d1, e1);
  }
  int *r = out + 5 * m;
  r[0] = res; r[1] = d0; r[2] = e0; r[3] = d1; r[4] = e1;
}

/* Phase C's decision per case: sums[4 m ..] = X0, X1, Y0, Y1 of one proposal (the exact integer sums of dt0, dt1
 * and of |dt0| + |dt1| over the taxa: Y0 = Y1 = Y as the one-workgroup kernels store them), cd[2 m ..] = c, d, uw[m]
 * the proposal's uniform_pos word.  out[m]: 0 rejected (u drawn), 1 accepted without drawing u (delta >= 0), 2
 * accepted with u drawn, 3 the exact sequential delta must decide (the sampler's fallback). */
__global__ void __launch_bounds__(64) sr_decide_selftest_kernel(const int *sums, const double *cd, const uint32_t *uw,
                                                                int n, int *out)
{
  __shared__ double tabs[512];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    ((uint64_t *)tabs)[i] = c_exp_tab[i];
    tabs[256 + i] = c_log_tab[i];
  }
  __syncthreads();
  sr_mtab tb;
  tb.exp_tab = (const uint64_t *)tabs; tb.log_tab = tabs + 256;
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  CD K;
  K.c = cd[2 * m]; K.d = cd[2 * m + 1];
  K.cc = sr_log_m(1. - sr_exp_m(K.c, &tb), &tb);
  K.dd = sr_log_m(1. - sr_exp_m(K.d, &tb), &tb);
  K.ec = 0.0;
  const double aC = __builtin_fabs(K.cc) + __builtin_fabs(K.d), aD = __builtin_fabs(K.dd) + __builtin_fabs(K.c);
  double Sp, Ebp;
  int Knz;
  const int cls = pc_classify(sums[4 * m], sums[4 * m + 1], sums[4 * m + 2], sums[4 * m + 3], K, aC, aD, false, uw[m], Sp,
                              Ebp, Knz);
  int res = 0;
  if (cls != 0) {
    bool accept, udrawn = false, have_exact;
    double dl;
    const double u = (double)uw[m] / 4294967296.0;
    if (!pc_resolve(Sp, Ebp, cls, Knz, u, tb, accept, udrawn, have_exact, dl)) res = 3;
    else res = accept ? (udrawn ? 2 : 1) : 0;
  }
  out[m] = res;
}

/* Host entry points of the self-tests (negative codes: -1 bad arguments, -2 device error).  ncases must be a
 * multiple of 64; P is [NW][ncases] u32, pre [NW + 1][ncases] u16, cd [ncases / 64][2]. */
extern "C" __attribute__((visibility("default"))) int sr_device_selftest_gibbs(int device, int mode, int N, int ncases,
                                                                              const uint32_t *P, const uint16_t *pre,
                                                                              const double *cd, const int *o, const int *L,
                                                                              const int *rev, const double *u, int *out,
                                                                              unsigned long long *fb)
{
  const int NW = (N + 31) >> 5;
  if (ncases <= 0 || ncases % 64 || N < 1 || N > 4095 || mode < 0 || mode > 3 || (mode == 0 && NW > 9) ||
      (mode == 1 && NW > 17))
    return -1;
  for (int m = 0; m < ncases; ++m)
    if (o[m] < 0 || o[m] > L[m] || L[m] > N) return -1;
  HIPCHK(hipSetDevice(device));
  const size_t C = (size_t)ncases;
  void *b[11] = {};
  const size_t sz[11] = {NW * C * 4, (NW + 1) * C * 2, C / 64 * 2 * 8, C * 4, C * 4, C * 4, C * 8, C * 5 * 4, C * 8,
                         (NW + 2) * C * 8, 0};
  int rc = 0;
  for (int k = 0; k < 10 && !rc; ++k) rc = hipMalloc(&b[k], sz[k]) != hipSuccess;
  const void *src[7] = {P, pre, cd, o, L, rev, u};
  for (int k = 0; k < 7 && !rc; ++k) rc = hipMemcpy(b[k], src[k], sz[k], hipMemcpyHostToDevice) != hipSuccess;
  if (!rc) rc = hipMemset(b[8], 0, sz[8]) != hipSuccess;
  if (!rc) {
    const dim3 g(ncases / 64), t(64);
    const uint32_t *dP = (const uint32_t *)b[0];
    const uint16_t *dpre = (const uint16_t *)b[1];
    const double *dcd = (const double *)b[2], *du = (const double *)b[6];
    const int *dO = (const int *)b[3], *dL = (const int *)b[4], *dR = (const int *)b[5];
    int *dout = (int *)b[7];
    unsigned long long *dfb = (unsigned long long *)b[8];
    double *dck = (double *)b[9];
    if (mode == 0) hipLaunchKernelGGL(sr_gibbs_selftest_kernel<0>, g, t, 0, 0, dP, dpre, N, ncases, dcd, dO, dL, dR, du, dout, dfb, dck);
    else if (mode == 1) hipLaunchKernelGGL(sr_gibbs_selftest_kernel<1>, g, t, 0, 0, dP, dpre, N, ncases, dcd, dO, dL, dR, du, dout, dfb, dck);
    else if (mode == 2) hipLaunchKernelGGL(sr_gibbs_selftest_kernel<2>, g, t, 0, 0, dP, dpre, N, ncases, dcd, dO, dL, dR, du, dout, dfb, dck);
    else hipLaunchKernelGGL(sr_gibbs_selftest_kernel<3>, g, t, 0, 0, dP, dpre, N, ncases, dcd, dO, dL, dR, du, dout, dfb, dck);
    rc = hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess;
  }
  if (!rc) rc = hipMemcpy(out, b[7], sz[7], hipMemcpyDeviceToHost) != hipSuccess;
  if (!rc) rc = hipMemcpy(fb, b[8], sz[8], hipMemcpyDeviceToHost) != hipSuccess;
  for (int k = 0; k < 10; ++k) (void)hipFree(b[k]);
  return rc ? -2 : 0;
}

extern "C" __attribute__((visibility("default"))) int sr_device_selftest_decide(int device, int ncases, const int *sums,
                                                                               const double *cd, const uint32_t *uw,
                                                                               int *out)
{
  if (ncases <= 0) return -1;
  HIPCHK(hipSetDevice(device));
  const size_t C = (size_t)ncases;
  void *b[4] = {};
  const size_t sz[4] = {C * 16, C * 16, C * 4, C * 4};
  int rc = 0;
  for (int k = 0; k < 4 && !rc; ++k) rc = hipMalloc(&b[k], sz[k]) != hipSuccess;
  const void *src[3] = {sums, cd, uw};
  for (int k = 0; k < 3 && !rc; ++k) rc = hipMemcpy(b[k], src[k], sz[k], hipMemcpyHostToDevice) != hipSuccess;
  if (!rc) {
    hipLaunchKernelGGL(sr_decide_selftest_kernel, dim3((ncases + 63) / 64), dim3(64), 0, 0, (const int *)b[0],
                       (const double *)b[1], (const uint32_t *)b[2], ncases, (int *)b[3]);
    rc = hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess;
  }
  if (!rc) rc = hipMemcpy(out, b[3], sz[3], hipMemcpyDeviceToHost) != hipSuccess;
  for (int k = 0; k < 4; ++k) (void)hipFree(b[k]);
  return rc ? -2 : 0;
}
#endif   /* !SR_JIT */
