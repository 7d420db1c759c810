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
#define SR_TABLES_NO_ARRAYS
#include "sr_tables.h"
#include "sr_math.h"
#include "sr_rng.h"
#include "sr_internal.h"

__constant__ double c_zig_y[128] = SR_ZIG_YTAB_INIT;
__constant__ unsigned int c_zig_k[128] = SR_ZIG_KTAB_INIT;
__constant__ double c_zig_w[128] = SR_ZIG_WTAB_INIT;
__constant__ double c_exp_thi[128] = SR_EXP_THI_INIT;
__constant__ double c_exp_tlo[128] = SR_EXP_TLO_INIT;
__constant__ double c_log_invc[128] = SR_LOG_INVC_INIT;
__constant__ double c_log_lhi[128] = SR_LOG_LHI_INIT;
__constant__ double c_log_llo[128] = SR_LOG_LLO_INIT;

#define SR_ZIGR 3.44428647676

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
};

/* ---------------------------------------------------------------- LDS carve */
struct Lay {
  size_t tab, tbuf, lbuf, mt, P, rpi0, rpi1, nhpos, misc, total;
};
__host__ __device__ static inline size_t sr_al16(size_t x) { return (x + 15) & ~(size_t)15; }
__host__ __device__ static inline Lay sr_layout(int N, int M, int NW)
{
  Lay L;
  size_t o = 0;
  L.tab = o;   o = sr_al16(o + 640 * sizeof(double));
  L.tbuf = o;  o = sr_al16(o + (size_t)M * sizeof(double));
  L.lbuf = o;  o = sr_al16(o + (size_t)M * sizeof(double));
  L.mt = o;    o = sr_al16(o + (size_t)SR_RING * SR_MT_N * 4);
  L.P = o;     o = sr_al16(o + (size_t)NW * M * 4);
  L.rpi0 = o;  o = sr_al16(o + (size_t)N * 4);
  L.rpi1 = o;  o = sr_al16(o + (size_t)N * 4);
  L.nhpos = o; o = sr_al16(o + (size_t)N * 4);
  L.misc = o;  o = sr_al16(o + 64 * 8);
  L.total = o;
  return L;
}
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

/* ---------------------------------------------------------------- RNG */
struct DRng {
  uint32_t *ring;   /* LDS, SR_RING blocks of 624 raw words */
  uint32_t blk, off, gen;   /* next word = block blk, index off; blocks [.., gen) exist */
};

template <bool WAVE>
__device__ __noinline__ void rng_gen(DRng &r, int t, int nthr)
{
  const uint32_t *prev = r.ring + ((r.gen - 1) & (SR_RING - 1)) * SR_MT_N;
  uint32_t *nxt = r.ring + (r.gen & (SR_RING - 1)) * SR_MT_N;
  for (int k = t; k < 227; k += nthr) nxt[k] = sr_mt_mix(prev[k], prev[k + 1], prev[k + 397]);
  gsync<WAVE>();
  for (int k = 227 + t; k < 454; k += nthr) nxt[k] = sr_mt_mix(prev[k], prev[k + 1], nxt[k - 227]);
  gsync<WAVE>();
  for (int k = 454 + t; k < 624; k += nthr)
    nxt[k] = (k < 623) ? sr_mt_mix(prev[k], prev[k + 1], nxt[k - 227]) : sr_mt_mix(prev[623], nxt[0], nxt[396]);
  gsync<WAVE>();
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

/* ------------------------------------------------ GSL beta/gamma/ziggurat (wave 0) */
__device__ double d_gauss_zig(DRng &r, int lane, const sr_mtab &tb)
{
  for (;;) {
    uint32_t k = rng_get<true>(r, lane, 64);
    uint32_t i = k & 0xFF;
    uint32_t j = (k >> 8) & 0xFFFFFF;
    int sign = (i & 0x80) ? +1 : -1;
    i &= 0x7f;
    double x = j * c_zig_w[i];
    if (j < c_zig_k[i]) return sign * 1.0 * x;
    double y;
    if (i < 127) {
      double y0 = c_zig_y[i], y1 = c_zig_y[i + 1];
      double U1 = rng_uniform<true>(r, lane, 64);
      y = y1 + (y0 - y1) * U1;
    } else {
      double U1 = 1.0 - rng_uniform<true>(r, lane, 64);
      double U2 = rng_uniform<true>(r, lane, 64);
      x = SR_ZIGR - sr_log_m(U1, &tb) / SR_ZIGR;
      y = sr_exp_m(-SR_ZIGR * (x - 0.5 * SR_ZIGR), &tb) * U2;
    }
    if (y < sr_exp_m(-0.5 * x * x, &tb)) return sign * 1.0 * x;
  }
}

__device__ double d_gamma(DRng &r, double a, int lane, const sr_mtab &tb)
{
  double boost = 1.0;
  if (a < 1) { /* unreachable from the sampler (a = 1 + count); kept for GSL parity */
    double u = rng_uniform_pos<true>(r, lane, 64);
    boost = sr_exp_m(sr_log_m(u, &tb) * (1.0 / a), &tb);
    a = 1.0 + a;
  }
  double x, v, u;
  double d = a - 1.0 / 3.0;
  double c = (1.0 / 3.0) / __builtin_sqrt(d);
  for (;;) {
    do {
      x = d_gauss_zig(r, lane, tb);
      v = 1.0 + c * x;
    } while (v <= 0);
    v = v * v * v;
    u = rng_uniform_pos<true>(r, lane, 64);
    if (u < 1 - 0.0331 * x * x * x * x) break;
    if (sr_log_m(u, &tb) < 0.5 * x * x + d * (1 - v + sr_log_m(v, &tb))) break;
  }
  double g = 1.0 * d * v;
  return (boost == 1.0) ? g : g * boost;
}

/* mcmc_samplebeta: y = beta(1+a, 1+b); keep the old value unless log y in [low, high] */
__device__ double d_samplebeta(DRng &r, double x, double a, double b, double low, double high, int lane,
                               const sr_mtab &tb)
{
  double x1 = d_gamma(r, 1. + a, lane, tb);
  double x2 = d_gamma(r, 1. + b, lane, tb);
  double y = x1 / (x1 + x2);
  if (y > 0.) {
    y = sr_log_m(y, &tb);
    if (low <= y && y <= high) x = y;
  }
  return x;
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
 * entries w = 0..L.  Returns the picked entry and the count deltas dt0,df0,dt1,df1 there. */
__device__ int draw_limit(const uint32_t *Pm, int M, int N, bool rev, int o, int L, double u, const CD &k,
                          const sr_mtab &tb, int &dt0, int &df0, int &dt1, int &df1)
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
  /* count deltas at the pick (the dt arrays of mcmc_auxa) */
  const int POp = wprefix(res);
  if (res == o) { dt0 = df0 = dt1 = df1 = 0; }
  else if (res < o) { int O = POo - POp; int Z = (o - res) - O; dt0 = -Z; df0 = Z; dt1 = O; df1 = -O; }
  else { int O = POp - POo; int Z = (res - o) - O; dt0 = Z; df0 = -Z; dt1 = -O; df1 = O; }
  return res;
}

__device__ __forceinline__ int ininterval(int i, int a, int b, int inc1, int inc2)
{
  int r;
  if (a > b) { r = a; a = b; b = r; }
  r = inc1 ? (a <= i) : (a < i);
  if (r) r = inc2 ? (i <= b) : (i < b);
  return r;
}

__device__ __forceinline__ int hard_count(const int *hp, int nh, int lo, int hi)
{
  int s = 0;
#pragma unroll
  for (int k = 0; k < SR_NHMAX; ++k) s += (k < nh && hp[k] >= lo && hp[k] <= hi) ? 1 : 0;
  return s;
}

__device__ __forceinline__ bool is_hard(const int *hp, int nh, int p)
{
  bool h = false;
#pragma unroll
  for (int k = 0; k < SR_NHMAX; ++k) h |= (k < nh && hp[k] == p);
  return h;
}

/* sequential sum of tbuf[0..M) in ascending m, skipping +-0 terms (exact: s never
 * becomes -0.0), on wave 0; result broadcast.  Two barriers. */
__device__ __forceinline__ double ordered_sum(const double *buf, int M, double *slot, int tid)
{
  __syncthreads();
  if (tid < 64) {
    double s = 0.0;
    for (int base = 0; base < M; base += 64) {
      int m = base + tid;
      double t = (m < M) ? buf[m] : 0.0;
      uint64_t mask = __ballot(t != 0.0);
      uint64_t tb = __builtin_bit_cast(uint64_t, t);
      int tlo = (int)(uint32_t)tb, thi = (int)(uint32_t)(tb >> 32);
      while (mask) {
        int l = __builtin_ctzll(mask);
        mask &= mask - 1;
        uint32_t a = (uint32_t)__builtin_amdgcn_readlane(tlo, l);
        uint32_t b = (uint32_t)__builtin_amdgcn_readlane(thi, l);
        s = s + __builtin_bit_cast(double, ((uint64_t)b << 32) | a);
      }
    }
    if (tid == 0) *slot = s;
  }
  __syncthreads();
  return *slot;
}

/* ---------------------------------------------------------------- kernel */
template <int TB, int TPT>
__global__ __launch_bounds__(TB) void sr_sweep_kernel(KArgs A)
{
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int chain = blockIdx.x;
  const int N = A.N, M = A.M, NW = A.NW, nh = A.nh;
  const Lay L = sr_layout(N, M, NW);
  double *tabs = (double *)(smem + L.tab);
  double *tbuf = (double *)(smem + L.tbuf);
  double *lbuf = (double *)(smem + L.lbuf);
  uint32_t *ring = (uint32_t *)(smem + L.mt);
  uint32_t *P = (uint32_t *)(smem + L.P);
  int32_t *rpiA = (int32_t *)(smem + L.rpi0);
  int32_t *rpiB = (int32_t *)(smem + L.rpi1);
  int32_t *nhpos = (int32_t *)(smem + L.nhpos);
  uint64_t *misc = (uint64_t *)(smem + L.misc);
  int *tot = (int *)(misc + MS_TOT);
  double *dslot = (double *)(misc + MS_DELTA);

  /* ---- load tables and state */
  for (int i = tid; i < 128; i += TB) {
    tabs[i] = c_exp_thi[i];
    tabs[128 + i] = c_exp_tlo[i];
    tabs[256 + i] = c_log_invc[i];
    tabs[384 + i] = c_log_lhi[i];
    tabs[512 + i] = c_log_llo[i];
  }
  sr_mtab tb;
  tb.exp_thi = tabs; tb.exp_tlo = tabs + 128; tb.log_invc = tabs + 256; tb.log_lhi = tabs + 384; tb.log_llo = tabs + 512;

  const uint32_t *gP = A.P + (size_t)chain * NW * M;
  for (int i = tid; i < NW * M; i += TB) P[i] = gP[i];
  const int32_t *grpi = A.rpi + (size_t)chain * N;
  for (int i = tid; i < N; i += TB) rpiA[i] = grpi[i];
  const uint32_t *gmt = A.mt + (size_t)chain * SR_RING * SR_MT_N;
  for (int i = tid; i < SR_RING * SR_MT_N; i += TB) ring[i] = gmt[i];
  if (tid < 4) tot[tid] = 0;
  if (tid == 0) misc[MS_CAB] = 0;

  int hp[SR_NHMAX];
#pragma unroll
  for (int k = 0; k < SR_NHMAX; ++k) hp[k] = (k < nh) ? A.hp[(size_t)chain * SR_NHMAX + k] : -1;

  int a_[TPT], b_[TPT], t0_[TPT], f0_[TPT], t1_[TPT], f1_[TPT];
#pragma unroll
  for (int k = 0; k < TPT; ++k) {
    int m = tid + k * TB;
    if (m < M) {
      a_[k] = A.ab[(size_t)chain * 2 * M + m];
      b_[k] = A.ab[(size_t)chain * 2 * M + M + m];
      t0_[k] = A.cnt[(size_t)chain * 4 * M + m];
      f0_[k] = A.cnt[(size_t)chain * 4 * M + M + m];
      t1_[k] = A.cnt[(size_t)chain * 4 * M + 2 * M + m];
      f1_[k] = A.cnt[(size_t)chain * 4 * M + 3 * M + m];
    } else {
      a_[k] = b_[k] = t0_[k] = f0_[k] = t1_[k] = f1_[k] = 0;
    }
  }
  double c = A.cdl[(size_t)chain * 4 + 0];
  double d = A.cdl[(size_t)chain * 4 + 1];
  double loglik = A.cdl[(size_t)chain * 4 + 2];   /* meaningful in wave 0 */
  DRng R;
  R.ring = ring;
  {
    uint64_t pos = A.rng[(size_t)chain * 2 + 0];
    uint64_t gen = A.rng[(size_t)chain * 2 + 1];
    R.blk = (uint32_t)(pos / SR_MT_N);
    R.off = (uint32_t)(pos % SR_MT_N);
    R.gen = (uint32_t)gen;
  }
  unsigned long long acc[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) acc[k] = 0;
  int rcur = 0;   /* which rpi buffer is current */
  __syncthreads();

  const double ec = sr_exp_m(SR_LOGEPSILON, &tb);
  const uint32_t nhard = (uint32_t)nh;

  for (int call = 0; call < A.calls; ++call) {
    for (int sw = 0; sw < A.spc; ++sw) {
      const bool want_logl = (sw == A.spc - 1);
      /* ---------------- totals for samplec/sampled (mcmc.c:977-984 / count01) */
      {
        int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
        for (int k = 0; k < TPT; ++k)
          if (tid + k * TB < M) { s0 += t0_[k]; s1 += f0_[k]; s2 += t1_[k]; s3 += f1_[k]; }
        for (int off = 32; off > 0; off >>= 1) {
          s0 += __shfl_xor(s0, off); s1 += __shfl_xor(s1, off);
          s2 += __shfl_xor(s2, off); s3 += __shfl_xor(s3, off);
        }
        if ((tid & 63) == 0) {
          atomicAdd(&tot[0], s0); atomicAdd(&tot[1], s1);
          atomicAdd(&tot[2], s2); atomicAdd(&tot[3], s3);
        }
      }
      rng_ensure(R, 128, tid, TB);
      __syncthreads();
      /* ---------------- c, d (wave 0) */
      if (tid < 64) {
        const int t0a = tot[0], f0a = tot[1], t1a = tot[2], f1a = tot[3];
        double nc = d_samplebeta(R, c, (double)f1a, (double)t0a, SR_MINC, SR_MAXC, tid, tb);
        double nd = d_samplebeta(R, d, (double)f0a, (double)t1a, SR_MIND, SR_MAXD, tid, tb);
        if (tid == 0) {
          ((double *)misc)[MS_C] = nc;
          ((double *)misc)[MS_D] = nd;
          ((double *)misc)[MS_CC] = sr_log_m(1. - sr_exp_m(nc, &tb), &tb);
          ((double *)misc)[MS_DD] = sr_log_m(1. - sr_exp_m(nd, &tb), &tb);
          misc[MS_BLK] = R.blk; misc[MS_OFF] = R.off; misc[MS_GEN] = R.gen;
          tot[0] = tot[1] = tot[2] = tot[3] = 0;
        }
      }
      __syncthreads();
      c = ((double *)misc)[MS_C];
      d = ((double *)misc)[MS_D];
      CD K;
      K.c = c; K.d = d;
      K.cc = ((double *)misc)[MS_CC];
      K.dd = ((double *)misc)[MS_DD];
      K.ec = ec;
      R.blk = (uint32_t)misc[MS_BLK]; R.off = (uint32_t)misc[MS_OFF]; R.gen = (uint32_t)misc[MS_GEN];
      if (tid == 0) { acc[0]++; acc[1]++; }

      /* ---------------- (a, b) Gibbs update (mcmc_sampleab) */
      rng_ensure(R, 2 * M, tid, TB);
      {
        unsigned long long nchg = 0;
#pragma unroll
        for (int k = 0; k < TPT; ++k) {
          const int m = tid + k * TB;
          if (m < M) {
            const uint32_t *Pm = P + m;
            const double ua = rng_peek(R, 2 * m) / 4294967296.0;
            const double ub = rng_peek(R, 2 * m + 1) / 4294967296.0;
            int d0, e0, d1, e1;
            int na = draw_limit(Pm, M, N, false, a_[k], b_[k], ua, K, tb, d0, e0, d1, e1);
            t0_[k] += d0; f0_[k] += e0; t1_[k] += d1; f1_[k] += e1;
            nchg += (na != a_[k]);
            a_[k] = na;
            int t = draw_limit(Pm, M, N, true, N - b_[k], N - na, ub, K, tb, d0, e0, d1, e1);
            t0_[k] += d0; f0_[k] += e0; t1_[k] += d1; f1_[k] += e1;
            int nb = N - t;
            nchg += (nb != b_[k]);
            b_[k] = nb;
            if (want_logl)
              lbuf[m] = (double)t0_[k] * K.cc + (double)f0_[k] * K.d + (double)t1_[k] * K.dd + (double)f1_[k] * K.c;
          }
        }
        for (int off = 32; off > 0; off >>= 1) nchg += __shfl_xor(nchg, off);
        if ((tid & 63) == 0 && nchg) atomicAdd((unsigned long long *)&misc[MS_CAB], nchg);
      }
      rng_skip(R, 2 * M);
      if (want_logl) {
        __syncthreads();
        if (tid < 64) {
          double s = 0.0;
          for (int base = 0; base < M; base += 64) {
            int m = base + tid;
            double t = (m < M) ? lbuf[m] : 0.0;
            uint64_t tbits = __builtin_bit_cast(uint64_t, t);
            int tlo = (int)(uint32_t)tbits, thi = (int)(uint32_t)(tbits >> 32);
            int cnt = min(64, M - base);
            for (int l = 0; l < cnt; ++l) {
              uint32_t lo32 = (uint32_t)__builtin_amdgcn_readlane(tlo, l);
              uint32_t hi32 = (uint32_t)__builtin_amdgcn_readlane(thi, l);
              s = s + __builtin_bit_cast(double, ((uint64_t)hi32 << 32) | lo32);
            }
          }
          loglik = s;
        }
      }

      /* ---------------- permutation proposals */
      for (int pr = 0; pr < 16; ++pr) {
        /* order: pi2(swap), then 5 x (pi1, pi2, pi3) (mcmc.c:237-243) */
        const int kind = (pr == 0) ? 21 : ((pr - 1) % 3 == 0 ? 1 : ((pr - 1) % 3 == 1 ? 20 : 3));
        int i, j, inc1 = 0, inc2 = 0, ii = 0, jj = 0, Kn = 0;
        bool veto = false;
        if (kind == 1) {
          i = (int)rng_uniform_int<false>(R, (uint32_t)N, tid, TB);
          j = (int)rng_uniform_int<false>(R, (uint32_t)(N - 1), tid, TB);
          if (j >= i) j++;
          ii = min(i, j); jj = max(i, j);
          if (is_hard(hp, nh, i) && hard_count(hp, nh, ii, jj) > 1) veto = true;
        } else if (kind == 20 || kind == 21) {
          if (kind == 20) {
            i = (int)rng_uniform_int<false>(R, (uint32_t)N, tid, TB);
            j = (int)rng_uniform_int<false>(R, (uint32_t)(N - 1), tid, TB);
            if (j >= i) j++;
            else { int t = i; i = j; j = t; }
          } else {
            i = (int)rng_uniform_int<false>(R, (uint32_t)(N - 1), tid, TB);
            j = i + 1;
          }
          if (hard_count(hp, nh, i, j) > 1) veto = true;
          if (!veto) {
            inc1 = (int)rng_uniform_int<false>(R, 2u, tid, TB);
            inc2 = (int)rng_uniform_int<false>(R, 2u, tid, TB);
          }
        } else {
          if ((uint32_t)N - nhard < 2) { veto = true; i = j = 0; }
          else {
            int n0 = (int)rng_uniform_int<false>(R, (uint32_t)N - nhard, tid, TB);
            int m0 = (int)rng_uniform_int<false>(R, (uint32_t)N - nhard - 1, tid, TB);
            if (n0 <= m0) { i = n0; j = m0 + 1; } else { i = m0; j = n0; }
            /* rank -> position (mcmc.c:1518-1533), hard positions ascending */
#pragma unroll
            for (int k = 0; k < SR_NHMAX; ++k) {
              if (k < nh) {
                if (hp[k] <= i) { i++; j++; }
                else if (hp[k] <= j) j++;
              }
            }
            inc1 = (int)rng_uniform_int<false>(R, 2u, tid, TB);
            inc2 = (int)rng_uniform_int<false>(R, 2u, tid, TB);
            Kn = (j - i + 1) - hard_count(hp, nh, i, j);
            /* non-hard positions of [i, j] in order: nhpos[rank] (barrier: a previous
               pi3's apply phase may still read nhpos when pi1/pi2 in between were vetoed) */
            __syncthreads();
            for (int n = i + tid; n <= j; n += TB) {
              if (!is_hard(hp, nh, n)) nhpos[(n - i) - hard_count(hp, nh, i, n - 1)] = n;
            }
            __syncthreads();
          }
        }
        if (veto) continue;

        /* ---- per-taxon count changes and terms */
        int dt0v[TPT], df0v[TPT], dt1v[TPT], df1v[TPT];
#pragma unroll
        for (int k = 0; k < TPT; ++k) {
          const int m = tid + k * TB;
          int dt0 = 0, df0 = 0, dt1 = 0, df1 = 0;
          if (m < M) {
            const uint32_t *Pm = P + m;
            const int a = a_[k], b = b_[k];
            if (kind == 1) {
              int ain, bin;
              const int v = colbit(Pm, M, i);
              if (i < j) {
                ain = (ii < a && a <= jj + 1);
                bin = (ii < b && b <= jj + 1);
                if (ain && !bin) { if (v) { dt1++; df1--; } else { dt0--; df0++; } }
                else if (!ain && bin) { if (v) { dt1--; df1++; } else { dt0++; df0--; } }
              } else {
                ain = (ii <= a && a <= jj);
                bin = (ii <= b && b <= jj);
                if (!ain && bin) { if (v) { dt1++; df1--; } else { dt0--; df0++; } }
                else if (ain && !bin) { if (v) { dt1--; df1++; } else { dt0++; df0--; } }
              }
            } else if (kind != 3) {
              const int ain = ininterval(a, i, j + 1, inc1, inc2);
              const int bin = ininterval(b, i, j + 1, inc1, inc2);
              if (ain && !bin) {
                int O1 = ones_range(Pm, M, i, a), Z1 = (a - i) - O1;
                int O2 = ones_range(Pm, M, a, j + 1), Z2 = (j + 1 - a) - O2;
                dt1 = O1 - O2; df1 = -O1 + O2; dt0 = -Z1 + Z2; df0 = Z1 - Z2;
              } else if (!ain && bin) {
                int O1 = ones_range(Pm, M, i, b), Z1 = (b - i) - O1;
                int O2 = ones_range(Pm, M, b, j + 1), Z2 = (j + 1 - b) - O2;
                dt1 = -O1 + O2; df1 = O1 - O2; dt0 = Z1 - Z2; df0 = -Z1 + Z2;
              }
            } else {
              const int ain = ininterval(a, i, j + 1, inc1, inc2);
              const int bin = ininterval(b, i, j + 1, inc1, inc2);
              int na, nb;
              if (ain && !bin) { na = i + j + 1 - a; nb = b; }
              else if (!ain && bin) { na = a; nb = i + j + 1 - b; }
              else if (ain && bin) { na = i + j + 1 - b; nb = i + j + 1 - a; }
              else { na = a; nb = b; }
              for (int r = 0; r < Kn; ++r) {
                const int n = nhpos[r], nn = nhpos[Kn - 1 - r];
                const int was = (a <= n && n < b), is = (na <= nn && nn < nb);
                if (was != is) {
                  const int v = colbit(Pm, M, n);
                  if (was) { if (v) { dt1--; df1++; } else { df0--; dt0++; } }
                  else { if (v) { dt1++; df1--; } else { df0++; dt0--; } }
                }
              }
#pragma unroll
              for (int q = 0; q < SR_NHMAX; ++q) {
                const int n = hp[q];
                if (q < nh && n >= i && n <= j) {
                  const int was = (a <= n && n < b), is = (na <= n && n < nb);
                  if (was != is) {
                    const int v = colbit(Pm, M, n);
                    if (was) { if (v) { dt1--; df1++; } else { df0--; dt0++; } }
                    else { if (v) { dt1++; df1--; } else { df0++; dt0--; } }
                  }
                }
              }
            }
            tbuf[m] = qval(dt0, df0, dt1, df1, K);
          }
          dt0v[k] = dt0; df0v[k] = df0; dt1v[k] = dt1; df1v[k] = df1;
        }
        const double delta = ordered_sum(tbuf, M, dslot, tid);
        /* ---- MH accept (mcmc.c:1261 / 1441 / 1636): uniform_pos only when delta < 0 */
        bool accept = (delta >= 0.);
        if (!accept) accept = delta > sr_log_m(rng_uniform_pos<false>(R, tid, TB), &tb);
        if (!accept) continue;
        if (tid == 0) acc[kind == 1 ? 3 : kind == 20 ? 4 : kind == 21 ? 5 : 6]++;
        if (tid < 64) loglik += delta;
        /* ---- apply: limits, counts, columns */
        const int32_t *ro = rcur ? rpiB : rpiA;
        int32_t *rn = rcur ? rpiA : rpiB;
#pragma unroll
        for (int k = 0; k < TPT; ++k) {
          const int m = tid + k * TB;
          if (m >= M) continue;
          uint32_t *Pm = P + m;
          int a = a_[k], b = b_[k];
          t0_[k] += dt0v[k]; f0_[k] += df0v[k]; t1_[k] += dt1v[k]; f1_[k] += df1v[k];
          if (kind == 1) {
            if (i < j) {
              if (ii < a && a <= jj + 1) a_[k] = a - 1;
              if (ii < b && b <= jj + 1) b_[k] = b - 1;
              const uint32_t vb = (uint32_t)colbit(Pm, M, i);
              for (int w = i >> 5; w <= (j >> 5); ++w) {
                const uint32_t old = Pm[w * M];
                const uint32_t nxt = (w + 1 < NW) ? Pm[(w + 1) * M] : 0u;
                const uint32_t sh = (old >> 1) | (nxt << 31);
                const int lo = max(i, 32 * w), hi2 = min(j - 1, 32 * w + 31);
                uint32_t m1 = 0;
                if (hi2 >= lo) {
                  const int nb2 = hi2 - lo + 1;
                  m1 = (nb2 == 32) ? 0xffffffffu : (((1u << nb2) - 1u) << (lo & 31));
                }
                uint32_t nw = (old & ~m1) | (sh & m1);
                if ((j >> 5) == w) nw = (nw & ~(1u << (j & 31))) | (vb << (j & 31));
                Pm[w * M] = nw;
              }
            } else {
              if (ii <= a && a <= jj) a_[k] = a + 1;
              if (ii <= b && b <= jj) b_[k] = b + 1;
              const uint32_t vb = (uint32_t)colbit(Pm, M, i);
              for (int w = i >> 5; w >= (j >> 5); --w) {
                const uint32_t old = Pm[w * M];
                const uint32_t prv = (w > 0) ? Pm[(w - 1) * M] : 0u;
                const uint32_t sh = (old << 1) | (prv >> 31);
                const int lo = max(j + 1, 32 * w), hi2 = min(i, 32 * w + 31);
                uint32_t m1 = 0;
                if (hi2 >= lo) {
                  const int nb2 = hi2 - lo + 1;
                  m1 = (nb2 == 32) ? 0xffffffffu : (((1u << nb2) - 1u) << (lo & 31));
                }
                uint32_t nw = (old & ~m1) | (sh & m1);
                if ((j >> 5) == w) nw = (nw & ~(1u << (j & 31))) | (vb << (j & 31));
                Pm[w * M] = nw;
              }
            }
          } else {
            const int ain = ininterval(a, i, j + 1, inc1, inc2);
            const int bin = ininterval(b, i, j + 1, inc1, inc2);
            if (ain && !bin) a_[k] = i + j + 1 - a;
            else if (!ain && bin) b_[k] = i + j + 1 - b;
            else if (ain && bin) { b_[k] = i + j + 1 - a; a_[k] = i + j + 1 - b; }
            if (kind != 3) {
              for (int n = i; n < i + j - n; ++n) {
                const int p2 = i + j - n;
                const uint32_t *w1 = &Pm[(n >> 5) * M];
                const uint32_t *w2 = &Pm[(p2 >> 5) * M];
                const uint32_t b1 = (*w1 >> (n & 31)) & 1u, b2 = (*w2 >> (p2 & 31)) & 1u;
                if (b1 != b2) {
                  Pm[(n >> 5) * M] ^= (1u << (n & 31));
                  Pm[(p2 >> 5) * M] ^= (1u << (p2 & 31));
                }
              }
            } else {
              for (int r = 0; r < Kn - 1 - r; ++r) {
                const int n = nhpos[r], p2 = nhpos[Kn - 1 - r];
                const uint32_t b1 = (Pm[(n >> 5) * M] >> (n & 31)) & 1u;
                const uint32_t b2 = (Pm[(p2 >> 5) * M] >> (p2 & 31)) & 1u;
                if (b1 != b2) {
                  Pm[(n >> 5) * M] ^= (1u << (n & 31));
                  Pm[(p2 >> 5) * M] ^= (1u << (p2 & 31));
                }
              }
            }
          }
        }
        /* ---- rpi (double-buffered full permutation) and hard positions */
        if (kind == 1) {
          for (int n = tid; n < N; n += TB) {
            int src = n;
            if (i < j) { if (n >= i && n < j) src = n + 1; else if (n == j) src = i; }
            else { if (n > j && n <= i) src = n - 1; else if (n == j) src = i; }
            rn[n] = ro[src];
          }
#pragma unroll
          for (int q = 0; q < SR_NHMAX; ++q) {
            if (q < nh) {
              const int h = hp[q];
              if (h == i) hp[q] = j;
              else if (i < j && h > i && h <= j) hp[q] = h - 1;
              else if (i > j && h >= j && h < i) hp[q] = h + 1;
            }
          }
        } else if (kind != 3) {
          for (int n = tid; n < N; n += TB) rn[n] = ro[(n >= i && n <= j) ? (i + j - n) : n];
#pragma unroll
          for (int q = 0; q < SR_NHMAX; ++q)
            if (q < nh && hp[q] >= i && hp[q] <= j) hp[q] = i + j - hp[q];
        } else {
          for (int n = tid; n < N; n += TB)
            if (n < i || n > j || is_hard(hp, nh, n)) rn[n] = ro[n];
          for (int r = tid; r < Kn; r += TB) rn[nhpos[r]] = ro[nhpos[Kn - 1 - r]];
        }
        rcur ^= 1;
      } /* proposals */
    } /* sweeps */

    /* ---------------- saved sample (mcmc_save_chain, mcmc.c:69-92) */
    if (A.save) {
      __syncthreads();
      const int slot = A.rec_base + call;
      const int W = 2 * M + N;
      int16_t *rec = A.rec_abpi + ((size_t)chain * A.rec_cap + slot) * W;
#pragma unroll
      for (int k = 0; k < TPT; ++k) {
        const int m = tid + k * TB;
        if (m < M) { rec[m] = (int16_t)a_[k]; rec[M + m] = (int16_t)b_[k]; }
      }
      const int32_t *rc = rcur ? rpiB : rpiA;
      for (int n = tid; n < N; n += TB) rec[2 * M + rc[n]] = (int16_t)n;
      if (tid == 0) {
        double *rd = A.rec_cdl + ((size_t)chain * A.rec_cap + slot) * 3;
        rd[0] = c; rd[1] = d; rd[2] = loglik;
      }
    }
  } /* calls */

  /* ---------------- store state */
  __syncthreads();
  uint32_t *oP = A.P + (size_t)chain * NW * M;
  for (int i = tid; i < NW * M; i += TB) oP[i] = P[i];
  const int32_t *rc = rcur ? rpiB : rpiA;
  int32_t *orpi = A.rpi + (size_t)chain * N;
  for (int i = tid; i < N; i += TB) orpi[i] = rc[i];
  uint32_t *omt = A.mt + (size_t)chain * SR_RING * SR_MT_N;
  for (int i = tid; i < SR_RING * SR_MT_N; i += TB) omt[i] = ring[i];
#pragma unroll
  for (int k = 0; k < TPT; ++k) {
    const int m = tid + k * TB;
    if (m < M) {
      A.ab[(size_t)chain * 2 * M + m] = a_[k];
      A.ab[(size_t)chain * 2 * M + M + m] = b_[k];
      A.cnt[(size_t)chain * 4 * M + m] = t0_[k];
      A.cnt[(size_t)chain * 4 * M + M + m] = f0_[k];
      A.cnt[(size_t)chain * 4 * M + 2 * M + m] = t1_[k];
      A.cnt[(size_t)chain * 4 * M + 3 * M + m] = f1_[k];
    }
  }
  if (tid == 0) {
#pragma unroll
    for (int k = 0; k < SR_NHMAX; ++k)
      if (k < nh) A.hp[(size_t)chain * SR_NHMAX + k] = hp[k];
    A.cdl[(size_t)chain * 4 + 0] = c;
    A.cdl[(size_t)chain * 4 + 1] = d;
    A.cdl[(size_t)chain * 4 + 2] = loglik;
    A.rng[(size_t)chain * 2 + 0] = (uint64_t)R.blk * SR_MT_N + R.off;
    A.rng[(size_t)chain * 2 + 1] = R.gen;
    for (int k = 0; k < 7; ++k) A.acc[(size_t)chain * 8 + k] += acc[k];
    A.acc[(size_t)chain * 8 + 2] += misc[MS_CAB];
  }
}

/* ================================================================ session layer */
#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "seriation: HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return -5; } } while (0)

struct srk_dev {
  int device, N, M, NW, nh, nchains, TB, TPT, rec_cap;
  size_t lds;
  hipStream_t stream;
  int own_stream;
  hipEvent_t ev0, ev1;
  int have_events;
  KArgs args;
  void *bufs[16];
  int nbufs;
};

typedef void (*sr_kfn)(KArgs);

static sr_kfn sr_pick_kernel(int TB, int TPT)
{
#define SR_K(tb, tpt) if (TB == tb && TPT == tpt) return (sr_kfn)sr_sweep_kernel<tb, tpt>;
  SR_K(64, 1) SR_K(128, 1) SR_K(256, 1) SR_K(512, 1) SR_K(1024, 1) SR_K(1024, 2) SR_K(1024, 4)
#undef SR_K
  return nullptr;
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

extern "C" int srk_create(const sr_state_host *st, int device, int block_threads, int rec_cap_calls, srk_dev **out)
{
  int ndev = srk_device_count();
  if (ndev <= 0 || device < 0 || device >= ndev) return -5;
  if (st->nh > SR_NHMAX || st->N > 32767 || st->M > 32767) return -6;
  HIPCHK(hipSetDevice(device));
  srk_dev *d = new srk_dev();
  d->device = device; d->N = st->N; d->M = st->M; d->NW = st->NW; d->nh = st->nh; d->nchains = st->nchains;
  int TB = block_threads;
  if (TB <= 0) { TB = 64; while (TB < st->M && TB < 1024) TB *= 2; }
  int TPT = (st->M + TB - 1) / TB;
  if (TPT == 3) TPT = 4;
  if (!sr_pick_kernel(TB, TPT)) { delete d; return -6; }
  d->TB = TB; d->TPT = TPT;
  Lay L = sr_layout(st->N, st->M, st->NW);
  d->lds = L.total;
  if (d->lds > 160 * 1024) { delete d; return -6; }
  d->rec_cap = rec_cap_calls > 0 ? rec_cap_calls : 1;
  const size_t C = st->nchains;
  KArgs &A = d->args;
  memset(&A, 0, sizeof(A));
  A.N = st->N; A.M = st->M; A.NW = st->NW; A.nh = st->nh; A.nchains = st->nchains; A.rec_cap = d->rec_cap;
  int rc = 0;
  rc |= dev_alloc_copy(d, &A.P, st->P, C * st->NW * st->M);
  rc |= dev_alloc_copy(d, &A.rpi, st->rpi, C * st->N);
  rc |= dev_alloc_copy(d, &A.hp, st->hp, C * SR_NHMAX);
  rc |= dev_alloc_copy(d, &A.ab, st->ab, C * 2 * st->M);
  rc |= dev_alloc_copy(d, &A.cnt, st->cnt, C * 4 * st->M);
  rc |= dev_alloc_copy(d, &A.cdl, st->cdl, C * 4);
  rc |= dev_alloc_copy(d, &A.mt, st->mt, C * SR_RING * SR_MT_N);
  rc |= dev_alloc_copy(d, &A.rng, st->rng, C * 2);
  rc |= dev_alloc_copy(d, &A.acc, st->acc, C * 8);
  rc |= dev_alloc_copy(d, &A.rec_abpi, (const int16_t *)nullptr, C * d->rec_cap * (2 * st->M + st->N));
  rc |= dev_alloc_copy(d, &A.rec_cdl, (const double *)nullptr, C * d->rec_cap * 3);
  if (rc) { srk_destroy(d); return -5; }
  sr_kfn k = sr_pick_kernel(TB, TPT);
  if (hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)d->lds) != hipSuccess) {
    srk_destroy(d);
    return -5;
  }
  if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) { srk_destroy(d); return -5; }
  d->own_stream = 1;
  if (hipEventCreate(&d->ev0) == hipSuccess && hipEventCreate(&d->ev1) == hipSuccess) d->have_events = 1;
  *out = d;
  return 0;
}

extern "C" int srk_set_stream(srk_dev *d, void *stream)
{
  HIPCHK(hipSetDevice(d->device));
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
  sr_kfn k = sr_pick_kernel(d->TB, d->TPT);
  if (d->have_events) HIPCHK(hipEventRecord(d->ev0, d->stream));
  hipLaunchKernelGGL(k, dim3(d->nchains), dim3(d->TB), d->lds, d->stream, A);
  HIPCHK(hipGetLastError());
  if (d->have_events) HIPCHK(hipEventRecord(d->ev1, d->stream));
  return 0;
}

extern "C" int srk_sync(srk_dev *d)
{
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipStreamSynchronize(d->stream));
  return 0;
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

extern "C" int srk_fetch_records(srk_dev *d, int first, int count, int16_t *ab_pi, double *cdl)
{
  if (first < 0 || count < 0 || first + count > d->rec_cap) return -1;
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipStreamSynchronize(d->stream));
  const size_t W = 2 * (size_t)d->M + d->N;
  for (int c = 0; c < d->nchains; ++c) {
    if (ab_pi)
      HIPCHK(hipMemcpy(ab_pi + (size_t)c * count * W, d->args.rec_abpi + ((size_t)c * d->rec_cap + first) * W,
                       (size_t)count * W * sizeof(int16_t), hipMemcpyDeviceToHost));
    if (cdl)
      HIPCHK(hipMemcpy(cdl + (size_t)c * count * 3, d->args.rec_cdl + ((size_t)c * d->rec_cap + first) * 3,
                       (size_t)count * 3 * sizeof(double), hipMemcpyDeviceToHost));
  }
  return 0;
}

extern "C" int srk_download_state(srk_dev *d, sr_state_host *st)
{
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipStreamSynchronize(d->stream));
  const size_t C = d->nchains;
  const KArgs &A = d->args;
  if (st->P) HIPCHK(hipMemcpy(st->P, A.P, C * d->NW * d->M * 4, hipMemcpyDeviceToHost));
  if (st->rpi) HIPCHK(hipMemcpy(st->rpi, A.rpi, C * d->N * 4, hipMemcpyDeviceToHost));
  if (st->hp) HIPCHK(hipMemcpy(st->hp, A.hp, C * SR_NHMAX * 4, hipMemcpyDeviceToHost));
  if (st->ab) HIPCHK(hipMemcpy(st->ab, A.ab, C * 2 * d->M * 4, hipMemcpyDeviceToHost));
  if (st->cnt) HIPCHK(hipMemcpy(st->cnt, A.cnt, C * 4 * d->M * 4, hipMemcpyDeviceToHost));
  if (st->cdl) HIPCHK(hipMemcpy(st->cdl, A.cdl, C * 4 * 8, hipMemcpyDeviceToHost));
  if (st->mt) HIPCHK(hipMemcpy(st->mt, A.mt, C * SR_RING * SR_MT_N * 4, hipMemcpyDeviceToHost));
  if (st->rng) HIPCHK(hipMemcpy(st->rng, A.rng, C * 2 * 8, hipMemcpyDeviceToHost));
  if (st->acc) HIPCHK(hipMemcpy(st->acc, A.acc, C * 8 * 8, hipMemcpyDeviceToHost));
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
  delete d;
}

/* ================================================================ self-test hook */
/* Device copies of the deterministic exp/log, for the host<->device bit-parity test. */
__global__ void sr_math_selftest_kernel(const double *in, long n, double *oe, double *ol)
{
  __shared__ double tabs[640];
  for (int i = threadIdx.x; i < 128; i += blockDim.x) {
    tabs[i] = c_exp_thi[i];
    tabs[128 + i] = c_exp_tlo[i];
    tabs[256 + i] = c_log_invc[i];
    tabs[384 + i] = c_log_lhi[i];
    tabs[512 + i] = c_log_llo[i];
  }
  __syncthreads();
  sr_mtab tb;
  tb.exp_thi = tabs; tb.exp_tlo = tabs + 128; tb.log_invc = tabs + 256; tb.log_lhi = tabs + 384; tb.log_llo = tabs + 512;
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
