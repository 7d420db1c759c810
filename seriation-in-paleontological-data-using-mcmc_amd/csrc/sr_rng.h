/*
 * sr_rng.h -- GSL-2.6-compatible MT19937 stream, laid out for the GPU.
 *
 * The reference draws every random number from one global gsl_rng of type mt19937
 * seeded from GSL_RNG_SEED (mcmc.c:47, 581-593).  The sampler keeps exactly that
 * stream per chain, but stores it as a ring of K raw (untempered) 624-word blocks:
 * block g+1 = twist(block g) can be produced by many lanes in three dependency phases
 * (k in [0,227) reads only block g; [227,454) also reads new[k-227]; [454,624) reads
 * new words from the second phase), and a word is tempered when read.  Word w of the
 * output stream lives in block 1 + w/624 (block 0 = the seeded state, as GSL's
 * mt_set leaves mti = 624), so stream position `pos` starts at 624.
 *
 * Host helpers below (sr_hrng_*) restate gsl_rng_uniform / uniform_int / ran_shuffle /
 * ran_choose for chain initialisation (mcmc_randomize, mcmc.c:477-578).
 */
#ifndef SR_RNG_H
#define SR_RNG_H
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#ifdef __HIPCC__
#define SR_RHD __host__ __device__ __forceinline__
#else
#define SR_RHD static inline
#endif

#define SR_MT_N 624
#define SR_MT_M 397

SR_RHD uint32_t sr_mt_temper(uint32_t k)
{
  k ^= (k >> 11);
  k ^= (k << 7) & 0x9d2c5680u;
  k ^= (k << 15) & 0xefc60000u;
  k ^= (k >> 18);
  return k;
}

/* the inverse of sr_mt_temper: sr_mt_temper(sr_mt_untemper(x)) == x for every x (the Philox
 * mode stores untempered words in the ring, so every read site keeps its tempering) */
SR_RHD uint32_t sr_mt_untemper(uint32_t y)
{
  y ^= y >> 18;
  y ^= (y << 15) & 0xefc60000u;
  uint32_t x = y;
  for (int i = 0; i < 4; ++i) x = y ^ ((x << 7) & 0x9d2c5680u);
  return x ^ (x >> 11) ^ (x >> 22);
}

/* ---- opt-in counter-based stream (SR_F_RNG_PHILOX; north_star "Philox state per lane") ----
 * Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11; the generator rocRAND's philox4x32_10
 * implements): word w of a chain's stream = philox(key, ctr = {w / 4 lo, w / 4 hi, 0, 0})[w % 4],
 * key = {seed lo, seed hi ^ SR_PHILOX_KEY1}.  Any block of words is computable lane-parallel with
 * no state but the counter.  Not the reference's stream: statistically equivalent, not bit-equal. */
#define SR_PHILOX_KEY1 0xA511E9B3u
SR_RHD void sr_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4])
{
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0, h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    c0 = h1 ^ c1 ^ k0; c1 = l1; c2 = h0 ^ c3 ^ k1; c3 = l0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* a chain's Philox key from its GSL_RNG_SEED value (0 -> GSL's default 4357, as mt_set) */
SR_RHD void sr_philox_key(uint64_t seed, uint32_t key[2])
{
  if (seed == 0) seed = 4357;
  key[0] = (uint32_t)seed;
  key[1] = (uint32_t)(seed >> 32) ^ SR_PHILOX_KEY1;
}

/* one recurrence step: y = upper(cur) | lower(next); far ^ (y >> 1) ^ mag(y) */
SR_RHD uint32_t sr_mt_mix(uint32_t cur, uint32_t next, uint32_t far)
{
  uint32_t y = (cur & 0x80000000u) | (next & 0x7fffffffu);
  return far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

/* GSL mt_set: seed 0 -> 4357; Knuth multiplier recurrence */
SR_RHD void sr_mt_seed_block(uint32_t *blk, unsigned long s)
{
  if (s == 0) s = 4357;
  blk[0] = (uint32_t)(s & 0xffffffffUL);
  for (int i = 1; i < SR_MT_N; i++) {
    uint32_t p = blk[i - 1];
    blk[i] = (uint32_t)(1812433253UL * (p ^ (p >> 30)) + (unsigned long)i);
  }
}

/* sequential twist (host): next = twist(prev), prev and next distinct */
SR_RHD void sr_mt_next_block(const uint32_t *prev, uint32_t *next)
{
  int k;
  for (k = 0; k < SR_MT_N - SR_MT_M; k++) next[k] = sr_mt_mix(prev[k], prev[k + 1], prev[k + SR_MT_M]);
  for (; k < SR_MT_N - 1; k++) next[k] = sr_mt_mix(prev[k], prev[k + 1], next[k - (SR_MT_N - SR_MT_M)]);
  next[SR_MT_N - 1] = sr_mt_mix(prev[SR_MT_N - 1], next[0], next[SR_MT_M - 1]);
}

/* ------------------------------------------------------------------ host stream */
typedef struct {
  uint32_t blk[SR_MT_N];  /* raw words of block `bidx` */
  uint64_t bidx;          /* index of the block held in blk (0 = seeded state) */
  uint64_t pos;           /* next word index; words of block b are [624b, 624b+624) */
} sr_hrng;

static inline void sr_hrng_seed(sr_hrng *r, unsigned long s)
{
  sr_mt_seed_block(r->blk, s);
  r->bidx = 0;
  r->pos = SR_MT_N;
}

static inline uint32_t sr_hrng_get(sr_hrng *r)
{
  if (r->pos >= (r->bidx + 1) * SR_MT_N) {
    uint32_t nb[SR_MT_N];
    sr_mt_next_block(r->blk, nb);
    memcpy(r->blk, nb, sizeof nb);
    r->bidx++;
  }
  uint32_t w = r->blk[r->pos - r->bidx * SR_MT_N];
  r->pos++;
  return sr_mt_temper(w);
}

static inline double sr_hrng_uniform(sr_hrng *r) { return sr_hrng_get(r) / 4294967296.0; }

static inline unsigned long sr_hrng_uniform_int(sr_hrng *r, unsigned long n)
{
  unsigned long scale = 0xffffffffUL / n, k;
  do { k = sr_hrng_get(r) / scale; } while (k >= n);
  return k;
}

/* gsl_ran_shuffle over int32 */
static inline void sr_hrng_shuffle(sr_hrng *r, int32_t *a, size_t n)
{
  if (n < 2) return;
  for (size_t i = n - 1; i > 0; i--) {
    size_t j = sr_hrng_uniform_int(r, i + 1);
    int32_t t = a[i]; a[i] = a[j]; a[j] = t;
  }
}

/* gsl_ran_choose over int32 (k of n, order preserved) */
static inline void sr_hrng_choose(sr_hrng *r, int32_t *dest, size_t k, const int32_t *src, size_t n)
{
  size_t j = 0;
  for (size_t i = 0; i < n && j < k; i++)
    if ((double)(n - i) * sr_hrng_uniform(r) < (double)(k - j)) dest[j++] = src[i];
}

#endif
