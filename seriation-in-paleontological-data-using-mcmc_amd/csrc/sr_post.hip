/*
 * sr_post.hip -- posterior summaries over saved samples on the GPU:
 * the per-sample accumulations of the reference's analysis script, bit for bit.
 *
 *   SR_POST_PAIR_ORDER   compute_pair_order_matrix + generate_po_matrix   script.py:155-189
 *   SR_POST_ALIVE        plot_taxa_occurence_probability_matrix (X_sum)    script.py:306-333
 *   SR_POST_FALSE_ALIVE  plot_false_taxa_occurence_probability (X_sum)    script.py:350-377
 *   SR_POST_FALSE_ONES   plot_false_ones_probability (X_sum)               script.py:392-417
 *   SR_POST_EXP_PI       compute_exp_pi                                    script.py:230-251
 *   SR_POST_EXP_A        compute_exp_a                                     script.py:254-275
 *
 * Every output element e follows the script's float operations exactly, in its order:
 *   acc = 0, tot = 0 (acc is never reset between chains -- the script's quirk)
 *   for each selected chain (selection order): for each sample s: acc += v_e(s)
 *                                               acc /= 1000; tot += acc   (EXP_PI: tot = acc)
 *   out = tot / chains_selected
 * with v in {-1, 0, 1} (or a position / limit for EXP_PI / EXP_A).  The element is owned by one
 * thread, so its sequential f64 sum is the script's; -ffp-contract=off keeps the ops separate.
 *
 * Layout: samples are the sweep kernel's records, int16 rows [a (M) | b (M) | pi (N)] with
 * pi[site] = position (mcmc_save_chain, mcmc.c:69-92), one row per saved mcmc_sample call;
 * chain k's rows start at rec + chain_off[k], consecutive rows row_stride apart.  A block owns a
 * tile of 16 output rows x 64 output columns: lane = column (its operand loads coalesce across
 * the wave), each thread keeps 4 rows' accumulators in registers.  Operands are staged through
 * LDS in chunks of CS samples, the next chunk's loads in flight while the current one is summed;
 * the row operand of PAIR_ORDER (pi of the row site) is an LDS broadcast.  The records of the
 * selected chains (at most a few MB) stay L2/MALL-resident across the tiles: the kernel is
 * bound by the dependent f64 add chains, one per element.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include <stdio.h>
#include "sr_internal.h"

#define TR 16   /* output rows per block (4 waves x 4 rows) */
#define TCOL 64 /* output columns per block (lanes) */
#define CS 64   /* samples per LDS-staged chunk (two chunks: one consumed, one in flight) */

struct PostArgs {
  const int16_t *rec;
  const long long *chain_off;   /* [n_sel] element offset of each chain's first row */
  long long row_stride;
  const uint8_t *X;             /* N x M dataset rows (FALSE_ONES only) */
  int n_sel, count, N, M, R, C;
  double div;
  double *out;                  /* R x C */
};

template <int KIND>
__global__ __launch_bounds__(256) void sr_post_kernel(PostArgs P)
{
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = blockIdx.x * TCOL + lane;
  const int r0 = __builtin_amdgcn_readfirstlane(blockIdx.y * TR + wave * 4);
  const bool cok = col < P.C;
  const int cc = cok ? col : 0;
  const int M = P.M, N = P.N;
  /* operand offsets inside a row */
  const int coff = (KIND == SRP_PAIR_ORDER || KIND == SRP_EXP_PI) ? 2 * M + cc : cc;
  int xo[4] = {0, 0, 0, 0};
  if (KIND == SRP_FALSE_ONES) {
#pragma unroll
    for (int k = 0; k < 4; ++k) xo[k] = (r0 + k < P.R && cok) ? P.X[(size_t)(r0 + k) * M + cc] : 0;
  }
  double acc[4] = {0.0, 0.0, 0.0, 0.0}, tot[4] = {0.0, 0.0, 0.0, 0.0};
  auto chain_end = [&]() {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc[k] = acc[k] / 1000.0;
      tot[k] = (KIND == SRP_EXP_PI) ? acc[k] : tot[k] + acc[k];
    }
  };
  /* The selected chains' samples form one stream g = chain * count + s (selection order, then
     sample order), consumed in chunks of CS samples.  A chunk's operands (x, y per column, the
     pair-order row operands) are staged in LDS by the whole block; chunk c+1's global loads are
     in flight while chunk c is accumulated, so one memory latency is paid per chunk, not per
     sample.  The accumulation order per element is still the script's sample order. */
  constexpr bool NEEDY = (KIND == SRP_ALIVE || KIND == SRP_FALSE_ALIVE || KIND == SRP_FALSE_ONES);
  constexpr bool NEEDP = (KIND == SRP_PAIR_ORDER);
  typedef typename std::conditional<NEEDY, uint32_t, uint16_t>::type xy_t;
  __shared__ xy_t xsh[2][CS][TCOL];   /* x (low half), y in the high half for NEEDY kinds */
  __shared__ __attribute__((aligned(8))) int16_t psh[NEEDP ? 2 : 1][NEEDP ? CS : 1][TR];
  const unsigned total = (unsigned)P.n_sel * (unsigned)P.count;
  const int t = threadIdx.x;
  const int prow = min((int)blockIdx.y * TR + (t & (TR - 1)), N - 1);   /* pair-order row operand */
  int16_t lx[CS / 4], ly[NEEDY ? CS / 4 : 1], lp[NEEDP ? CS / 16 : 1];
  auto rowp = [&](unsigned g) -> const int16_t * {
    g = min(g, total - 1u);
    const unsigned ch = g / (unsigned)P.count, sm = g - ch * (unsigned)P.count;
    return P.rec + P.chain_off[ch] + (long long)sm * P.row_stride;
  };
  auto load_chunk = [&](unsigned g0) {   /* thread t: samples wave + 4k (x, y), t/16 + 16k (p) */
#pragma unroll
    for (int k = 0; k < CS / 4; ++k) {
      const int16_t *row = rowp(g0 + wave + 4 * k);
      lx[k] = row[coff];
      if (NEEDY) ly[k] = row[M + cc];
    }
    if (NEEDP) {
#pragma unroll
      for (int k = 0; k < CS / 16; ++k) lp[k] = rowp(g0 + (t >> 4) + 16 * k)[2 * M + prow];
    }
  };
  auto store_chunk = [&](int b) {
#pragma unroll
    for (int k = 0; k < CS / 4; ++k) {
      xsh[b][wave + 4 * k][lane] = (xy_t)((uint32_t)(uint16_t)lx[k] | (NEEDY ? (uint32_t)(uint16_t)ly[k] << 16 : 0u));
    }
    if (NEEDP) {
#pragma unroll
      for (int k = 0; k < CS / 16; ++k) psh[b][(t >> 4) + 16 * k][t & (TR - 1)] = lp[k];
    }
  };
  if (total == 0) {
    for (int ch = 0; ch < P.n_sel; ++ch) chain_end();
  } else {
    const unsigned nchunk = (total + CS - 1) / CS;
    load_chunk(0);
    store_chunk(0);
    __syncthreads();
    int sm = 0;   /* sample index inside the current chain (uniform) */
    for (unsigned c = 0; c < nchunk; ++c) {
      const int b = c & 1;
      if (c + 1 < nchunk) load_chunk((c + 1) * CS);
      const unsigned g0 = c * CS;
      const int nu = (int)min((unsigned)CS, total - g0);
      for (int u0 = 0; u0 < nu;) {   /* runs of samples up to the next chain boundary: no branch inside */
        const int run = min(nu - u0, P.count - sm);
#pragma unroll 16
        for (int u = u0; u < u0 + run; ++u) {   /* unrolled: the LDS reads run ahead of the add chain */
          const uint32_t xy = (uint32_t)xsh[b][u][lane];
          const int x = (int16_t)(uint16_t)(xy & 0xffffu);
          const int y = NEEDY ? (int16_t)(uint16_t)(xy >> 16) : 0;
          /* the wave's 4 row operands: one 8-byte LDS broadcast */
          const uint64_t pr4 = NEEDP ? *(const uint64_t *)&psh[NEEDP ? b : 0][NEEDP ? u : 0][wave * 4] : 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int r = r0 + k;   /* output row: PAIR_ORDER site i; ALIVE.. site index j; EXP_* 0 */
            int v;
            if (KIND == SRP_PAIR_ORDER) {
              const int pr = (int16_t)(uint16_t)(pr4 >> (16 * k));
              v = (r == col) ? -1 : (pr < x ? 1 : 0);                /* generate_po_matrix, script.py:183-188 */
            } else if (KIND == SRP_ALIVE) {
              v = (r >= x && r <= y) ? 1 : 0;                       /* script.py:326 */
            } else if (KIND == SRP_FALSE_ALIVE) {
              v = (r < x || r > y) ? 1 : 0;                         /* script.py:370 */
            } else if (KIND == SRP_FALSE_ONES) {
              v = (xo[k] == 1 && !(r >= x && r <= y)) ? 1 : 0;      /* script.py:408-413 */
            } else {
              v = x;                                                /* EXP_PI: pi[site]; EXP_A: a[taxon] */
            }
            acc[k] = acc[k] + (double)v;
          }
        }
        u0 += run;
        sm += run;
        if (sm == P.count) { sm = 0; chain_end(); }
      }
      if (c + 1 < nchunk) store_chunk(b ^ 1);   /* buffer b^1 was last read before the previous barrier */
      __syncthreads();
    }
  }
  if (cok) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (r0 + k < P.R) P.out[(size_t)(r0 + k) * P.C + col] = tot[k] / P.div;
  }
}

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "seriation: HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); rc = -5; goto done; } } while (0)

/* One summary kind over device-resident records; out_host receives R x C doubles. */
extern "C" int srp_posterior_dev(int device, void *stream, int kind, const int16_t *d_rec, const long long *chain_off,
                                 int n_sel, int count, long long row_stride, int N, int M, const uint8_t *X_host,
                                 int chains_selected, double *out_host, float *ms)
{
  int rc = 0;
  long long *d_off = nullptr;
  uint8_t *d_X = nullptr;
  double *d_out = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipStream_t st = (hipStream_t)stream;
  int R, C;
  switch (kind) {
    case SRP_PAIR_ORDER: R = N; C = N; break;
    case SRP_ALIVE: case SRP_FALSE_ALIVE: case SRP_FALSE_ONES: R = N; C = M; break;
    case SRP_EXP_PI: R = 1; C = N; break;
    case SRP_EXP_A: R = 1; C = M; break;
    default: return -1;
  }
  if (n_sel <= 0 || count < 0 || N < 1 || M < 1 || chains_selected == 0) return -1;
  if ((long long)n_sel * count >= (1LL << 31)) return -1;   /* the kernel indexes samples in 32 bits */
  if (kind == SRP_FALSE_ONES && !X_host) return -1;
  {
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipMalloc(&d_off, sizeof(long long) * n_sel));
    HIPCHK(hipMemcpy(d_off, chain_off, sizeof(long long) * n_sel, hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&d_out, sizeof(double) * (size_t)R * C));
    if (kind == SRP_FALSE_ONES) {
      HIPCHK(hipMalloc(&d_X, (size_t)N * M));
      HIPCHK(hipMemcpy(d_X, X_host, (size_t)N * M, hipMemcpyHostToDevice));
    }
    PostArgs A;
    A.rec = d_rec; A.chain_off = d_off; A.row_stride = row_stride; A.X = d_X;
    A.n_sel = n_sel; A.count = count; A.N = N; A.M = M; A.R = R; A.C = C;
    A.div = (double)chains_selected; A.out = d_out;
    dim3 grid((C + TCOL - 1) / TCOL, (R + TR - 1) / TR);
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, st));
    switch (kind) {
      case SRP_PAIR_ORDER: hipLaunchKernelGGL(sr_post_kernel<SRP_PAIR_ORDER>, grid, dim3(256), 0, st, A); break;
      case SRP_ALIVE: hipLaunchKernelGGL(sr_post_kernel<SRP_ALIVE>, grid, dim3(256), 0, st, A); break;
      case SRP_FALSE_ALIVE: hipLaunchKernelGGL(sr_post_kernel<SRP_FALSE_ALIVE>, grid, dim3(256), 0, st, A); break;
      case SRP_FALSE_ONES: hipLaunchKernelGGL(sr_post_kernel<SRP_FALSE_ONES>, grid, dim3(256), 0, st, A); break;
      case SRP_EXP_PI: hipLaunchKernelGGL(sr_post_kernel<SRP_EXP_PI>, grid, dim3(256), 0, st, A); break;
      default: hipLaunchKernelGGL(sr_post_kernel<SRP_EXP_A>, grid, dim3(256), 0, st, A); break;
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(e1, st));
    HIPCHK(hipStreamSynchronize(st));
    if (ms) HIPCHK(hipEventElapsedTime(ms, e0, e1));
    HIPCHK(hipMemcpy(out_host, d_out, sizeof(double) * (size_t)R * C, hipMemcpyDeviceToHost));
  }
done:
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (d_off) (void)hipFree(d_off);
  if (d_out) (void)hipFree(d_out);
  if (d_X) (void)hipFree(d_X);
  return rc;
}

/* Records from host memory: ab_pi [n_sel][count][2M+N] int16 (selection order). */
extern "C" int srp_posterior_host(int device, int kind, const int16_t *ab_pi, int n_sel, int count, int N, int M,
                                  const uint8_t *X_host, int chains_selected, double *out_host, float *ms)
{
  int rc = 0;
  int16_t *d_rec = nullptr;
  long long *off = nullptr;
  const long long W = 2LL * M + N;
  const size_t bytes = (size_t)n_sel * count * W * sizeof(int16_t);
  if (n_sel <= 0 || count < 0) return -1;
  off = (long long *)malloc(sizeof(long long) * n_sel);
  if (!off) return -4;
  for (int k = 0; k < n_sel; ++k) off[k] = (long long)k * count * W;
  {
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipMalloc(&d_rec, bytes + 16));
    if (bytes) HIPCHK(hipMemcpy(d_rec, ab_pi, bytes, hipMemcpyHostToDevice));
    rc = srp_posterior_dev(device, nullptr, kind, d_rec, off, n_sel, count, W, N, M, X_host, chains_selected, out_host, ms);
  }
done:
  if (d_rec) (void)hipFree(d_rec);
  free(off);
  return rc;
}
