// Latency microbenchmarks on gfx950 (diagnostic): dependent chains timed with s_memtime.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#pragma clang diagnostic ignored "-Wunused-result"

__global__ void k_fma64(void *outv, unsigned long long *cyc, int n, double a)
{ double *out = (double *)outv;
  double x = threadIdx.x * 1e-3;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 32
  for (int i = 0; i < n; ++i) x = __builtin_fma(x, a, 1e-9);
  __builtin_amdgcn_s_waitcnt(0);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}
__global__ void k_mul64(void *outv, unsigned long long *cyc, int n, double a)
{ double *out = (double *)outv;
  double x = threadIdx.x * 1e-3 + 1.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 32
  for (int i = 0; i < n; ++i) x = x * a;
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}
__global__ void k_add32(void *outv, unsigned long long *cyc, int n, double ad)
{ int *out = (int *)outv; int a = (int)ad;
  int x = threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 32
  for (int i = 0; i < n; ++i) x = (x ^ a) + i;
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}
__global__ void k_lds(void *outv, unsigned long long *cyc, int n, double)
{ int *out = (int *)outv;
  __shared__ int buf[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) buf[i] = (i * 97 + 13) & 4095;
  __syncthreads();
  int p = threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 32
  for (int i = 0; i < n; ++i) p = buf[p];
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = p;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}
__global__ void k_shfl(void *outv, unsigned long long *cyc, int n, double)
{ int *out = (int *)outv;
  int x = threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 32
  for (int i = 0; i < n; ++i) x += __shfl_xor(x, 1 + (i & 31));
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}
__global__ void k_rfl(void *outv, unsigned long long *cyc, int n, double)
{ int *out = (int *)outv;
  __shared__ int buf[64];
  if (threadIdx.x < 64) buf[threadIdx.x] = (threadIdx.x + 1) & 63;
  __syncthreads();
  int p = 0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 32
  for (int i = 0; i < n; ++i) p = __builtin_amdgcn_readfirstlane(buf[p]);   /* LDS -> SGPR chain */
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = p;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

__global__ void k_branch(void *outv, unsigned long long *cyc, int n, double)
{ int *out = (int *)outv;
  int x = threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma nounroll
  for (int i = 0; i < n; ++i) { x ^= i; __builtin_amdgcn_sched_barrier(0); }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}
typedef void (*KF)(void *, unsigned long long *, int, double);
static void run(const char *name, KF kern, int threads, int n, double arg, bool)
{
  void *out; unsigned long long *cyc;
  hipMalloc(&out, 100 * 1024 * 8);
  hipMalloc(&cyc, 100 * 16 * 8);
  hipMemset(cyc, 0, 100 * 16 * 8);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(kern, dim3(100), dim3(threads), 0, 0, out, cyc, n, arg);
  }
  hipDeviceSynchronize();
  unsigned long long h[100 * 16];
  hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
  double s = 0; int c = 0;
  for (int b = 0; b < 100; ++b) for (int w = 0; w < threads / 64; ++w) { s += h[b * 16 + w]; c++; }
  printf("%-28s threads %4d: %.2f cycles per step\n", name, threads, s / c / n);
  hipFree(out); hipFree(cyc);
}
int main()
{
  const int n = 4096;
  for (int t : {64, 512}) {
    run("fma_f64 dependent", k_fma64, t, n, 1.0000001, true);
    run("mul_f64 dependent", k_mul64, t, n, 1.0000001, true);
    run("int xor+add dependent", k_add32, t, n, 12345, false);
    run("ds_read_b32 pointer chase", k_lds, t, n, 0.0, false);
    run("shfl_xor (bpermute) chain", k_shfl, t, n, 0.0, false);
    run("LDS->readfirstlane chain", k_rfl, t, n, 0.0, false);
    run("loop iteration (taken branch)", k_branch, t, n, 0.0, false);
  }
  return 0;
}
