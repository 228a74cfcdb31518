// Micro-benchmark of fc1-shaped int8 GEMM variants (M=1024, K=4096, N=512):
// times the library kernel vs candidate tilings.  Build on the box:
//   hipcc --offload-arch=gfx950 -O3 -I../../include fc_bench.hip -o fc_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// variant A: block = WAVES waves, tile 32 rows x 32*NT feats, K split over waves, U-deep batches
template <int WAVES, int NTF, int U>
__global__ __launch_bounds__(WAVES * 64) void kA(const unsigned char* x, int m, int k, const signed char* w, int n, int* out) {
  __shared__ int part[WAVES][NTF][16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l32 = lane & 31, hi = lane >> 5;
  const int f0 = blockIdx.x * 32 * NTF, r0 = blockIdx.y * 32;
  const int kq = k / WAVES, kb = wave * kq;
  const unsigned char* xr = x + (long)(r0 + l32) * k + hi * 16;
  const signed char* wr[NTF];
  for (int i = 0; i < NTF; ++i) wr[i] = w + (long)(f0 + i * 32 + l32) * k + hi * 16;
  v16i acc[NTF];
  for (int i = 0; i < NTF; ++i) acc[i] = (v16i){0};
  for (int kk = kb; kk < kb + kq; kk += 32 * U) {
    v4i xb[U], wa[U][NTF];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xb[u] = *(const v4i*)(xr + kk + 32 * u);
#pragma unroll
      for (int i = 0; i < NTF; ++i) wa[u][i] = *(const v4i*)(wr[i] + kk + 32 * u);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < NTF; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wa[u][i], xb[u], acc[i], 0, 0, 0);
  }
  for (int i = 0; i < NTF; ++i) for (int r = 0; r < 16; ++r) part[wave][i][r][lane] = acc[i][r];
  __syncthreads();
  if (wave == 0) {
    for (int i = 0; i < NTF; ++i) for (int r = 0; r < 16; ++r) {
      int s = 0;
      for (int q = 0; q < WAVES; ++q) s += part[q][i][r][lane];
      out[((long)(r0 + l32)) * n + f0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi] = s;
    }
  }
}

// variant B: operands pre-packed K-chunk-major: X'[k/32][m][32], W'[k/32][n][32]
// so a 32-row fragment load is one contiguous 1 KB.
template <int WAVES, int NTF, int U>
__global__ __launch_bounds__(WAVES * 64) void kB(const unsigned char* x, int m, int k, const signed char* w, int n, int* out) {
  __shared__ int part[WAVES][NTF][16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l32 = lane & 31, hi = lane >> 5;
  const int f0 = blockIdx.x * 32 * NTF, r0 = blockIdx.y * 32;
  const int kcq = (k / 32) / WAVES, kc0 = wave * kcq;
  v16i acc[NTF];
  for (int i = 0; i < NTF; ++i) acc[i] = (v16i){0};
  for (int kc = kc0; kc < kc0 + kcq; kc += U) {
    v4i xb[U], wa[U][NTF];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xb[u] = *(const v4i*)(x + ((long)(kc + u) * m + r0 + l32) * 32 + hi * 16);
#pragma unroll
      for (int i = 0; i < NTF; ++i) wa[u][i] = *(const v4i*)(w + ((long)(kc + u) * n + f0 + i * 32 + l32) * 32 + hi * 16);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < NTF; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wa[u][i], xb[u], acc[i], 0, 0, 0);
  }
  for (int i = 0; i < NTF; ++i) for (int r = 0; r < 16; ++r) part[wave][i][r][lane] = acc[i][r];
  __syncthreads();
  if (wave == 0) {
    for (int i = 0; i < NTF; ++i) for (int r = 0; r < 16; ++r) {
      int s = 0;
      for (int q = 0; q < WAVES; ++q) s += part[q][i][r][lane];
      out[((long)(r0 + l32)) * n + f0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi] = s;
    }
  }
}

template <int WAVES, int NTF, int U>
__global__ __launch_bounds__(WAVES * 64) void kC(const unsigned char* x, int m, int k, const signed char* w, int n, int* out) {
  __shared__ int part[WAVES][NTF][16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l32 = lane & 31, hi = lane >> 5;
  const int f0 = blockIdx.y * 32 * NTF, r0 = blockIdx.x * 32;
  const int kcq = (k / 32) / WAVES, kc0 = wave * kcq;
  v16i acc[NTF];
  for (int i = 0; i < NTF; ++i) acc[i] = (v16i){0};
  for (int kc = kc0; kc < kc0 + kcq; kc += U) {
    v4i xb[U], wa[U][NTF];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xb[u] = *(const v4i*)(x + ((long)(kc + u) * m + r0 + l32) * 32 + hi * 16);
#pragma unroll
      for (int i = 0; i < NTF; ++i) wa[u][i] = *(const v4i*)(w + ((long)(kc + u) * n + f0 + i * 32 + l32) * 32 + hi * 16);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < NTF; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wa[u][i], xb[u], acc[i], 0, 0, 0);
  }
  for (int i = 0; i < NTF; ++i) for (int r = 0; r < 16; ++r) part[wave][i][r][lane] = acc[i][r];
  __syncthreads();
  if (wave == 0) {
    for (int i = 0; i < NTF; ++i) for (int r = 0; r < 16; ++r) {
      int s = 0;
      for (int q = 0; q < WAVES; ++q) s += part[q][i][r][lane];
      out[((long)(r0 + l32)) * n + f0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi] = s;
    }
  }
}

template <class K>
float timeit(K launch, int iters = 50) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 5; ++i) launch();
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / iters;
}

int main() {
  const int M = 1024, K = 4096, N = 512;
  std::vector<unsigned char> hx((size_t)M * K); std::vector<signed char> hw((size_t)N * K);
  for (auto& v : hx) v = rand() & 0xff; for (auto& v : hw) v = (rand() & 0xff) - 128;
  unsigned char* x; signed char* w; int *o1, *o2;
  CK(hipMalloc(&x, hx.size())); CK(hipMalloc(&w, hw.size())); CK(hipMalloc(&o1, M * N * 4)); CK(hipMalloc(&o2, M * N * 4));
  CK(hipMemcpy(x, hx.data(), hx.size(), hipMemcpyHostToDevice)); CK(hipMemcpy(w, hw.data(), hw.size(), hipMemcpyHostToDevice));
#define RUN(W, NT, U) { float us = timeit([&] { hipLaunchKernelGGL((kA<W, NT, U>), dim3(N / (32 * NT), M / 32), dim3(W * 64), 0, 0, x, M, K, w, N, o2); }); \
    printf("kA<waves=%d, ntf=%d, U=%d>: %.2f us  (%.0f TOPS)\n", W, NT, U, us, 2.0 * M * N * K / us / 1e6); }
#define RUNB(W, NT, U) { float us = timeit([&] { hipLaunchKernelGGL((kB<W, NT, U>), dim3(N / (32 * NT), M / 32), dim3(W * 64), 0, 0, x, M, K, w, N, o1); }); \
    printf("kB<waves=%d, ntf=%d, U=%d>: %.2f us  (%.0f TOPS)\n", W, NT, U, us, 2.0 * M * N * K / us / 1e6); }
#define RUNC(W, NT, U) { float us = timeit([&] { hipLaunchKernelGGL((kC<W, NT, U>), dim3(M / 32, N / (32 * NT)), dim3(W * 64), 0, 0, x, M, K, w, N, o1); }); \
    printf("kC<waves=%d, ntf=%d, U=%d>: %.2f us  (%.0f TOPS)\n", W, NT, U, us, 2.0 * M * N * K / us / 1e6); }
  RUNB(8, 1, 4) RUNC(8, 1, 4) RUNC(8, 2, 4) RUNC(4, 2, 8) RUNC(16, 1, 2) RUNC(8, 2, 2) RUNC(4, 4, 4) RUNC(16, 2, 1)
  RUN(4, 2, 4) RUN(4, 2, 8)
  return 0;
}
