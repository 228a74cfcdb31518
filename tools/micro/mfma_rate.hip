// Probe: issue cycles of v_mfma_i32_32x32x32_i8 (and 16x16x64) back to back on
// one SIMD, one wave, 8 independent accumulators, random operands.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef int v4acc __attribute__((ext_vector_type(4)));
template <int BIG>
__global__ __launch_bounds__(64) void k(const int* in, int* out, long long* cyc, int iters) {
  const int lane = threadIdx.x & 63;
  v4i a = {in[lane], in[lane + 64], in[lane + 128], in[lane + 192]};
  v4i b = {in[lane + 256], in[lane + 320], in[lane + 384], in[lane + 448]};
  long long t0 = 0, t1 = 0;
  if constexpr (BIG) {
    v16i acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = (v16i){0};
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
    t1 = __builtin_amdgcn_s_memtime();
    int s = 0;
    for (int i = 0; i < 8; ++i) for (int r = 0; r < 16; ++r) s += acc[i][r];
    out[blockIdx.x * 64 + lane] = s;
  } else {
    v4acc acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = (v4acc){0};
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[i], 0, 0, 0);
    t1 = __builtin_amdgcn_s_memtime();
    int s = 0;
    for (int i = 0; i < 8; ++i) for (int r = 0; r < 4; ++r) s += acc[i][r];
    out[blockIdx.x * 64 + lane] = s;
  }
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  int *din, *dout; long long* dc;
  (void)hipMalloc(&din, 512 * 4); (void)hipMalloc(&dout, 1024 * 64 * 4); (void)hipMalloc(&dc, 1024 * 8);
  int h[512];
  unsigned s = 1;
  for (int i = 0; i < 512; ++i) { s = s * 1103515245u + 12345u; h[i] = (int)s; }
  (void)hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  const int iters = 4096;
  for (int big = 1; big >= 0; --big) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0);
      // one wave per workgroup, 1024 workgroups = one wave per SIMD on 256 CUs
      if (big) hipLaunchKernelGGL(k<1>, dim3(1024), dim3(64), 0, 0, din, dout, dc, iters);
      else hipLaunchKernelGGL(k<0>, dim3(1024), dim3(64), 0, 0, din, dout, dc, iters);
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      long long c[1024]; (void)hipMemcpy(c, dc, sizeof c, hipMemcpyDeviceToHost);
      double avg = 0; for (int i = 0; i < 1024; ++i) avg += c[i]; avg /= 1024;
      const double n = (double)iters * 8;
      const double ops = 2.0 * (big ? 32768 : 16384) * n * 1024;
      printf("%s: %.2f cycles/MFMA (s_memtime), %.3f ms, %.0f TOP/s (1 wave/SIMD, 1024 waves)\n",
             big ? "mfma_i32_32x32x32_i8" : "mfma_i32_16x16x64_i8", avg / n, ms, ops / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
