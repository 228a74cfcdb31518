// Probe: one wave per SIMD, 8 MFMA (32x32x32 i8) per half-step on 8 accumulators,
// with the next half-step's 6 fragments (ds_read_b128) issued (a) not at all,
// (b) as a burst before the MFMAs, (c) interleaved one per MFMA.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
template <int MODE>
__global__ __launch_bounds__(256) void k(int* out, long long* cyc, int iters) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[65536];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 65536 / 4; i += 256) reinterpret_cast<int*>(lds)[i] = i * 2654435761u;
  __syncthreads();
  v16i acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = (v16i){0};
  v4i f0[6], f1[6];
  const int base = wave * 16384 + lane * 16;
  for (int i = 0; i < 6; ++i) f0[i] = *reinterpret_cast<const v4i*>(lds + ((base + i * 1024) & 65535));
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    const int o = (it * 6144) & 16383;
    if constexpr (MODE == 1) {
      for (int i = 0; i < 6; ++i) f1[i] = *reinterpret_cast<const v4i*>(lds + ((base + o + i * 1024) & 65535));
      __builtin_amdgcn_sched_barrier(0);
      for (int m = 0; m < 8; ++m) acc[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(f0[m >> 2], f0[2 + (m & 3)], acc[m], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      for (int i = 0; i < 6; ++i) f0[i] = *reinterpret_cast<const v4i*>(lds + ((base + o + 512 + i * 1024) & 65535));
      __builtin_amdgcn_sched_barrier(0);
      for (int m = 0; m < 8; ++m) acc[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(f1[m >> 2], f1[2 + (m & 3)], acc[m], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    } else if constexpr (MODE == 2) {
      for (int m = 0; m < 8; ++m) {
        if (m < 6) f1[m] = *reinterpret_cast<const v4i*>(lds + ((base + o + m * 1024) & 65535));
        __builtin_amdgcn_sched_barrier(0);
        acc[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(f0[m >> 2], f0[2 + (m & 3)], acc[m], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      for (int m = 0; m < 8; ++m) {
        if (m < 6) f0[m] = *reinterpret_cast<const v4i*>(lds + ((base + o + 512 + m * 1024) & 65535));
        __builtin_amdgcn_sched_barrier(0);
        acc[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(f1[m >> 2], f1[2 + (m & 3)], acc[m], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      for (int m = 0; m < 8; ++m) acc[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(f0[m >> 2], f0[2 + (m & 3)], acc[m], 0, 0, 0);
      for (int m = 0; m < 8; ++m) acc[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(f0[m >> 2], f0[2 + (m & 3)], acc[m], 0, 0, 0);
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  int s = 0;
  for (int i = 0; i < 8; ++i) for (int r = 0; r < 16; ++r) s ^= acc[i][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  int* dout; long long* dc;
  (void)hipMalloc(&dout, 256 * 256 * 4); (void)hipMalloc(&dc, 256 * 8);
  const int iters = 2048;
  const char* names[3] = {"no LDS reads", "6 reads burst / 8 MFMA", "6 reads interleaved / 8 MFMA"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(256), 0, 0, dout, dc, iters);
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(256), dim3(256), 0, 0, dout, dc, iters);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(256), dim3(256), 0, 0, dout, dc, iters);
      (void)hipDeviceSynchronize();
      long long c[256]; (void)hipMemcpy(c, dc, sizeof c, hipMemcpyDeviceToHost);
      double avg = 0; for (int i = 0; i < 256; ++i) avg += c[i]; avg /= 256;
      printf("%-32s: %.1f cycles per MFMA\n", names[mode], avg / (iters * 16.0));
    }
  }
  return 0;
}
