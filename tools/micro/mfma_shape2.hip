// Probe (r05): int8 MFMA shape under DVFS, with clean code generation.
// r01's probe (mfma_shape.hip) compiled the 16x16x64 loop with ~90
// v_accvgpr_mov per 32 MFMAs (loop-carried accumulator shuffles), so its
// "2x the cycles" was the compiler, not the matrix pipe.  Here each step's
// kernels are register-bounded to 256 (no AGPR split), and the loop body is checked
// for accvgpr moves in the disassembly before running.
//
// Same 64 x 128 output tile per wave, same LDS bytes per MAC:
//   32x32x32: 2 x 4 blocks, per 64-K step 4 A + 8 B ds_read_b128, 16 MFMAs
//   16x16x64: 4 x 8 blocks, per 64-K step 4 A + 8 B ds_read_b128, 32 MFMAs
// and register-only forms (operands fixed in registers, no LDS reads).
// Reports TOP/s, cycles per 64-K step and the in-kernel clock.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

#define PIN(x) do {} while (0)

template <int BIG, int LDSRD, int WPS>
__global__ __launch_bounds__(256 * WPS, 2 / WPS) void k(const int* in, int* out, long long* clk, int iters) {
  __shared__ __attribute__((aligned(16))) int lds[16384];   // 64 KB of random bytes
  for (int i = threadIdx.x; i < 16384; i += 256 * WPS) lds[i] = in[(i * 7 + blockIdx.x) & 16383];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int* base = lds + ((wave * 1024 + lane * 4) & 16383);
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  int s = 0;
  v4i ra[4], rb[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) ra[i] = *reinterpret_cast<const v4i*>(base + i * 256);
#pragma unroll
  for (int j = 0; j < 8; ++j) rb[j] = *reinterpret_cast<const v4i*>(base + 1024 + j * 256);
  if constexpr (BIG) {
    v16i acc[2][4];
    for (int i = 0; i < 2; ++i) for (int j = 0; j < 4; ++j) acc[i][j] = (v16i){0};
    for (int it = 0; it < iters; ++it) {
      const int o = (it * 1280) & 8191;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        v4i a[2], b[4];
        if constexpr (LDSRD) {
#pragma unroll
          for (int i = 0; i < 2; ++i) a[i] = *reinterpret_cast<const v4i*>(base + ((o + kk * 2048 + i * 256) & 16383));
#pragma unroll
          for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const v4i*>(base + ((o + kk * 2048 + 512 + j * 256) & 16383));
        } else {
#pragma unroll
          for (int i = 0; i < 2; ++i) a[i] = ra[kk * 2 + i];
#pragma unroll
          for (int j = 0; j < 4; ++j) b[j] = rb[kk * 4 + j];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b[j], acc[i][j], 0, 0, 0);
            PIN(acc[i][j]);
          }
      }
    }
    for (int i = 0; i < 2; ++i) for (int j = 0; j < 4; ++j) for (int r = 0; r < 16; ++r) s += acc[i][j][r];
  } else {
    v4i acc[4][8];
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 8; ++j) acc[i][j] = (v4i){0};
    for (int it = 0; it < iters; ++it) {
      const int o = (it * 1280) & 8191;
      v4i a[4], b[8];
      if constexpr (LDSRD) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const v4i*>(base + ((o + i * 256) & 16383));
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = *reinterpret_cast<const v4i*>(base + ((o + 1024 + j * 256) & 16383));
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = ra[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = rb[j];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i], b[j], acc[i][j], 0, 0, 0);
          PIN(acc[i][j]);
        }
    }
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 8; ++j) for (int r = 0; r < 4; ++r) s += acc[i][j][r];
  }
  const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 * WPS + threadIdx.x] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int BIG, int LDSRD, int WPS>
static void run(const char* name, int* din, int* dout, long long* dc, int iters) {
  const int nwg = 256;
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL((k<BIG, LDSRD, WPS>), dim3(nwg), dim3(256 * WPS), 0, 0, din, dout, dc, iters);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  static long long c[2 * 256]; (void)hipMemcpy(c, dc, sizeof c, hipMemcpyDeviceToHost);
  double cyc = 0, ghz = 0;
  for (int i = 0; i < nwg; ++i) { cyc += c[2 * i]; ghz += (double)c[2 * i] / (c[2 * i + 1] * 10.0); }
  cyc /= nwg; ghz /= nwg;
  const double macs = 64.0 * 128 * 64 * iters * 4 * WPS * nwg;   // per wave per step: 64x128x64
  printf("%-28s %7.1f ms  %6.0f TOP/s  clock %.2f GHz  %7.1f cyc per 64-K step per wave\n",
         name, ms, 2 * macs / (ms * 1e-3) / 1e12, ghz, cyc / iters);
  fflush(stdout);
}

int main() {
  int *din, *dout; long long* dc;
  (void)hipMalloc(&din, 16384 * 4); (void)hipMalloc(&dout, 256 * 1024 * 4); (void)hipMalloc(&dc, 256 * 16);
  static int h[16384];
  unsigned s = 1;
  for (int i = 0; i < 16384; ++i) { s = s * 1103515245u + 12345u; h[i] = (int)(s ^ (s >> 13)); }
  (void)hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  const int iters = 1000000;   // ~0.3 s per run
  // warm the clock governor
  run<1, 1, 1>("warm 32x32x32 lds", din, dout, dc, iters);
  for (int rep = 0; rep < 2; ++rep) {
    run<1, 1, 1>("32x32x32 lds  1w/SIMD", din, dout, dc, iters);
    run<0, 1, 1>("16x16x64 lds  1w/SIMD", din, dout, dc, iters);
    run<1, 0, 1>("32x32x32 regs 1w/SIMD", din, dout, dc, iters);
    run<0, 0, 1>("16x16x64 regs 1w/SIMD", din, dout, dc, iters);
    run<1, 1, 2>("32x32x32 lds  2w/SIMD", din, dout, dc, iters / 2);
    run<0, 1, 2>("16x16x64 lds  2w/SIMD", din, dout, dc, iters / 2);
  }
  return 0;
}
