// Probe: issue cost (cycles per wave-instruction) of the epilogue's VALU ops on
// gfx950, 8 independent chains, 1 or 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));
template <int OP>
__global__ __launch_bounds__(512) void k(float* out, long long* cyc, int iters) {
  const int lane = threadIdx.x;
  float f[8]; int n[8]; v2f p[8]; unsigned u[8];
  for (int i = 0; i < 8; ++i) { f[i] = lane * 0.37f + i; n[i] = lane * 7 + i; p[i] = (v2f){f[i], f[i] + 1}; u[i] = lane + i; }
  const v2f c1 = {1.0001f, 0.9999f}, c2 = {0.5f, 0.25f};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (OP == 0) f[i] = (float)n[i] + f[i];                       // cvt + add (2 ops)
      if constexpr (OP == 1) p[i] = __builtin_elementwise_fma(p[i], c1, c2);   // pk_fma
      if constexpr (OP == 2) p[i] = p[i] * c1;                                 // pk_mul
      if constexpr (OP == 3) u[i] = __builtin_amdgcn_cvt_pk_u8_f32(f[i], i & 3, u[i]);
      if constexpr (OP == 4) f[i] = __builtin_fmaf(f[i], 1.0001f, 0.5f);       // fma
      if constexpr (OP == 5) { auto s = __builtin_amdgcn_permlane32_swap(u[i], u[(i + 1) & 7], false, false); u[i] = s[0] + 1; }
      if constexpr (OP == 6) f[i] = __builtin_rintf(f[i] * 1.0001f);           // mul + rndne
    }
    asm volatile("" :: "v"(f[0]), "v"(u[0]));
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0; for (int i = 0; i < 8; ++i) s += f[i] + p[i].x + p[i].y + u[i] + n[i];
  out[blockIdx.x * 512 + lane] = s;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  float* o; long long* c; (void)hipMalloc(&o, 1024 * 512 * 4); (void)hipMalloc(&c, 1024 * 8);
  const char* nm[7] = {"cvt_f32_i32+add", "pk_fma_f32", "pk_mul_f32", "cvt_pk_u8_f32", "fma_f32", "permlane32_swap+add", "mul+rndne"};
  const int iters = 4096;
  for (int op = 0; op < 7; ++op)
    for (int wps = 1; wps <= 2; ++wps) {
      auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(256), dim3(256 * wps), 0, 0, o, c, iters); };
      if (op == 0) launch(k<0>); if (op == 1) launch(k<1>); if (op == 2) launch(k<2>);
      if (op == 3) launch(k<3>); if (op == 4) launch(k<4>); if (op == 5) launch(k<5>); if (op == 6) launch(k<6>);
      (void)hipDeviceSynchronize();
      long long h[256]; (void)hipMemcpy(h, c, sizeof h, hipMemcpyDeviceToHost);
      double a = 0; for (int i = 0; i < 256; ++i) a += h[i]; a /= 256;
      printf("%-22s %d wave/SIMD: %.2f cycles per instruction-slot (per wave)\n", nm[op], wps, a / (iters * 8.0));
    }
  return 0;
}
