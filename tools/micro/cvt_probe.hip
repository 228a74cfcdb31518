// Probe: rounding / saturation of v_cvt_pk_u8_f32 on gfx950 (is it RNE with
// [0,255] saturation?  What do NaN / inf / huge values give?).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>
__global__ void k(const float* x, unsigned* y, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = __builtin_amdgcn_cvt_pk_u8_f32(x[i], 0, 0u) & 0xff;
}
int main() {
  std::vector<float> v = {-1e30f, -256.f, -1.f, -0.75f, -0.5f, -0.4f, -0.f, 0.f, 0.25f, 0.5f, 0.75f, 1.f,
                          1.5f, 2.5f, 3.5f, 126.5f, 127.5f, 253.5f, 254.5f, 254.6f, 255.f, 255.4f, 255.5f,
                          255.6f, 256.f, 300.f, 1e10f, INFINITY, -INFINITY, NAN, 0.49999997f, 1.4999999f,
                          2.5000002f};
  // exhaustive-ish: every k/8 in [-4, 260]
  for (int t = -32; t <= 260 * 8; ++t) v.push_back(t / 8.0f);
  const int n = (int)v.size();
  float* dx; unsigned* dy;
  hipMalloc(&dx, n * 4); hipMalloc(&dy, n * 4);
  hipMemcpy(dx, v.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dy, n);
  std::vector<unsigned> y(n);
  hipMemcpy(y.data(), dy, n * 4, hipMemcpyDeviceToHost);
  int bad_rne = 0, bad_trunc = 0;
  for (int i = 0; i < n; ++i) {
    const float f = v[i];
    float r = std::nearbyint(f);  // host default rounding = RNE
    if (std::isnan(f)) r = 0;
    r = r < 0 ? 0 : (r > 255 ? 255 : r);
    float t = std::trunc(f);
    if (std::isnan(f)) t = 0;
    t = t < 0 ? 0 : (t > 255 ? 255 : t);
    if ((unsigned)r != y[i]) ++bad_rne;
    if ((unsigned)t != y[i]) ++bad_trunc;
    if (i < 33) printf("%14.8g -> %u\n", f, y[i]);
  }
  printf("mismatches vs clamp(rne): %d, vs clamp(trunc): %d of %d\n", bad_rne, bad_trunc, n);
  return 0;
}
