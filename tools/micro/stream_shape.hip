// Probe: HBM rate of the ResNet 64->256 1x1 conv's memory traffic (read
// x[npix][64], read r[npix][256], write y[npix][256]; 925 MB at batch 512,
// 56x56) under two per-instruction access shapes, no compute:
//   lane-pixel : a wave instruction covers 32 pixel rows x 32 B (lane (p, hi)
//                -> 16 B of row p), the MFMA-output layout after the
//                permlane swap (the streaming conv kernel)
//   row-contig : a wave instruction covers 8 rows x 128 B (16 lanes per
//                256-B row: whole lines), the LDS-staged layout of the tiled
//                kernel
// and two grid forms: one 32-pixel strip x 32 channels per wave (many
// workgroups), or persistent waves looping over strips.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int NPIX = 512 * 56 * 56;
constexpr int CI = 64, CO = 256;

// one wave = (strip of 32 pixels, 32-channel tile)
template <int SHAPE>
__device__ __forceinline__ void unit(const uint8_t* x, const uint8_t* r, uint8_t* y, int strip, int ct, int lane) {
  const int l32 = lane & 31, hi = lane >> 5;
  if constexpr (SHAPE == 0) {
    const long p = (long)strip * 32 + l32;
    const v4i a = *reinterpret_cast<const v4i*>(x + p * CI + hi * 16);
    const v4i b = *reinterpret_cast<const v4i*>(x + p * CI + 32 + hi * 16);
    const v4i c = *reinterpret_cast<const v4i*>(r + p * CO + ct * 32 + hi * 16);
    *reinterpret_cast<v4i*>(y + p * CO + ct * 32 + hi * 16) = a ^ b ^ c;
  } else {
    // the same bytes: x rows of the strip (2 KB), r/y: 32 rows x 32 B of the
    // tile — regrouped so that one instruction covers 8 rows x 128 B of the
    // 4-tile (128-channel) block this wave's tile belongs to
    const int ctb = ct & ~3, sub = ct & 3;   // 4 tiles share a 128-B line
    const long p0 = (long)strip * 32;
    const v4i a = *reinterpret_cast<const v4i*>(x + p0 * CI + lane * 16);
    const v4i b = *reinterpret_cast<const v4i*>(x + p0 * CI + 1024 + lane * 16);
    const int row = sub * 8 + lane / 8, col = (lane % 8) * 16;
    const long off = (p0 + row) * CO + ctb * 32 + col;
    const v4i c = *reinterpret_cast<const v4i*>(r + off);
    *reinterpret_cast<v4i*>(y + off) = a ^ b ^ c;
  }
}

template <int SHAPE>
__global__ __launch_bounds__(256) void k_grid(const uint8_t* x, const uint8_t* r, uint8_t* y) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int u = blockIdx.x * 4 + wave;   // unit = strip * 8 + ct
  unit<SHAPE>(x, r, y, u >> 3, u & 7, lane);
}

template <int SHAPE>
__global__ __launch_bounds__(256) void k_pers(const uint8_t* x, const uint8_t* r, uint8_t* y, int nunits) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int u = blockIdx.x * 4 + wave; u < nunits; u += gridDim.x * 4) unit<SHAPE>(x, r, y, u >> 3, u & 7, lane);
}

int main() {
  uint8_t *x, *r, *y;
  (void)hipMalloc(&x, (size_t)NPIX * CI);
  (void)hipMalloc(&r, (size_t)NPIX * CO);
  (void)hipMalloc(&y, (size_t)NPIX * CO);
  (void)hipMemset(x, 1, (size_t)NPIX * CI);
  (void)hipMemset(r, 2, (size_t)NPIX * CO);
  const int nunits = NPIX / 32 * (CO / 32);
  const double bytes = (double)NPIX * (CI + 2 * CO);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    (void)hipEventRecord(e0);
    const int reps = 20;
    for (int i = 0; i < reps; ++i) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    printf("%-28s %.3f ms  %.2f TB/s\n", name, ms, bytes / ms / 1e9);
  };
  run("lane-pixel grid", [&] { hipLaunchKernelGGL(k_grid<0>, dim3(nunits / 4), dim3(256), 0, 0, x, r, y); });
  run("row-contig grid", [&] { hipLaunchKernelGGL(k_grid<1>, dim3(nunits / 4), dim3(256), 0, 0, x, r, y); });
  for (int wg : {512, 1024, 2048}) {
    char n0[64], n1[64];
    snprintf(n0, 64, "lane-pixel pers %d", wg);
    snprintf(n1, 64, "row-contig pers %d", wg);
    run(n0, [&] { hipLaunchKernelGGL(k_pers<0>, dim3(wg), dim3(256), 0, 0, x, r, y, nunits); });
    run(n1, [&] { hipLaunchKernelGGL(k_pers<1>, dim3(wg), dim3(256), 0, 0, x, r, y, nunits); });
  }
  return 0;
}
