// Probe (r05): what sets the dispatch ramp of a one-workgroup-per-CU
// persistent launch?  The one-launch convs start their last of 256
// workgroups 3.5-4.5 us after the first (DESIGN §9 'Dispatch skew'), against
// 0.34-0.69 us for 1024 light workgroups (MI355X_MICROARCH.md).  Each
// variant: 256 workgroups, every wave stamps s_memrealtime at entry, then the
// workgroup spins ~20 us; reported: spread of the workgroup start times
// (first wave of each) and of their last-wave start, in us.
// Variants: threads per workgroup (256 / 512), dynamic LDS (0 / 64 / 160 KiB),
// VGPRs per wave (~64 / 256, via an asm clobber list) and scratch use.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

template <int BIGV, int SCR>
__global__ __launch_bounds__(512, 1) void k(unsigned long long* st, int spin_ticks, int* sink, int ldsb) {
  extern __shared__ int lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const int lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int wave = threadIdx.x >> 6;
  if (lane == 0) st[(blockIdx.x * 8 + wave)] = t0 + lane;
  if constexpr (BIGV) {   // occupy ~256 VGPRs
    asm volatile("" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12",
                 "v13", "v14", "v15", "v200", "v240", "v250", "v255");
  }
  int acc = 0;
  if constexpr (SCR) {
    volatile int buf[64];
    for (int i = 0; i < 64; ++i) buf[i] = i + threadIdx.x;
    acc += buf[threadIdx.x & 63];
  }
  if (threadIdx.x < 16 && ldsb > 0) lds[threadIdx.x] = acc;
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin_ticks) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0) sink[blockIdx.x] = acc + (ldsb > 0 ? lds[0] : 0);
}

template <int BIGV, int SCR>
static void run(const char* name, int threads, int ldsb, unsigned long long* d, int* sink) {
  const int nwg = 256;
  if (ldsb > 65536) (void)hipFuncSetAttribute((const void*)k<BIGV, SCR>, hipFuncAttributeMaxDynamicSharedMemorySize, ldsb);
  std::vector<double> spreads, lastw;
  for (int rep = 0; rep < 6; ++rep) {
    (void)hipMemset(d, 0, nwg * 8 * 8);
    hipLaunchKernelGGL((k<BIGV, SCR>), dim3(nwg), dim3(threads), ldsb, 0, d, 2000 /* 20 us */, sink, ldsb);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(nwg * 8);
    (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    const int wpg = threads / 64;
    unsigned long long mn = ~0ull, mx = 0, mxl = 0;
    for (int b = 0; b < nwg; ++b) {
      unsigned long long f = ~0ull, l = 0;
      for (int w = 0; w < wpg; ++w) { f = std::min(f, h[b * 8 + w]); l = std::max(l, h[b * 8 + w]); }
      mn = std::min(mn, f); mx = std::max(mx, f); mxl = std::max(mxl, l);
    }
    if (rep > 0) { spreads.push_back((mx - mn) / 100.0); lastw.push_back((mxl - mn) / 100.0); }
  }
  std::sort(spreads.begin(), spreads.end());
  std::sort(lastw.begin(), lastw.end());
  printf("%-40s start spread median %.2f us (min %.2f), last wave %.2f us\n", name, spreads[spreads.size() / 2],
         spreads[0], lastw[lastw.size() / 2]);
  fflush(stdout);
}

int main() {
  unsigned long long* d;
  int* sink;
  (void)hipMalloc(&d, 256 * 8 * 8);
  (void)hipMalloc(&sink, 256 * 4);
  run<1, 0>("512 thr, 160 KiB LDS, 256 VGPR", 512, 160 * 1024, d, sink);
  run<1, 0>("512 thr, 160 KiB LDS, 256 VGPR", 512, 160 * 1024, d, sink);
  run<1, 0>("512 thr,  64 KiB LDS, 256 VGPR", 512, 64 * 1024, d, sink);
  run<1, 0>("512 thr,   0 KiB LDS, 256 VGPR", 512, 0, d, sink);
  run<0, 0>("512 thr, 160 KiB LDS,  ~40 VGPR", 512, 160 * 1024, d, sink);
  run<0, 0>("512 thr,   0 KiB LDS,  ~40 VGPR", 512, 0, d, sink);
  run<1, 1>("512 thr, 160 KiB LDS, 256 VGPR, scratch", 512, 160 * 1024, d, sink);
  run<1, 0>("256 thr, 160 KiB LDS, 256 VGPR", 256, 160 * 1024, d, sink);
  run<0, 0>("256 thr,   0 KiB LDS,  ~40 VGPR", 256, 0, d, sink);
  return 0;
}
