// Diagnostic: per-workgroup phase timing of the int8 conv kernels (patch
// staging / MFMA main loop / epilogue) with s_memtime stamps, on random data.
// Build + run on the box (from the repo root):
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -DQCN_STAMPS \
//     -Iinclude -Iconvnet-quantization_amd/csrc tools/micro/conv_stamp.hip -o /tmp/conv_stamp
//   /tmp/conv_stamp
#include "../../convnet-quantization_amd/csrc/conv3x3.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static void run(int cin, int cout, int hw, int pool, int nimg) {
  const long nin = (long)nimg * hw * hw * cin;
  const int oh = pool ? hw / 2 : hw;
  const long nout = (long)nimg * oh * oh * cout;
  std::vector<uint8_t> hx(nin);
  std::vector<int8_t> hw8((long)cout * cin * 9), hp(9L * cin * cout);
  std::vector<int32_t> wsum(cout), corr(cout);
  std::vector<float> u(cout, 0.5f), v(cout, 1.0f), mult(cout, 1e-3f);
  unsigned s = 12345;
  for (auto& e : hx) { s = s * 1103515245u + 12345u; e = (uint8_t)(s >> 16); }
  for (auto& e : hw8) { s = s * 1103515245u + 12345u; e = (int8_t)(s >> 16); }
  qcn_pack_conv3x3_weight(hw8.data(), cout, cin, hp.data(), wsum.data());
  for (int i = 0; i < cout; ++i) corr[i] = (128 - 3) * wsum[i];
  uint8_t *dx, *dy; int8_t* dw; float *du, *dv, *dm; int* dc;
  CK(hipMalloc(&dx, nin)); CK(hipMalloc(&dy, nout)); CK(hipMalloc(&dw, hp.size()));
  CK(hipMalloc(&du, cout * 4)); CK(hipMalloc(&dv, cout * 4)); CK(hipMalloc(&dm, cout * 4));
  CK(hipMalloc(&dc, cout * 4));
  CK(hipMemcpy(dx, hx.data(), nin, hipMemcpyHostToDevice));
  CK(hipMemcpy(dw, hp.data(), hp.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(du, u.data(), cout * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dv, v.data(), cout * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dm, mult.data(), cout * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc, corr.data(), cout * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 20; ++i)
    qcn_conv3x3_u8s8_nhwc(dx, nimg, hw, hw, cin, 3, dw, cout, du, dv, dm, dc, 0, 1, pool, nullptr, dy, 0);
  CK(hipEventRecord(e0));
  const int iters = 50;
  for (int i = 0; i < iters; ++i)
    qcn_conv3x3_u8s8_nhwc(dx, nimg, hw, hw, cin, 3, dw, cout, du, dv, dm, dc, 0, 1, pool, nullptr, dy, 0);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  // one more launch for clean stamps
  static unsigned long long zero[1 << 16][8];
  CK(hipMemcpyToSymbol(HIP_SYMBOL(qcn_stamps), zero, sizeof(zero)));
  qcn_conv3x3_u8s8_nhwc(dx, nimg, hw, hw, cin, 3, dw, cout, du, dv, dm, dc, 0, 1, pool, nullptr, dy, 0);
  CK(hipDeviceSynchronize());
  static unsigned long long st[1 << 16][8];
  CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(qcn_stamps), sizeof(st)));
  const long pxb_total = (long)nimg * hw * hw;
  // workgroup count: derive from the config used by the dispatcher
  int nwg = 0;
  for (int b = 0; b < (1 << 16); ++b) if (st[b][0]) nwg = b + 1;
  unsigned long long r0 = ~0ull, r1 = 0;
  double pro = 0, main = 0, epi = 0, clk = 0, q1 = 0, q2 = 0, q3 = 0;
  std::vector<double> starts, ends;
  for (int b = 0; b < nwg; ++b) {
    r0 = std::min(r0, st[b][6]); r1 = std::max(r1, st[b][7]);
    pro += st[b][1] - st[b][0]; main += st[b][2] - st[b][1]; epi += st[b][5] - st[b][2];
    q1 += st[b][3] - st[b][2]; q2 += st[b][4] - st[b][3]; q3 += st[b][5] - st[b][4];
    clk += (double)(st[b][5] - st[b][0]) / ((double)(st[b][7] - st[b][6]) * 10.0);
  }
  clk /= nwg;
  for (int b = 0; b < nwg; ++b) {
    starts.push_back((double)(st[b][6] - r0) * 10.0);
    ends.push_back((double)(st[b][7] - r0) * 10.0);
  }
  std::sort(starts.begin(), starts.end());
  std::sort(ends.begin(), ends.end());
  const double rspan = (double)(r1 - r0) * 10.0;  // ns
  const double macs = (double)pxb_total * cout * cin * 9;
  const double mfma_cyc = macs / 32768.0 * 32.0 / 1024.0;  // per SIMD at 32 cyc/MFMA
  printf("conv %d->%d @%d pool=%d  n=%d: %.2f us/launch (events), %.1f TOP/s; nwg=%d\n", cin, cout, hw,
         pool, nimg, ms * 1e3, 2 * macs / (ms * 1e-3) / 1e12, nwg);
  printf("  stamped launch: first start -> last end %.2f us; WG clock %.2f GHz; ideal MFMA cyc/SIMD %.0f = %.2f us\n",
         rspan / 1e3, clk, mfma_cyc, mfma_cyc / clk / 1e3);
  printf("  per-WG avg cycles: prologue %.0f  mainloop %.0f  epilogue %.0f (requant+stage %.0f, sync %.0f, store %.0f)\n",
         pro / nwg, main / nwg, epi / nwg, q1 / nwg, q2 / nwg, q3 / nwg);
  printf("  WG start (ns) pct 0/25/50/75/90/100: %.0f %.0f %.0f %.0f %.0f %.0f\n", starts[0],
         starts[nwg / 4], starts[nwg / 2], starts[3 * nwg / 4], starts[9 * nwg / 10], starts[nwg - 1]);
  printf("  WG end   (ns) pct 0/25/50/75/90/100: %.0f %.0f %.0f %.0f %.0f %.0f\n", ends[0],
         ends[nwg / 4], ends[nwg / 2], ends[3 * nwg / 4], ends[9 * nwg / 10], ends[nwg - 1]);
  CK(hipFree(dx)); CK(hipFree(dy)); CK(hipFree(dw)); CK(hipFree(du)); CK(hipFree(dv));
  CK(hipFree(dm)); CK(hipFree(dc));
}

int main() {
  const int n = 1024;
  run(64, 128, 16, 0, n);   // conv3
  run(128, 128, 16, 1, n);  // conv4
  run(128, 256, 8, 0, n);   // conv5
  run(256, 256, 8, 1, n);   // conv6
  return 0;
}
