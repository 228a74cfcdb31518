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
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <class F>
static void report(const char* title, double macs, F launch) {
  hipEvent_t ev0, ev1;
  CK(hipEventCreate(&ev0)); CK(hipEventCreate(&ev1));
  for (int i = 0; i < 20; ++i) launch();
  CK(hipEventRecord(ev0));
  const int iters = 50;
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(ev1));
  CK(hipEventSynchronize(ev1));
  float ms; CK(hipEventElapsedTime(&ms, ev0, ev1));
  ms /= iters;
  static unsigned long long zero[1 << 16][8], st[1 << 16][8];
  CK(hipMemcpyToSymbol(HIP_SYMBOL(qcn_stamps), zero, sizeof(zero)));
  launch();
  CK(hipDeviceSynchronize());
  CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(qcn_stamps), sizeof(st)));
  int nwg = 0;
  for (int b = 0; b < 4096; ++b) if (st[b][0]) nwg = b + 1;
  {
    double a = 0, b2 = 0; int cnt = 0;
    for (int b = 4096; b < 4096 + nwg; ++b) if (st[b][1]) { a += st[b][0]; b2 += st[b][1]; ++cnt; }
    if (cnt) printf("  producer per WG: stage_load %.0f, conv1 %.0f cycles\n", a / cnt, b2 / cnt);
    double w0 = 0, w1 = 0, e0 = 0, e1 = 0; cnt = 0;
    for (int b = 8192; b < 8192 + nwg; ++b) if (st[b][2]) { w0 += st[b][0]; w1 += st[b][1]; e0 += st[b][2]; e1 += st[b][3]; ++cnt; }
    if (cnt) printf("  tile loop per WG: consumer wait %.0f of %.0f, producer wait %.0f of %.0f cycles\n",
                    w0 / cnt, e0 / cnt, w1 / cnt, e1 / cnt);
  }
  if (nwg == 0) {
    printf("%s: %.2f us/launch (events), %.1f TOP/s (no stamps)\n", title, ms * 1e3,
           2 * macs / (ms * 1e-3) / 1e12);
    return;
  }
  unsigned long long r0 = ~0ull, r1 = 0;
  double ph[5] = {0, 0, 0, 0, 0}, clk = 0;
  std::vector<double> starts, ends;
  for (int b = 0; b < nwg; ++b) {
    r0 = std::min(r0, st[b][6]); r1 = std::max(r1, st[b][7]);
    for (int k = 0; k < 5; ++k) ph[k] += (double)(st[b][k + 1] - st[b][k]);
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
  const double mfma_cyc = macs / 32768.0 * 32.0 / 1024.0;  // per SIMD at 32 cyc/MFMA
  printf("%s: %.2f us/launch (events), %.1f TOP/s; nwg=%d\n", title, ms * 1e3,
         2 * macs / (ms * 1e-3) / 1e12, nwg);
  printf("  stamped launch: %.2f us; WG clock %.2f GHz; ideal MFMA cyc/SIMD %.0f = %.2f us\n",
         rspan / 1e3, clk, mfma_cyc, mfma_cyc / clk / 1e3);
  printf("  per-WG avg cycles: stage %.0f | pre-mfma %.0f | mainloop %.0f | requant+stage+sync %.0f | store %.0f\n",
         ph[0] / nwg, ph[1] / nwg, ph[2] / nwg, ph[3] / nwg, ph[4] / nwg);
  printf("  WG start (ns) pct 0/25/50/75/90/100: %.0f %.0f %.0f %.0f %.0f %.0f\n", starts[0],
         starts[nwg / 4], starts[nwg / 2], starts[3 * nwg / 4], starts[9 * nwg / 10], starts[nwg - 1]);
  printf("  WG end   (ns) pct 0/25/50/75/90/100: %.0f %.0f %.0f %.0f %.0f %.0f\n", ends[0],
         ends[nwg / 4], ends[nwg / 2], ends[3 * nwg / 4], ends[9 * nwg / 10], ends[nwg - 1]);
  // per XCD (workgroup b on XCD b % 8): mean workgroup duration, mean clock,
  // last end
  printf("  per XCD: mean WG us | GHz | last end us:");
  for (int x = 0; x < 8; ++x) {
    double d = 0, g = 0, e = 0; int c = 0;
    for (int b = x; b < nwg; b += 8) {
      const double rt = (double)(st[b][7] - st[b][6]) * 10.0;
      d += rt; g += (double)(st[b][5] - st[b][0]) / rt;
      e = std::max(e, (double)(st[b][7] - r0) * 10.0); ++c;
    }
    if (c) printf("  [%d] %.1f %.2f %.1f", x, d / c / 1e3, g / c, e / 1e3);
  }
  printf("\n");
}

static unsigned rng = 12345;
static int8_t r8() { rng = rng * 1103515245u + 12345u; return (int8_t)(rng >> 16); }

template <class T>
static T* up(const std::vector<T>& h) {
  T* d; CK(hipMalloc(&d, h.size() * sizeof(T)));
  CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

static void run(int cin, int cout, int hw, int pool, int nimg) {
  const long nin = (long)nimg * hw * hw * cin;
  const int oh = pool ? hw / 2 : hw;
  const long nout = (long)nimg * oh * oh * cout;
  std::vector<uint8_t> hx(nin);
  std::vector<int8_t> hw8((long)cout * cin * 9), hp(9L * cin * cout);
  std::vector<int32_t> wsum(cout), corr(cout);
  for (auto& e : hx) e = (uint8_t)r8();
  for (auto& e : hw8) e = r8();
  qcn_pack_conv3x3_weight(hw8.data(), cout, cin, hp.data(), wsum.data());
  for (int i = 0; i < cout; ++i) corr[i] = (128 - 3) * wsum[i];
  uint8_t* dx = up(hx); int8_t* dw = up(hp); int* dc = up(corr);
  float* du = up(std::vector<float>(cout, 0.5f)); float* dv = up(std::vector<float>(cout, 1.0f));
  float* dm = up(std::vector<float>(cout, 1e-3f));
  uint8_t* dy; CK(hipMalloc(&dy, nout));
  char title[128];
  snprintf(title, sizeof title, "conv %d->%d @%d pool=%d n=%d", cin, cout, hw, pool, nimg);
  report(title, (double)nimg * hw * hw * cout * cin * 9, [&] {
    qcn_conv3x3_u8s8_nhwc(dx, nimg, hw, hw, cin, 3, dw, cout, du, dv, dm, dc, 0, 1, pool, nullptr, dy, 0);
  });
  CK(hipFree(dx)); CK(hipFree(dy)); CK(hipFree(dw)); CK(hipFree(du)); CK(hipFree(dv));
  CK(hipFree(dm)); CK(hipFree(dc));
}

static void run12(int nimg) {
  std::vector<float> hx((long)nimg * 3 * 32 * 32);
  for (auto& e : hx) e = r8() / 64.0f;
  std::vector<int8_t> w1((long)64 * 27), w1p(64 * 32), w2(64L * 64 * 9), w2p(64L * 64 * 9);
  for (auto& e : w1) e = r8();
  for (auto& e : w2) e = r8();
  std::vector<int32_t> s1(64), s2(64), c1(64), c2(64);
  qcn_pack_conv1_weight(w1.data(), 64, w1p.data(), s1.data());
  qcn_pack_conv3x3_weight(w2.data(), 64, 64, w2p.data(), s2.data());
  for (int i = 0; i < 64; ++i) { c1[i] = (128 - 7) * s1[i]; c2[i] = 128 * s2[i]; }
  float* dx = up(hx); int8_t* dw1 = up(w1p); int8_t* dw2 = up(w2p);
  int* dc1 = up(c1); int* dc2 = up(c2);
  float* du = up(std::vector<float>(64, 0.5f)); float* dv = up(std::vector<float>(64, 1.0f));
  float* dm = up(std::vector<float>(64, 1e-3f));
  uint8_t* dy; CK(hipMalloc(&dy, (long)nimg * 16 * 16 * 64));
  report("conv12 fused (3->64->64 @32, pool)", (double)nimg * 1024 * 64 * (27 + 576), [&] {
    qcn_conv12_fused_f32_nchw(dx, nimg, 0.05f, 7, dw1, du, dv, dm, dc1, 0, 1, nullptr, 0, dw2, du, dv,
                              dm, dc2, 0, 1, nullptr, dy, 0);
  });
}

static void runpair(int cin, int cmid, int cout, int hw, int nimg) {
  const long nin = (long)nimg * hw * hw * cin;
  std::vector<uint8_t> hx(nin);
  for (auto& e : hx) e = (uint8_t)r8();
  std::vector<int8_t> wa((long)cmid * cin * 9), wb((long)cout * cmid * 9), pa(wa.size()), pb(wb.size());
  for (auto& e : wa) e = r8();
  for (auto& e : wb) e = r8();
  std::vector<int32_t> sa(cmid), sb(cout), ca(cmid), cb(cout);
  qcn_pack_conv3x3_weight(wa.data(), cmid, cin, pa.data(), sa.data());
  qcn_pack_conv3x3_weight(wb.data(), cout, cmid, pb.data(), sb.data());
  for (int i = 0; i < cmid; ++i) ca[i] = (128 - 3) * sa[i];
  for (int i = 0; i < cout; ++i) cb[i] = 128 * sb[i];
  uint8_t* dx = up(hx); int8_t* dwa = up(pa); int8_t* dwb = up(pb); int* dca = up(ca); int* dcb = up(cb);
  float* dua = up(std::vector<float>(cmid, 0.5f)); float* dva = up(std::vector<float>(cmid, 1.0f));
  float* dma = up(std::vector<float>(cmid, 1e-3f));
  float* dub = up(std::vector<float>(cout, 0.5f)); float* dvb = up(std::vector<float>(cout, 1.0f));
  float* dmb = up(std::vector<float>(cout, 1e-3f));
  uint8_t* dy; CK(hipMalloc(&dy, (long)nimg * hw * hw / 4 * cout));
  char title[128];
  snprintf(title, sizeof title, "pair %d->%d->%d @%d (pool) n=%d  [stage|A|A-epi|B|B-epi]", cin, cmid, cout, hw, nimg);
  report(title, (double)nimg * hw * hw * (cmid * cin + cout * cmid) * 9, [&] {
    qcn_conv3x3_pair_u8s8(dx, nimg, hw, cin, 3, dwa, cmid, dua, dva, dma, dca, 0, 1, nullptr, dwb, cout,
                          dub, dvb, dmb, dcb, 0, 1, nullptr, 0, dy, 0);
  });
}

int main() {
  if (const char* e = getenv("QCN_SWEEP12")) {   // conv12 launch time vs batch
    (void)e;
    for (int nb : {256, 512, 1024, 2048, 4096, 8192}) run12(nb);
    return 0;
  }
  const int n = 1024;
  runpair(64, 128, 128, 16, n);
  runpair(128, 256, 256, 8, n);
  run12(n);
  run(64, 128, 16, 0, n);   // conv3
  run(128, 128, 16, 1, n);  // conv4
  run(128, 256, 8, 0, n);   // conv5
  run(256, 256, 8, 1, n);   // conv6
  return 0;
}
