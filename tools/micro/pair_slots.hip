// Diagnostic: where do the pair kernel's workgroups run (XCC / SE / CU /
// workgroup slot, from HW_ID) and when, relative to their co-resident
// partner?  Tests the lockstep hypothesis of DESIGN §5 (the lead-sleep knob
// QCN_PAIR_SLEEP it was first run with is gone from the kernel).  Build + run on the box (repo root):
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -DQCN_STAMPS \
//     -Iinclude -Iconvnet-quantization_amd/csrc tools/micro/pair_slots.hip -o /tmp/pair_slots
//   QCN_PAIR_SLEEP=8 /tmp/pair_slots 64    (64: conv3+conv4; 128: conv5+conv6)
#include "../../convnet-quantization_amd/csrc/conv3x3.hip"
#include <algorithm>
#include <cstdio>
#include <map>
#include <tuple>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static uint32_t rs = 12345;
static int8_t r8() { rs = rs * 1664525u + 1013904223u; return (int8_t)(rs >> 24); }
template <class T> static T* up(const std::vector<T>& h) {
  T* d; CK(hipMalloc(&d, h.size() * sizeof(T)));
  CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  const int cin = argc > 1 ? atoi(argv[1]) : 64;
  const int cmid = 2 * cin, cout = cmid, hw = cin == 64 ? 16 : 8, nimg = 1024;
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
  auto launch = [&] {
    qcn_conv3x3_pair_u8s8(dx, nimg, hw, cin, 3, dwa, cmid, dua, dva, dma, dca, 0, 1, nullptr, dwb, cout,
                          dub, dvb, dmb, dcb, 0, 1, nullptr, 0, dy, 0);
  };
  for (int i = 0; i < 200; ++i) launch();   // warm, let the clock settle
  static unsigned long long zero[1 << 16][8], st[1 << 16][8];
  CK(hipDeviceSynchronize());
  CK(hipMemcpyToSymbol(HIP_SYMBOL(qcn_stamps), zero, sizeof(zero)));
  launch();
  CK(hipDeviceSynchronize());
  CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(qcn_stamps), sizeof(st)));
  const int nwg = nimg * hw * hw / 256;
  unsigned long long r0 = ~0ull;
  for (int b = 0; b < nwg; ++b) r0 = std::min(r0, st[b][6]);
  // per CU: (start_ns, end_ns, slot, block, phase stamps)
  std::map<std::tuple<int, int, int, int>, std::vector<int>> cus;
  std::map<int, int> slots;
  for (int b = 0; b < nwg; ++b) {
    const unsigned hid = (unsigned)st[16384 + b][0], xcc = (unsigned)st[16384 + b][1] & 0xf;
    const int cu = (hid >> 8) & 15, sh = (hid >> 12) & 1, se = (hid >> 13) & 7, slot = (hid >> 16) & 15;
    cus[{(int)xcc, se, sh, cu}].push_back(b);
    slots[slot]++;
  }
  printf("cin %d: %d workgroups on %zu CUs; slot histogram:", cin, nwg, cus.size());
  for (auto& kv : slots) printf(" %d:%d", kv.first, kv.second);
  printf("\n");
  // lockstep measure: for each CU, the two earliest-starting WGs; offset of
  // their A-main-loop start and of their B-main-loop start (s_memtime cycles)
  std::vector<double> d_start, d_a, d_b;
  int shown = 0;
  for (auto& kv : cus) {
    auto v = kv.second;
    std::sort(v.begin(), v.end(), [&](int a, int b) { return st[a][6] < st[b][6]; });
    if (shown < 6) {
      printf("CU x%d se%d sh%d cu%d:", std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first),
             std::get<3>(kv.first));
      for (int b : v) {
        const unsigned hid = (unsigned)st[16384 + b][0];
        printf("  [b%d s%d %.2f-%.2f us | A@%llu B@%llu]", b, (hid >> 16) & 15, (st[b][6] - r0) * 0.01,
               (st[b][7] - r0) * 0.01, st[b][1] - st[b][0], st[b][3] - st[b][0]);
      }
      printf("\n");
      ++shown;
    }
    if (v.size() >= 2) {
      const int a = v[0], b = v[1];
      d_start.push_back(((double)st[b][6] - (double)st[a][6]) * 10.0);
      d_a.push_back((double)st[b][1] - (double)st[a][1]);
      d_b.push_back((double)st[b][3] - (double)st[a][3]);
    }
    if (v.size() >= 4) {   // second round pair
      const int a = v[2], b = v[3];
      d_start.push_back(((double)st[b][6] - (double)st[a][6]) * 10.0);
    }
  }
  auto pct = [](std::vector<double> v, const char* name) {
    if (v.empty()) return;
    std::sort(v.begin(), v.end());
    printf("%s pct 10/50/90: %.0f %.0f %.0f\n", name, v[v.size() / 10], v[v.size() / 2], v[9 * v.size() / 10]);
  };
  pct(d_start, "partner start offset (ns)");
  pct(d_a, "partner A-loop start offset (cyc)");
  pct(d_b, "partner B-loop start offset (cyc)");
  return 0;
}
