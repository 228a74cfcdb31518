// Diagnostic build (NOT the product): the in-kernel clock the chip holds under
// the SimpleConvNet conv launches, measured as MI355X_MICROARCH.md 'DVFS
// give-back' item 6 prescribes: Δs_memtime ÷ Δs_memrealtime × 100 MHz,
// stamped once around each workgroup's whole body.
//
// This translation unit includes the product's conv3x3.hip unchanged and
// renames its two conv entry points, then defines entry points of the same
// names and signatures that launch STAMPED copies of the same kernels: a
// __global__ wrapper that reads s_memtime / s_memrealtime, runs the product's
// own body function (convpair_body / conv12p_body), passes a workgroup
// barrier and has thread 0 store the four stamps (vector stores into a
// buffer of their own that nothing else reads).  Linked with the product's
// other objects into libqconvnet_clock.so and loaded via QCN_LIB by
// tools/clock_probe.py; the product library never contains a stamp.
// the pipelined conv3+conv4 kernel's own stamps (g_p34_stamp) are compiled in
#define QCN_PIPE34_STAMP 1
// and the one-launch conv1..conv6 kernels' per-phase stamps (g_c16_stamp)
#define QCN_CONVNET_STAMP 1
// and conv12p's per-tile-iteration stamps (g_c12_stamp)
#define QCN_C12_STAMP 1
#define qcn_conv3x3_pair_u8s8 qcn_conv3x3_pair_u8s8__product
#define qcn_conv12_fused_f32_nchw qcn_conv12_fused_f32_nchw__product
#include "conv3x3.hip"
#undef qcn_conv3x3_pair_u8s8
#undef qcn_conv12_fused_f32_nchw

namespace qcn {

constexpr int kClkMaxWg = 4096;
// [kind][workgroup][t0, t1, r0, r1]; kind 0 = conv12, 1 = conv3+4, 2 = conv5+6
__device__ unsigned long long g_qcn_clk[3][kClkMaxWg][4];

QCN_DEV void clk_store(int kind, unsigned long long t0, unsigned long long r0) {
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  // lane 0 of wave 0; the lane id comes from v_mbcnt (a VGPR), so the stored
  // values are per-lane vector data and the stores are plain vector stores
  const unsigned lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if ((threadIdx.x >> 6) == 0 && lane == 0 && blockIdx.x < kClkMaxWg) {
    const unsigned long long v[4] = {t0, t1, r0, r1};
    volatile unsigned long long* d = g_qcn_clk[kind][blockIdx.x];
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = v[i] + lane;
  }
}

template <class CA, class CB>
__global__ __launch_bounds__(CA::NT, CA::WI == 4 ? 1 : 2)
void convpair_stamped(int kind, const uint8_t* __restrict__ x, int nimg, int x_zp,
                      const int8_t* __restrict__ wa, ConvEpi epa, int xb_zp,
                      const int8_t* __restrict__ wb, ConvEpi epb, uint8_t* __restrict__ y) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  convpair_body<CA, CB>((int)blockIdx.x, x, nimg, x_zp, wa, epa, xb_zp, wb, epb, y);
  clk_store(kind, t0, r0);
}

template <class CA, class CB, int D, int COUTB>
__global__ __launch_bounds__(CA::NT, 2)
void convpair_ga_split_stamped(int kind, const uint8_t* __restrict__ x, int nimg, int x_zp,
                               const int8_t* __restrict__ wa, ConvEpi epa, int xb_zp,
                               const int8_t* __restrict__ wb, ConvEpi epb, uint8_t* __restrict__ y) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  convpair_ga_split_body<CA, CB, D, COUTB>((int)blockIdx.x, x, nimg, x_zp, wa, epa, xb_zp, wb, epb, y);
  clk_store(kind, t0, r0);
}

template <class CA, class CB, int D>
__global__ __launch_bounds__(CA::NT, 2)
void convpair_ga_stamped(int kind, const uint8_t* __restrict__ x, int nimg, int x_zp,
                         const int8_t* __restrict__ wa, ConvEpi epa, int xb_zp,
                         const int8_t* __restrict__ wb, ConvEpi epb, uint8_t* __restrict__ y) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  convpair_ga_body<CA, CB, D>((int)blockIdx.x, x, nimg, x_zp, wa, epa, xb_zp, wb, epb, y);
  clk_store(kind, t0, r0);
}

__global__ __launch_bounds__(512, 1)
void conv12p_stamped(const float* __restrict__ x, int nimg, float in_inv, int in_zp,
                     const int8_t* __restrict__ w1, ConvEpi ep1, int x2_zp,
                     const int8_t* __restrict__ w2, ConvEpi ep2, uint8_t* __restrict__ y) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  const int T = (int)blockIdx.x < nimg ? 2 * ((nimg - 1 - (int)blockIdx.x) / (int)gridDim.x + 1) : 0;
  conv12p_body((int)blockIdx.x, (int)gridDim.x, T, x, nimg, in_inv, in_zp, w1, ep1, x2_zp, w2, ep2, y);
  clk_store(0, t0, r0);
}

namespace {
template <class CA, class CB>
int launch_pair_stamped(int kind, const uint8_t* x, int nimg, int x_zp, const int8_t* wa,
                        const ConvEpi& epa, int xb_zp, const int8_t* wb, const ConvEpi& epb,
                        uint8_t* y, hipStream_t st) {
  using P = PairCfg<CA, CB>;
  const long pix = (long)nimg * CA::IMG;
  const int grid = (int)((pix + CA::PXB - 1) / CA::PXB);
  auto k = convpair_stamped<CA, CB>;
  static bool attr_done[QCN_MAX_DEV] = {};
  if (!qcn_set_lds_once((const void*)k, P::LDS, attr_done)) return QCN_ERR_HIP;
  hipLaunchKernelGGL(k, dim3(grid), dim3(CA::NT), P::LDS, st, kind, x, nimg, x_zp, wa, epa, xb_zp,
                     wb, epb, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}
template <class CA, class CB, int D>
int launch_pair_ga_stamped(int kind, const uint8_t* x, int nimg, int x_zp, const int8_t* wa,
                           const ConvEpi& epa, int xb_zp, const int8_t* wb, const ConvEpi& epb,
                           uint8_t* y, hipStream_t st) {
  using P = PairGaCfg<CA, CB>;
  const long pix = (long)nimg * CA::IMG;
  const int grid = (int)((pix + CA::PXB - 1) / CA::PXB);
  auto k = convpair_ga_stamped<CA, CB, D>;
  static bool attr_done[QCN_MAX_DEV] = {};
  if (!qcn_set_lds_once((const void*)k, P::LDS, attr_done)) return QCN_ERR_HIP;
  hipLaunchKernelGGL(k, dim3(grid), dim3(CA::NT), P::LDS, st, kind, x, nimg, x_zp, wa, epa, xb_zp,
                     wb, epb, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}
}  // namespace
}  // namespace qcn

// the last conv3+conv4 / conv5+conv6 launch was the wave-specialised kernel
static bool g_last34_ws = false, g_last56_ws = false;

extern "C" {

// Same signature and shape dispatch as the product's qcn_conv3x3_pair_u8s8.
int qcn_conv3x3_pair_u8s8(const uint8_t* x, int nimg, int hw, int cin, int x_zp,
                          const int8_t* wa_packed, int cmid, const float* ua, const float* va,
                          const float* multa, const int32_t* corra, int zmid, int relua,
                          const qcn_qdq_t* qdqa, const int8_t* wb_packed, int cout, const float* ub,
                          const float* vb, const float* multb, const int32_t* corrb, int y_zp,
                          int relub, const qcn_qdq_t* qdqb, int kmajor, uint8_t* y, void* stream) {
  using namespace qcn;
  ConvEpi epa{ua, va, multa, corra, zmid, relua ? zmid : 0, 0, 0.f, 0, 0.f, 0, 0};
  int xb_zp = zmid;
  if (qdqa) {
    epa.qdq = 1;
    epa.s1 = qdqa->s1; epa.z1 = qdqa->z1; epa.inv2 = qdqa->inv2; epa.z2 = qdqa->z2;
    xb_zp = qdqa->z2;
  }
  ConvEpi epb{ub, vb, multb, corrb, y_zp, relub ? y_zp : 0, 0, 0.f, 0, 0.f, 0, kmajor ? 1 : 0};
  if (qdqb) {
    epb.qdq = 1;
    epb.s1 = qdqb->s1; epb.z1 = qdqb->z1; epb.inv2 = qdqb->inv2; epb.z2 = qdqb->z2;
  }
  hipStream_t st = (hipStream_t)stream;
  // the product's default forms (qcn_conv3x3_pair_u8s8): at <= 1 image per
  // CU conv3+4 on eight waves per image and the cout-split conv5+6
  const int ncu = qcn_cu_count();
  const bool small = ncu > 0 && nimg <= ncu;
  if (hw == 16 && cin == 64 && cmid == 128 && cout == 128) {
    g_last34_ws = nimg >= 2 * ncu;
    if (small)
      return launch_pair_stamped<ConvCfg<64, 128, 16, false, 4, 16, 96, 0, false, 2, 2>,
                                 ConvCfg<128, 128, 16, true, 2, 16, 32, 0, true, 1, 4>>(
          1, x, nimg, x_zp, wa_packed, epa, xb_zp, wb_packed, epb, y, st);
    // the product's wave-specialised kernel, built here with its stamps
    return launch_pair_ws<ConvCfg<64, 128, 16, false, 2, 16, 96, 0, false>,
                          ConvCfg<128, 128, 16, true, 2, 16, 32, 0, true>, kPipeD>(
        x, nimg, x_zp, wa_packed, epa, xb_zp, wb_packed, epb, kmajor != 0, y, st, ncu);
  }
  if (hw == 8 && cin == 128 && cmid == 256 && cout == 256) {
    using A1 = ConvCfg<128, 256, 8, false, 1, 16, 224, 0, false>;
    if (small) {
      using BS = ConvCfg<256, 128, 8, true, 1, 16, 32, 64, true, 1>;
      using P = PairGaCfg<A1, BS>;
      const int grid = (int)(((long)nimg * A1::IMG + A1::PXB - 1) / A1::PXB) * 2;
      auto k = convpair_ga_split_stamped<A1, BS, 4, 256>;
      static bool attr_done[QCN_MAX_DEV] = {};
      if (!qcn_set_lds_once((const void*)k, P::LDS, attr_done)) return QCN_ERR_HIP;
      hipLaunchKernelGGL(k, dim3(grid), dim3(A1::NT), P::LDS, st, 2, x, nimg, x_zp, wa_packed, epa,
                         xb_zp, wb_packed, epb, y);
      return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
    }
    using B1 = ConvCfg<256, 256, 8, true, 1, 16, 32, 64, true>;
    g_last56_ws = nimg >= 4 * ncu;
    if (g_last56_ws)
      return launch_pair_ws<A1, B1, kPipeD>(x, nimg, x_zp, wa_packed, epa, xb_zp, wb_packed, epb,
                                                  kmajor != 0, y, st, ncu);
    return launch_pair_ga_stamped<A1, B1, 4>(2, x, nimg, x_zp, wa_packed, epa, xb_zp, wb_packed, epb, y, st);
  }
  return QCN_ERR_UNSUPPORTED;
}

int qcn_conv12_fused_f32_nchw(const float* x, int nimg, float in_scale, int in_zp,
                              const int8_t* w1_packed, const float* u1, const float* v1,
                              const float* mult1, const int32_t* corr1, int z1, int relu1,
                              const qcn_qdq_t* qdq1, int x2_zp, const int8_t* w2_packed,
                              const float* u2, const float* v2, const float* mult2,
                              const int32_t* corr2, int y_zp, int relu2, const qcn_qdq_t* qdq2,
                              uint8_t* y, void* stream) {
  using namespace qcn;
  ConvEpi ep1{u1, v1, mult1, corr1, z1, relu1 ? z1 : 0, 0, 0.f, 0, 0.f, 0, 0};
  if (qdq1) { ep1.qdq = 1; ep1.s1 = qdq1->s1; ep1.z1 = qdq1->z1; ep1.inv2 = qdq1->inv2; ep1.z2 = qdq1->z2; }
  ConvEpi ep2{u2, v2, mult2, corr2, y_zp, relu2 ? y_zp : 0, 0, 0.f, 0, 0.f, 0, 0};
  if (qdq2) { ep2.qdq = 1; ep2.s1 = qdq2->s1; ep2.z1 = qdq2->z1; ep2.inv2 = qdq2->inv2; ep2.z2 = qdq2->z2; }
  static bool attr_done[QCN_MAX_DEV] = {};
  if (!qcn_set_lds_once((const void*)conv12p_stamped, Conv12P::LDS, attr_done)) return QCN_ERR_HIP;
  const int ncu = qcn_cu_count();
  if (ncu <= 0) return QCN_ERR_HIP;
  const int grid = nimg < ncu ? nimg : ncu;
  hipLaunchKernelGGL(conv12p_stamped, dim3(grid), dim3(512), Conv12P::LDS, (hipStream_t)stream, x,
                     nimg, 1.0f / in_scale, in_zp, w1_packed, ep1, x2_zp, w2_packed, ep2, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

// The one-launch conv1..conv6's stamps of the last launch: [wg][t0..t3, r0..r3]
// (start, after the conv12 phase, after the conv3+4 phase, end).
int qcn_clock_read_c16(unsigned long long* host, int n) {
  if (n <= 0 || n > 4096 || !host) return QCN_ERR_ARG;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(qcn::g_c16_stamp), (size_t)n * 64, 0, hipMemcpyDeviceToHost) ==
                 hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

// the 16x16 pair phases' per-period role stamps of the last launch
// ([wg][phase][role][period 0..7][k 0..2], s_memtime; see g_ws16_stamp)
int qcn_clock_read_ws16(unsigned long long* host, int n) {
  if (n <= 0 || n > 4096 || !host) return QCN_ERR_ARG;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(qcn::g_ws16_stamp), (size_t)n * 2 * 2 * 8 * 3 * 8, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

// conv12p's per-iteration stamps of the last launch: [wg][consumer w0, producer
// w4, producer w5][iteration 0..11][top, before barrier, after conv2's main loop] (s_memtime).
int qcn_clock_read_c12(unsigned long long* host, int n) {
  if (n <= 0 || n > 4096 || !host) return QCN_ERR_ARG;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(qcn::g_c12_stamp), (size_t)n * 3 * 12 * 3 * 8, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

// Copy kind's stamps of the last launch ([wg][t0, t1, r0, r1], n workgroups) to host.
// kind 3: the one-launch conv1..conv6 (whole body).
int qcn_clock_read(int kind, unsigned long long* host, int n) {
  if (kind == 3) {
    if (n <= 0 || n > 4096 || !host) return QCN_ERR_ARG;
    static unsigned long long st[4096][8];
    if (hipMemcpyFromSymbol(st, HIP_SYMBOL(qcn::g_c16_stamp), (size_t)n * 64, 0, hipMemcpyDeviceToHost) !=
        hipSuccess)
      return QCN_ERR_HIP;
    for (int w = 0; w < n; ++w) {
      host[4 * w + 0] = st[w][0];
      host[4 * w + 1] = st[w][3];
      host[4 * w + 2] = st[w][4];
      host[4 * w + 3] = st[w][7];
    }
    return QCN_OK;
  }
  if (kind < 0 || kind > 2 || n <= 0 || n > qcn::kClkMaxWg || !host) return QCN_ERR_ARG;
  if ((kind == 1 && g_last34_ws) || (kind == 2 && g_last56_ws)) {
    // g_p34_stamp[k][wg] = [realtime start, memtime ..., realtime end]: the
    // last nonzero entry is the end realtime, the one before it the end memtime
    if (n > 1024) return QCN_ERR_ARG;
    static unsigned long long st[1024][64];
    if (hipMemcpyFromSymbol(st, HIP_SYMBOL(qcn::g_p34_stamp), sizeof st, (size_t)(kind - 1) * sizeof st,
                            hipMemcpyDeviceToHost) != hipSuccess)
      return QCN_ERR_HIP;
    for (int w = 0; w < n; ++w) {
      int last = 63;
      while (last > 3 && st[w][last] == 0) --last;
      host[4 * w + 0] = st[w][1];
      host[4 * w + 1] = st[w][last - 1];
      host[4 * w + 2] = st[w][0];
      host[4 * w + 3] = st[w][last];
    }
    return QCN_OK;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(qcn::g_qcn_clk), (size_t)n * 32,
                             (size_t)kind * qcn::kClkMaxWg * 32, hipMemcpyDeviceToHost) == hipSuccess
             ? QCN_OK : QCN_ERR_HIP;
}

}  // extern "C"
