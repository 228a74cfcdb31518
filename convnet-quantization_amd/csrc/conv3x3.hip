// Fused int8 3x3 convolution (pad 1, stride 1) for gfx950:
//   u8 NHWC activations x s8 weights -> int32 MFMA accumulators
//   -> (+ zero-point correction) -> [2x2 max-pool on the accumulators]
//   -> FBGEMM-exact requant (+ReLU) -> [per-layer QDQ hand-off] -> u8 NHWC.
//
// Reference semantics: QuantizedConv2d / QuantizedConvReLU2d as torch.ao's
// fbgemm engine runs them for the stubs of
// /root/reference/models/custom_quantization_model.py:34-45 (SURVEY §8(a)
// rows A5, A6, A10).  Max-pool is applied to the int32 accumulators before
// requantization: requant is monotone non-decreasing in acc, so
// max(requant(a_i)) == requant(max(a_i)) bit for bit.
//
// Design (MI355X-first, not a port):
//  * implicit GEMM, D[cout][pixel] = W[cout][k] * X[k][pixel], k = (tap, cin);
//  * one workgroup owns a run of whole output rows for ALL output channels:
//    its input patch (rows+2 halo, cols+2 halo, CIN bytes per pixel) is staged
//    ONCE in LDS and reused by all 9 taps (9x less activation traffic than an
//    explicit im2col);
//  * weights stream through a double-buffered LDS ring in K-chunks of 64 bytes
//    (one tap, 64 input channels) shared by every wave of the workgroup;
//  * v_mfma_i32_32x32x32_i8, wave tile = 64 cout x 128 pixels (2x4 MFMA tiles,
//    128 accumulator VGPRs); activations are fed as (q - 128) signed bytes and
//    the (128 - zp_x) * sum(w) term is added back exactly in int32;
//  * for pooled layers a wave's four pixel tiles are the four 2x2-window
//    quadrants of the same 32 pooled pixels, so pooling is a register max.
#include "common.hpp"

namespace qcn {

template <int CIN, int COUT, int HW, bool POOL, int WPX>
struct ConvCfg {
  static constexpr int W = HW, H = HW;
  static constexpr int WCO = COUT / 64;          // waves along cout
  static constexpr int NWAVES = WCO * WPX;
  static constexpr int NT = NWAVES * 64;         // threads
  static constexpr int PXB = WPX * 128;          // output pixels per workgroup
  static constexpr int IMG = H * W;
  static constexpr int SEGS = PXB >= IMG ? PXB / IMG : 1;
  static constexpr int R = PXB >= IMG ? H : PXB / W;   // rows per segment
  static constexpr int PS = CIN + 16;            // LDS bytes per staged pixel
  static constexpr int PROWS = R + 2, PCOLS = W + 2;
  static constexpr int PATCH = SEGS * PROWS * PCOLS * PS;
  static constexpr int WS = 64 + 16;             // LDS bytes per cout per chunk
  static constexpr int WBUF = COUT * WS;
  static constexpr int NCH = 9 * CIN / 64;       // K chunks
  static constexpr int LDS = PATCH + 2 * WBUF;
  static constexpr int WLOADS = COUT * 4 / NT;   // 16-B weight loads per thread per chunk
  static_assert(CIN % 64 == 0 && COUT % 64 == 0, "channel multiples of 64");
  static_assert(PXB % W == 0, "workgroup covers whole rows");
  static_assert(PXB >= IMG ? (PXB % IMG == 0) : (H % R == 0), "rows tile the image");
  static_assert(!POOL || (R % 2 == 0), "pooled rows come in pairs");
  static_assert(COUT * 4 % NT == 0 && WLOADS >= 1, "weight staging split");
};

struct ConvEpi {
  const float* u;      // [COUT]
  const float* v;      // [COUT]
  const float* mult;   // [COUT]
  const int* corr;     // [COUT] (128 - zp_x) * sum_k w[k]
  int zp_y, lo;        // output zero point, lower clamp (zp_y if relu else 0)
  int qdq;             // 0: write requantized u8; 1: apply qdq_next
  float s1; int z1; float inv2; int z2;
};

template <int CIN, int COUT, int HW, bool POOL, int WPX>
__global__ __launch_bounds__(COUT * WPX)
void conv3x3_u8s8_kernel(const uint8_t* __restrict__ x, int nimg, int x_zp,
                         const int8_t* __restrict__ wpk, ConvEpi ep,
                         uint8_t* __restrict__ y) {
  using C = ConvCfg<CIN, COUT, HW, POOL, WPX>;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t* patch = lds;
  uint8_t* wbuf0 = lds + C::PATCH;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wc = wave % C::WCO;      // cout group of this wave
  const int wp = wave / C::WCO;      // pixel group of this wave
  const int l32 = lane & 31;
  const int hi = lane >> 5;

  const long p0 = (long)blockIdx.x * C::PXB;         // first output pixel
  const int n0 = (int)(p0 / C::IMG);
  const int y0 = (int)((p0 % C::IMG) / C::W);

  // ---- stage the input patch (q ^ 0x80 = q - 128 as s8; halo = zp ^ 0x80)
  const uint32_t padw = xor80(splat_u8(x_zp));
  constexpr int CH16 = CIN / 16;
  constexpr int NSLOT = C::SEGS * C::PROWS * C::PCOLS;
  for (int it = tid; it < NSLOT * CH16; it += C::NT) {
    const int slot = it / CH16, chunk = it % CH16;
    const int seg = slot / (C::PROWS * C::PCOLS);
    const int rem = slot % (C::PROWS * C::PCOLS);
    const int pr = rem / C::PCOLS, pc = rem % C::PCOLS;
    const int n = n0 + seg, yy = y0 + pr - 1, xx = pc - 1;
    uint4 val = make_uint4(padw, padw, padw, padw);
    if (n < nimg && yy >= 0 && yy < C::H && xx >= 0 && xx < C::W) {
      const uint4 g = *reinterpret_cast<const uint4*>(
          x + (((long)n * C::H + yy) * C::W + xx) * CIN + chunk * 16);
      val = make_uint4(xor80(g.x), xor80(g.y), xor80(g.z), xor80(g.w));
    }
    *reinterpret_cast<uint4*>(patch + slot * C::PS + chunk * 16) = val;
  }

  // ---- stage weight chunk 0
  auto wsrc = [&](int ch, int i) {
    const int e = tid + i * C::NT;          // 16-byte element within the chunk
    return reinterpret_cast<const uint4*>(wpk + (long)ch * COUT * 64) + e;
  };
  auto wdst = [&](uint8_t* buf, int i) {
    const int e = tid + i * C::NT;
    return reinterpret_cast<uint4*>(buf + (e >> 2) * C::WS + (e & 3) * 16);
  };
#pragma unroll
  for (int i = 0; i < C::WLOADS; ++i) *wdst(wbuf0, i) = *wsrc(0, i);

  // ---- per-lane pixel slots of the four pixel tiles
  int pslot[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int seg, yy, xx;
    if constexpr (POOL) {
      constexpr int PW = C::W / 2, PR = C::R / 2;
      const int q = wp * 32 + l32;
      seg = q / (PR * PW);
      yy = 2 * ((q / PW) % PR) + (j >> 1);
      xx = 2 * (q % PW) + (j & 1);
    } else {
      const int m = (wp * 4 + j) * 32 + l32;
      seg = m / (C::R * C::W);
      yy = (m / C::W) % C::R;
      xx = m % C::W;
    }
    pslot[j] = ((seg * C::PROWS + yy) * C::PCOLS + xx) * C::PS + hi * 16;
  }
  const int wrow0 = (wc * 64 + l32) * C::WS + hi * 16;

  v16i acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (v16i){0};

  __syncthreads();

  uint4 pre[C::WLOADS];
  for (int ch = 0; ch < C::NCH; ++ch) {
    const bool more = ch + 1 < C::NCH;
    if (more) {
#pragma unroll
      for (int i = 0; i < C::WLOADS; ++i) pre[i] = *wsrc(ch + 1, i);
    }
    const uint8_t* wb = wbuf0 + (ch & 1) * C::WBUF;
    const int tap = ch / (CIN / 64);
    const int cb = ch % (CIN / 64);
    const int r = tap / 3, s = tap % 3;
    const int poff = (r * C::PCOLS + s) * C::PS + cb * 64;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v4i a[2], b[4];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        a[i] = *reinterpret_cast<const v4i*>(wb + wrow0 + i * 32 * C::WS + kk * 32);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = *reinterpret_cast<const v4i*>(patch + pslot[j] + poff + kk * 32);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      uint8_t* nb = wbuf0 + ((ch + 1) & 1) * C::WBUF;
#pragma unroll
      for (int i = 0; i < C::WLOADS; ++i) *wdst(nb, i) = pre[i];
    }
    __syncthreads();
  }

  // ---- epilogue
  // accumulator element (reg rg) of tile (i, j): cout row = 32i + (rg&3) + 8(rg>>2) + 4hi,
  // pixel column = l32 of pixel tile j.
  const long total_out = POOL ? (long)nimg * C::IMG / 4 : (long)nimg * C::IMG;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int res[4][16];
    constexpr int NJ = POOL ? 1 : 4;
#pragma unroll
    for (int rg = 0; rg < 16; ++rg) {
      const int co = wc * 64 + i * 32 + (rg & 3) + 8 * (rg >> 2) + 4 * hi;
      const int corr = ep.corr[co];
      const float u = ep.u[co], v = ep.v[co], mu = ep.mult[co];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        int a;
        if constexpr (POOL) {
          a = max(max(acc[i][0][rg], acc[i][1][rg]), max(acc[i][2][rg], acc[i][3][rg]));
        } else {
          a = acc[i][j][rg];
        }
        int q = requant_one(a + corr, u, v, mu, ep.zp_y, ep.lo);
        if (ep.qdq) q = qdq_next(q, ep.s1, ep.z1, ep.inv2, ep.z2);
        res[j][rg] = q;
      }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      long opix;
      if constexpr (POOL) {
        opix = (long)blockIdx.x * (C::PXB / 4) + wp * 32 + l32;
      } else {
        opix = p0 + (wp * 4 + j) * 32 + l32;
      }
      if (opix < total_out) {
        uint8_t* dst = y + opix * COUT + wc * 64 + i * 32 + 4 * hi;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint32_t w32 = (uint32_t)res[j][4 * g] | ((uint32_t)res[j][4 * g + 1] << 8) |
                               ((uint32_t)res[j][4 * g + 2] << 16) |
                               ((uint32_t)res[j][4 * g + 3] << 24);
          *reinterpret_cast<uint32_t*>(dst + 8 * g) = w32;
        }
      }
    }
  }
}

// --------------------------------------------------------------------------
// conv1: CIN = 3, input fp32 NCHW quantized on the fly (aten quantize_per_tensor
// semantics, oracle qref A1), im2col rows of K = 27 (+5 zero) bytes in LDS,
// one 32x32x32 MFMA k-step.  HBM-bound layer (52 op/B).
// Block: 16 output rows x 32 cols of one image, all 64 output channels.
struct Conv1Cfg {
  static constexpr int H = 32, W = 32, R = 16, COUT = 64, NT = 256;
  static constexpr int PXB = R * W;                     // 512
  static constexpr int PR = R + 2, PC = W + 2;
  static constexpr int PATCH = 3 * PR * PC;              // s8 bytes, [c][row][col]
  static constexpr int PATCH_AL = (PATCH + 15) / 16 * 16;
  static constexpr int KS = 32 + 16;                     // im2col row stride (padded)
  static constexpr int LDS = PATCH_AL + PXB * KS;
};

template <int HW>
__global__ __launch_bounds__(256)
void conv1_f32_kernel(const float* __restrict__ x, int nimg, float in_inv, int in_zp,
                      const int8_t* __restrict__ w1, ConvEpi ep, uint8_t* __restrict__ y,
                      uint8_t* __restrict__ qin_out) {
  constexpr int H = HW, W = HW;
  constexpr int R = (HW * HW >= 512) ? 512 / W : H;       // rows per image segment
  constexpr int SEGS = (HW * HW >= 512) ? 1 : 512 / (HW * HW);
  constexpr int PR = R + 2, PC = W + 2;
  constexpr int PATCH = SEGS * 3 * PR * PC;
  constexpr int PATCH_AL = (PATCH + 15) / 16 * 16;
  constexpr int KS = 48;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  int8_t* patch = reinterpret_cast<int8_t*>(lds);
  uint8_t* cols = lds + PATCH_AL;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hi = lane >> 5;
  const long p0 = (long)blockIdx.x * 512;
  const int n0 = (int)(p0 / (H * W));
  const int y0 = (int)((p0 % (H * W)) / W);
  const int8_t padv = (int8_t)(in_zp - 128);

  for (int it = tid; it < PATCH; it += 256) {
    const int seg = it / (3 * PR * PC);
    const int rem = it % (3 * PR * PC);
    const int c = rem / (PR * PC);
    const int rr = (rem / PC) % PR, cc = rem % PC;
    const int n = n0 + seg, yy = y0 + rr - 1, xx = cc - 1;
    int8_t v = padv;
    if (n < nimg && yy >= 0 && yy < H && xx >= 0 && xx < W) {
      const long gi = (((long)n * 3 + c) * H + yy) * W + xx;
      float t = x[gi] * in_inv;
      t = fminf(fmaxf(t, -1.0e9f), 1.0e9f);
      int q = (int)__builtin_rintf(t) + in_zp;
      q = q < 0 ? 0 : (q > 255 ? 255 : q);
      v = (int8_t)(q - 128);
      if (qin_out != nullptr && seg < SEGS && rr >= 1 && rr <= R && cc >= 1 && cc <= W)
        qin_out[(((long)n * H + yy) * W + xx) * 3 + c] = (uint8_t)q;
    }
    patch[it] = v;
  }
  __syncthreads();
  // im2col: k = (r*3 + s)*3 + c, k in [27, 32) zero
  for (int pp = tid; pp < 512; pp += 256) {
    const int seg = pp / (R * W), yy = (pp / W) % R, xx = pp % W;
    uint32_t wds[8];
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      uint32_t wv = 0;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        const int k = d * 4 + bb;
        uint32_t byte = 0;
        if (k < 27) {
          const int tap = k / 3, c = k % 3, r = tap / 3, s = tap % 3;
          byte = (uint8_t)patch[((seg * 3 + c) * PR + yy + r) * PC + xx + s];
        }
        wv |= byte << (8 * bb);
      }
      wds[d] = wv;
    }
    uint4* dst = reinterpret_cast<uint4*>(cols + pp * KS);
    dst[0] = make_uint4(wds[0], wds[1], wds[2], wds[3]);
    dst[1] = make_uint4(wds[4], wds[5], wds[6], wds[7]);
  }
  __syncthreads();

  // weights: [64][32] s8 packed, k order as above (zero for k >= 27)
  v4i a[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
    a[i] = *reinterpret_cast<const v4i*>(w1 + (i * 32 + l32) * 32 + hi * 16);
  v16i acc[2][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = (wave * 4 + j) * 32 + l32;
    const v4i b = *reinterpret_cast<const v4i*>(cols + m * KS + hi * 16);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b, (v16i){0}, 0, 0, 0);
  }
  const long total = (long)nimg * H * W;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long opix = p0 + (wave * 4 + j) * 32 + l32;
      int res[16];
#pragma unroll
      for (int rg = 0; rg < 16; ++rg) {
        const int co = i * 32 + (rg & 3) + 8 * (rg >> 2) + 4 * hi;
        int q = requant_one(acc[i][j][rg] + ep.corr[co], ep.u[co], ep.v[co], ep.mult[co],
                            ep.zp_y, ep.lo);
        if (ep.qdq) q = qdq_next(q, ep.s1, ep.z1, ep.inv2, ep.z2);
        res[rg] = q;
      }
      if (opix < total) {
        uint8_t* dst = y + opix * 64 + i * 32 + 4 * hi;
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<uint32_t*>(dst + 8 * g) =
              (uint32_t)res[4 * g] | ((uint32_t)res[4 * g + 1] << 8) |
              ((uint32_t)res[4 * g + 2] << 16) | ((uint32_t)res[4 * g + 3] << 24);
      }
    }
  }
}

// --------------------------------------------------------------------------
// Generic fallback (any CIN/COUT/H/W, no MFMA): one thread per output element.
// Used only for shapes without a tuned instantiation (unit tests, odd sizes).
__global__ void conv3x3_generic_kernel(const uint8_t* __restrict__ x, int nimg, int H, int W,
                                       int cin, int x_zp, const int8_t* __restrict__ wpk,
                                       int tiled, int cout, ConvEpi ep, int pool,
                                       uint8_t* __restrict__ y) {
  const int OH = pool ? H / 2 : H, OW = pool ? W / 2 : W;
  const long total = (long)nimg * OH * OW * cout;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int co = (int)(e % cout);
    const long pix = e / cout;
    const int ox = (int)(pix % OW), oy = (int)((pix / OW) % OH);
    const int n = (int)(pix / ((long)OW * OH));
    int best = INT32_MIN;
    const int nq = pool ? 4 : 1;
    for (int qd = 0; qd < nq; ++qd) {
      const int yy = pool ? 2 * oy + (qd >> 1) : oy;
      const int xx = pool ? 2 * ox + (qd & 1) : ox;
      int acc = 0;
      for (int r = 0; r < 3; ++r)
        for (int s = 0; s < 3; ++s) {
          const int iy = yy + r - 1, ix = xx + s - 1;
          if (iy < 0 || iy >= H || ix < 0 || ix >= W) continue;  // (zp - zp) * w = 0
          const uint8_t* xp = x + (((long)n * H + iy) * W + ix) * cin;
          const int tap = r * 3 + s;
          for (int c = 0; c < cin; ++c) {
            const long wi = tiled ? ((long)(tap * (cin / 64) + c / 64) * cout + co) * 64 + (c % 64)
                                  : ((long)co * 9 + tap) * cin + c;
            acc += ((int)xp[c] - x_zp) * (int)wpk[wi];
          }
        }
      best = acc > best ? acc : best;
    }
    int q = requant_one(best, ep.u[co], ep.v[co], ep.mult[co], ep.zp_y, ep.lo);
    if (ep.qdq) q = qdq_next(q, ep.s1, ep.z1, ep.inv2, ep.z2);
    y[e] = (uint8_t)q;
  }
}

}  // namespace qcn

// ==========================================================================
// C-ABI dispatch
// ==========================================================================
#include "qconvnet_abi.hpp"

namespace {
using namespace qcn;

template <int CIN, int COUT, int HW, bool POOL, int WPX>
int launch_conv(const uint8_t* x, int nimg, int x_zp, const int8_t* wpk, const ConvEpi& ep,
                uint8_t* y, hipStream_t st) {
  using C = ConvCfg<CIN, COUT, HW, POOL, WPX>;
  const long pix = (long)nimg * C::IMG;
  const int grid = (int)((pix + C::PXB - 1) / C::PXB);
  auto k = conv3x3_u8s8_kernel<CIN, COUT, HW, POOL, WPX>;
  static bool attr_done = false;
  if (!attr_done) {
    if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS) !=
        hipSuccess)
      return QCN_ERR_HIP;
    attr_done = true;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(C::NT), C::LDS, st, x, nimg, x_zp, wpk, ep, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

// Tuned instantiations: the SimpleConvNet layers and the
// small shapes the parity fixtures use.
int dispatch_conv(int cin, int cout, int hw, int pool, const uint8_t* x, int nimg, int x_zp,
                  const int8_t* wpk, const ConvEpi& ep, uint8_t* y, hipStream_t st) {
#define QCN_CONV_CASE(CI, CO, HWV, PL, WPXV)                                          \
  if (cin == CI && cout == CO && hw == HWV && pool == PL)                              \
    return launch_conv<CI, CO, HWV, PL, WPXV>(x, nimg, x_zp, wpk, ep, y, st);
  QCN_CONV_CASE(64, 64, 32, 1, 4)
  QCN_CONV_CASE(64, 64, 32, 0, 4)
  QCN_CONV_CASE(64, 128, 16, 0, 2)
  QCN_CONV_CASE(128, 128, 16, 1, 2)
  QCN_CONV_CASE(128, 128, 16, 0, 2)
  QCN_CONV_CASE(128, 256, 8, 0, 2)
  QCN_CONV_CASE(256, 256, 8, 1, 2)
  QCN_CONV_CASE(256, 256, 8, 0, 2)
  QCN_CONV_CASE(64, 64, 16, 0, 2)
  QCN_CONV_CASE(64, 64, 16, 1, 2)
  QCN_CONV_CASE(64, 64, 8, 0, 1)
  QCN_CONV_CASE(64, 64, 8, 1, 2)
  QCN_CONV_CASE(64, 128, 8, 0, 1)
  QCN_CONV_CASE(128, 256, 4, 0, 2)
  QCN_CONV_CASE(256, 256, 4, 0, 1)
  QCN_CONV_CASE(256, 256, 4, 1, 1)
#undef QCN_CONV_CASE
  return QCN_ERR_UNSUPPORTED;
}
}  // namespace

extern "C" {

int qcn_conv3x3_packed_size(int cin, int cout) { return 9 * cin * cout; }

// Host: pack OIHW (torch) s8 weights into the kernel's K-chunk-major layout
// [chunk = tap*(cin/64) + cb][cout][64] and return per-cout weight sums.
int qcn_pack_conv3x3_weight(const int8_t* w_oihw, int cout, int cin, int8_t* out,
                            int32_t* wsum) {
  if (!w_oihw || !out || !wsum || cout <= 0 || cin <= 0) return QCN_ERR_ARG;
  const bool tiled = (cin % 64 == 0) && (cout % 64 == 0);
  for (int co = 0; co < cout; ++co) {
    int32_t s = 0;
    for (int c = 0; c < cin; ++c)
      for (int t = 0; t < 9; ++t) {
        const int8_t v = w_oihw[((long)co * cin + c) * 9 + t];
        s += v;
        long dst;
        if (tiled) {
          const int ch = t * (cin / 64) + c / 64;
          dst = ((long)ch * cout + co) * 64 + (c % 64);
        } else {  // plain OHWI for the generic kernel
          dst = ((long)co * 9 + t) * cin + c;
        }
        out[dst] = v;
      }
    wsum[co] = s;
  }
  return QCN_OK;
}

// Host: conv1 (cin = 3) packing, [64][32] with k = tap*3 + c, zero for k >= 27.
int qcn_pack_conv1_weight(const int8_t* w_oihw, int cout, int8_t* out, int32_t* wsum) {
  if (!w_oihw || !out || !wsum || cout != 64) return QCN_ERR_ARG;
  for (int co = 0; co < 64; ++co) {
    int32_t s = 0;
    for (int k = 0; k < 32; ++k) {
      int8_t v = 0;
      if (k < 27) {
        const int t = k / 3, c = k % 3;
        v = w_oihw[(co * 3 + c) * 9 + t];
      }
      out[co * 32 + k] = v;
      s += v;
    }
    wsum[co] = s;
  }
  return QCN_OK;
}

int qcn_conv3x3_u8s8_nhwc(const uint8_t* x, int nimg, int h, int w, int cin, int x_zp,
                          const int8_t* w_packed, int cout, const float* u, const float* v,
                          const float* mult, const int32_t* corr, int y_zp, int relu, int pool,
                          const qcn_qdq_t* qdq, uint8_t* y, void* stream) {
  if (!x || !w_packed || !u || !v || !mult || !corr || !y) return QCN_ERR_ARG;
  if (nimg <= 0 || h <= 0 || w <= 0 || cin <= 0 || cout <= 0) return QCN_ERR_ARG;
  if (x_zp < 0 || x_zp > 255 || y_zp < 0 || y_zp > 255) return QCN_ERR_ARG;
  if (pool && ((h & 1) || (w & 1))) return QCN_ERR_ARG;
  ConvEpi ep{u, v, mult, corr, y_zp, relu ? y_zp : 0, 0, 0.f, 0, 0.f, 0};
  if (qdq) {
    ep.qdq = 1;
    ep.s1 = qdq->s1; ep.z1 = qdq->z1; ep.inv2 = qdq->inv2; ep.z2 = qdq->z2;
  }
  hipStream_t st = (hipStream_t)stream;
  if (h == w && cin % 64 == 0 && cout % 64 == 0) {
    const int rc = dispatch_conv(cin, cout, h, pool, x, nimg, x_zp, w_packed, ep, y, st);
    if (rc != QCN_ERR_UNSUPPORTED) return rc;
  }
  const int tiled = (cin % 64 == 0) && (cout % 64 == 0);
  const long total = (long)nimg * (pool ? h / 2 : h) * (pool ? w / 2 : w) * cout;
  const int grid = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(conv3x3_generic_kernel, dim3(grid), dim3(256), 0, st, x, nimg, h, w, cin,
                     x_zp, w_packed, tiled, cout, ep, pool, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_conv1_f32_nchw(const float* x, int nimg, int hw, float in_scale, int in_zp,
                       const int8_t* w1_packed, const float* u, const float* v, const float* mult,
                       const int32_t* corr, int y_zp, int relu, const qcn_qdq_t* qdq, uint8_t* y,
                       uint8_t* q_in, void* stream) {
  if (!x || !w1_packed || !u || !v || !mult || !corr || !y) return QCN_ERR_ARG;
  if (nimg <= 0 || in_zp < 0 || in_zp > 255 || !(in_scale > 0.f)) return QCN_ERR_ARG;
  ConvEpi ep{u, v, mult, corr, y_zp, relu ? y_zp : 0, 0, 0.f, 0, 0.f, 0};
  if (qdq) {
    ep.qdq = 1;
    ep.s1 = qdq->s1; ep.z1 = qdq->z1; ep.inv2 = qdq->inv2; ep.z2 = qdq->z2;
  }
  const float inv = 1.0f / in_scale;
  hipStream_t st = (hipStream_t)stream;
  const long pix = (long)nimg * hw * hw;
  const int grid = (int)((pix + 511) / 512);
#define QCN_C1(HWV)                                                                       \
  if (hw == HWV) {                                                                        \
    constexpr int R = (HWV * HWV >= 512) ? 512 / HWV : HWV;                              \
    constexpr int SEGS = (HWV * HWV >= 512) ? 1 : 512 / (HWV * HWV);                     \
    constexpr int LDS = ((SEGS * 3 * (R + 2) * (HWV + 2) + 15) / 16 * 16) + 512 * 48;     \
    hipLaunchKernelGGL(qcn::conv1_f32_kernel<HWV>, dim3(grid), dim3(256), LDS, st, x, nimg, \
                       inv, in_zp, w1_packed, ep, y, q_in);                              \
    return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;                       \
  }
  QCN_C1(32)
  QCN_C1(16)
  QCN_C1(8)
#undef QCN_C1
  return QCN_ERR_UNSUPPORTED;
}

}  // extern "C"
