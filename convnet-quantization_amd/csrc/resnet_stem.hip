// Fused ResNet stem (torchvision's conv1 7x7/2 pad 3 -> ReLU ->
// MaxPool2d(3, 2, padding=1), as the static int8 ResNet of
// custom_quantization_model.py:117-141 runs it after its QuantStub):
//
//   fp32 NCHW [n][3][S][S]  --quantize (A1)-->  7x7/2 conv 3->64 on
//   v_mfma_i32_32x32x32_i8  --FBGEMM requant + ReLU (A6)-->  3x3/2 max-pool
//   --> u8 NHWC [n][S/4][S/4][64]
//
// in one persistent launch, with nothing in HBM between the steps (the
// three-launch form — qcn_stem_pack_f32_nchw, the 7x1 conv_gemm over the
// packed rows, qcn_maxpool3x3s2_u8_nhwc — moved ~1.6 GB per 512 images).
//
// One 512-thread workgroup per CU loops over bands of P = 4 (or 2) pool rows
// of one image.  A band needs CR = 2P + 1 conv rows (the conv row shared with the
// previous band is recomputed) and IR = 4P + 7 input rows.  Per band:
//   A  the input rows are quantized (A1: q = clamp(zp + rint(x * inv), 0, 255))
//      into QIN, 3 bytes per column (channel fastest), zero-point columns on
//      both sides and zero-point rows outside the image;
//   B  the tap rows are built from QIN: TAP[ir][ox] holds, at byte 3 s + c,
//      q[c][ir][2 ox - 3 + s] (s < 7) — the same 32-byte K chunk per conv tap
//      row as qcn_stem_pack_f32_nchw, so the conv is a 7x1 conv over Cin = 32
//      (K = 224) with the weights packed by stem_weight_rows; bytes 21..31 meet
//      zero weights;
//   C  every wave takes 32-pixel conv tiles: 7 B fragments (one ds_read_b128
//      per tap row) against both 32-channel A blocks held in registers for the
//      whole kernel, 14 MFMAs, then the requant + ReLU into CS, u8 [conv px][64];
//   D  the 3x3/2 max-pool over CS (padding taps skipped; max commutes with the
//      monotone requant, as qcn_maxpool3x3s2_u8_nhwc), 16-byte NHWC stores.
// The next band's fp32 input is loaded into registers during C and D.
#include "common.hpp"
#include "qconvnet_abi.hpp"


namespace qcn {

// Per-byte max of u8 x 4 dwords, kept split as two packed u16 pairs: the
// even bytes (0, 2) and the odd bytes (1, 3) of each dword, zero-extended.
// Per tap dword: one AND, one v_perm, two v_pk_max_u16; joined once at the end.
typedef unsigned short stem_us2 __attribute__((ext_vector_type(2)));
struct StemMax {
  stem_us2 lo, hi;
  QCN_DEV void add(uint32_t s) {
    const stem_us2 sl = __builtin_bit_cast(stem_us2, s & 0x00ff00ffu);
    // bytes 1 and 3 of s into bytes 0 and 2, zeros (selector 0x0c) above them
    const stem_us2 sh = __builtin_bit_cast(stem_us2, __builtin_amdgcn_perm(0u, s, 0x0c030c01u));
    lo = __builtin_elementwise_max(lo, sl);
    hi = __builtin_elementwise_max(hi, sh);
  }
  QCN_DEV uint32_t get() const {
    return __builtin_bit_cast(uint32_t, lo) | (__builtin_bit_cast(uint32_t, hi) << 8);
  }
};

template <int S, int P_ = 2>
struct StemCfg {
  static constexpr int P = P_, CR = 2 * P + 1, IR = 4 * P + 7;
  static constexpr int OW = S / 2, PW = S / 4, C = 64;
  static constexpr int BANDS = PW / P;            // bands per image
  static constexpr int QL = 4;                    // zero-point columns left of a QIN row
  static constexpr int QROW = (((QL + S + 3) * 3 + 4) + 15) / 16 * 16;
  static constexpr int TAPROW = OW * 32;
  static constexpr int NPX = CR * OW;             // conv pixels per band
  static constexpr int NT = (NPX + 31) / 32;      // 32-pixel tiles
  static constexpr int CSP = C + 4;               // CS pixel stride (conflict-free dword writes)
  static constexpr int OFF_TAP = 0, TAP_B = IR * TAPROW;
  static constexpr int OFF_R2 = TAP_B;            // QIN (phases A, B) / CS (phases C, D)
  static constexpr int QIN_B = IR * QROW, CS_B = (NPX * CSP + 15) / 16 * 16;
  static constexpr int R2_B = QIN_B > CS_B ? QIN_B : CS_B;
  static constexpr int OFF_EPI = OFF_R2 + R2_B;   // u | v | mult (fp32) | corr (int32), x 64 each
  static constexpr int LDS = OFF_EPI + 4 * C * 4;
  static constexpr int NTH = 512;
  static constexpr int ITEMS = IR * (S / 4);      // phase A items: (row, 4 columns)
  static constexpr int NPF = (ITEMS + NTH - 1) / NTH;
  static_assert(PW % P == 0, "bands tile the pool rows");
  static_assert(S % 4 == 0, "4-column quantize items");
  static_assert(LDS <= 160 * 1024, "fits one CU's LDS");
};

struct StemArgs {
  const float* x;
  int n;
  float inv;   // fp32(1 / in_scale)
  int zp;
  const int8_t* w;   // [7][64][32] (stem_weight_rows, k-major)
  const float *u, *v, *mult;
  const int* corr;
  int zp_y, lo;
  uint8_t* y;
};

template <int S, int P = 2>
__global__ __launch_bounds__(512, 1) void stem_fused_kernel(StemArgs a) {
  using C = StemCfg<S, P>;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, hi = lane >> 5;
  uint8_t* tap = lds + C::OFF_TAP;
  uint8_t* r2 = lds + C::OFF_R2;
  float* epi = reinterpret_cast<float*>(lds + C::OFF_EPI);
  const uint32_t zp4 = splat_u8(a.zp);

  // epilogue constants and corr in LDS: a global load inside the band loop
  // would queue behind the next band's prefetch (vmcnt retires in order)
  if (tid < 3 * C::C) {
    const float* src = tid < C::C ? a.u : (tid < 2 * C::C ? a.v : a.mult);
    epi[tid] = src[tid % C::C];
  } else if (tid < 4 * C::C) {
    reinterpret_cast<int*>(epi)[tid] = a.corr[tid - 3 * C::C];
  }
  // A blocks (couts 32 i .. 32 i + 31) of all 7 tap-row chunks, in registers
  v4i wa[2][7];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 7; ++r)
      wa[i][r] = *reinterpret_cast<const v4i*>(a.w + ((r * 64) + 32 * i + l32) * 32 + 16 * hi);

  const int nb = a.n * C::BANDS;
  // a contiguous run of bands per workgroup (mostly one image, top to
  // bottom): the 7 input rows two neighbouring bands share were fetched by
  // this CU one band earlier and come from its XCD's L2, not HBM
  const int bbeg = (int)((long)blockIdx.x * nb / gridDim.x);
  const int bend = (int)((long)(blockIdx.x + 1) * nb / gridDim.x);
  // phase-A prefetch: item it = tid + NTH k -> (QIN row, 4-column group)
  float4 pf[C::NPF][3];
  auto prefetch = [&](int band) {
    const int img = band / C::BANDS, pr0 = (band % C::BANDS) * C::P;
#pragma unroll
    for (int k = 0; k < C::NPF; ++k) {
      const int it = tid + C::NTH * k;
      const int row = it / (S / 4), c4 = it % (S / 4);
      const int iy = 4 * pr0 - 5 + row;
      const bool ok = band < bend && it < C::ITEMS && iy >= 0 && iy < S;
#pragma unroll
      for (int c = 0; c < 3; ++c)
        pf[k][c] = ok ? *reinterpret_cast<const float4*>(a.x + (((long)img * 3 + c) * S + iy) * S + 4 * c4)
                      : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto quant = [&](float v) {
    const float t = fminf(fmaxf(v * a.inv, -1.0e9f), 1.0e9f);
    int q = (int)__builtin_rintf(t) + a.zp;
    return (uint32_t)(q < 0 ? 0 : (q > 255 ? 255 : q));
  };

  int band = bbeg;
  prefetch(band);
  for (; band < bend; ++band) {
    const int img = band / C::BANDS, pr0 = (band % C::BANDS) * C::P;
    // ---- A: quantize the input rows into QIN (3 B per column, channel fastest)
#pragma unroll
    for (int k = 0; k < C::NPF; ++k) {
      const int it = tid + C::NTH * k;
      if (it < C::ITEMS) {
        const int row = it / (S / 4), c4 = it % (S / 4);
        const int iy = 4 * pr0 - 5 + row;
        uint32_t d[3];
        if (iy >= 0 && iy < S) {
          const float* f0 = &pf[k][0].x;
          const float* f1 = &pf[k][1].x;
          const float* f2 = &pf[k][2].x;
          uint32_t b[12];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            b[3 * e] = quant(f0[e]);
            b[3 * e + 1] = quant(f1[e]);
            b[3 * e + 2] = quant(f2[e]);
          }
#pragma unroll
          for (int j = 0; j < 3; ++j)
            d[j] = b[4 * j] | (b[4 * j + 1] << 8) | (b[4 * j + 2] << 16) | (b[4 * j + 3] << 24);
        } else {
          d[0] = d[1] = d[2] = zp4;
        }
        uint32_t* q = reinterpret_cast<uint32_t*>(r2 + row * C::QROW + 3 * (C::QL + 4 * c4));
        q[0] = d[0]; q[1] = d[1]; q[2] = d[2];
      }
    }
    // zero-point columns: 3 QL bytes on the left, the rest of the row on the right
    constexpr int RPAD0 = 3 * (C::QL + S), RPADW = (C::QROW - RPAD0) / 4;
    for (int e = tid; e < C::IR * (3 * C::QL / 4 + RPADW); e += C::NTH) {
      const int row = e / (3 * C::QL / 4 + RPADW), k = e % (3 * C::QL / 4 + RPADW);
      const int off = k < 3 * C::QL / 4 ? 4 * k : RPAD0 + 4 * (k - 3 * C::QL / 4);
      *reinterpret_cast<uint32_t*>(r2 + row * C::QROW + off) = zp4;
    }
    __syncthreads();
    // ---- B: tap rows.  Entry (ir, ox) starts at QIN byte 3 (2 ox - 3 + QL);
    // its two 16-B halves swap when (ox >> 3) & 1 (conflict-free B reads)
    for (int e = tid; e < C::IR * C::OW; e += C::NTH) {
      const int ir = e / C::OW, ox = e % C::OW;
      const int st = 3 * (2 * ox - 3 + C::QL), d0 = st >> 2, sh = st & 3;
      const uint32_t* q = reinterpret_cast<const uint32_t*>(r2 + ir * C::QROW) + d0;
      uint32_t w[7];
#pragma unroll
      for (int k = 0; k < 7; ++k) w[k] = q[k];
      uint32_t o[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) o[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
      uint4* t = reinterpret_cast<uint4*>(tap + (ir * C::OW + ox) * 32);
      const int sw = (ox >> 3) & 1;
      t[sw] = make_uint4(o[0], o[1], o[2], o[3]);
      t[sw ^ 1] = make_uint4(o[4], o[5], zp4, zp4);
    }
    __syncthreads();
    // next band's input: in flight during C and D
    prefetch(band + 1);
    // ---- C: conv tiles -> requant + ReLU -> CS [conv px][CSP]
    const bool row0_pad = pr0 == 0;   // local conv row 0 is conv row -1 (pool padding)
    for (int t = wave; t < C::NT; t += C::NTH / 64) {
      int m = t * 32 + l32;
      const bool live = m < C::NPX;
      m = live ? m : C::NPX - 1;
      const int crow = m / C::OW, ccol = m % C::OW;
      const int base = ((2 * crow) * C::OW + ccol) * 32 + ((hi ^ ((ccol >> 3) & 1)) << 4);
      v16i acc[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int4 c4 = *reinterpret_cast<const int4*>(reinterpret_cast<const int*>(epi) + 3 * C::C +
                                                         32 * i + 8 * g + 4 * hi);
          acc[i][4 * g] = c4.x; acc[i][4 * g + 1] = c4.y; acc[i][4 * g + 2] = c4.z; acc[i][4 * g + 3] = c4.w;
        }
      v4i b[7];
#pragma unroll
      for (int r = 0; r < 7; ++r) b[r] = *reinterpret_cast<const v4i*>(tap + base + r * C::TAPROW);
#pragma unroll
      for (int r = 0; r < 7; ++r) {
#pragma unroll
        for (int d = 0; d < 4; ++d) b[r][d] ^= (int)0x80808080u;   // u8 -> s8 (q - 128)
        acc[0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wa[0][r], b[r], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wa[1][r], b[r], acc[1], 0, 0, 0);
      }
      if (live && !(row0_pad && crow == 0)) {
        const float zpf = (float)a.zp_y, lof = (float)a.lo;
        uint32_t* cs = reinterpret_cast<uint32_t*>(r2 + m * C::CSP);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int co = 32 * i + 8 * g + 4 * hi;
            const float4 u4 = *reinterpret_cast<const float4*>(epi + co);
            const float4 v4 = *reinterpret_cast<const float4*>(epi + C::C + co);
            const float4 m4 = *reinterpret_cast<const float4*>(epi + 2 * C::C + co);
            uint32_t wd = __builtin_amdgcn_cvt_pk_u8_f32(requant_f(acc[i][4 * g], u4.x, v4.x, m4.x, zpf, lof), 0, 0u);
            wd = __builtin_amdgcn_cvt_pk_u8_f32(requant_f(acc[i][4 * g + 1], u4.y, v4.y, m4.y, zpf, lof), 1, wd);
            wd = __builtin_amdgcn_cvt_pk_u8_f32(requant_f(acc[i][4 * g + 2], u4.z, v4.z, m4.z, zpf, lof), 2, wd);
            wd = __builtin_amdgcn_cvt_pk_u8_f32(requant_f(acc[i][4 * g + 3], u4.w, v4.w, m4.w, zpf, lof), 3, wd);
            cs[co / 4] = wd;
          }
      }
    }
    __syncthreads();
    // ---- D: 3x3/2 max-pool (pool row pr0 + pr reads local conv rows 2 pr .. 2 pr + 2)
    for (int e = tid; e < C::P * C::PW * 4; e += C::NTH) {
      const int q16 = e & 3, pc = (e >> 2) % C::PW, pr = (e >> 2) / C::PW;
      StemMax r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k].lo = r[k].hi = (stem_us2){0, 0};
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const int lr = 2 * pr + dy;
        if (row0_pad && lr == 0) continue;
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
          const int cx = 2 * pc + dx;
          if (cx < 0) continue;
          const uint32_t* s = reinterpret_cast<const uint32_t*>(r2 + (lr * C::OW + cx) * C::CSP + 16 * q16);
#pragma unroll
          for (int k = 0; k < 4; ++k) r[k].add(s[k]);
        }
      }
      uint8_t* o = a.y + ((((long)img * C::PW + pr0 + pr) * C::PW + pc) * C::C + 16 * q16);
      *reinterpret_cast<uint4*>(o) = make_uint4(r[0].get(), r[1].get(), r[2].get(), r[3].get());
    }
    __syncthreads();   // QIN (next phase A) aliases CS
  }
}

}  // namespace qcn

namespace {
template <int S, int P = 2>
int launch_stem(const qcn::StemArgs& a, hipStream_t st) {
  using C = qcn::StemCfg<S, P>;
  static bool attr_done[QCN_MAX_DEV] = {};
  if (!qcn_set_lds_once((const void*)qcn::stem_fused_kernel<S, P>, C::LDS, attr_done)) return QCN_ERR_HIP;
  const int ncu = qcn_cu_count();
  if (ncu <= 0) return QCN_ERR_HIP;
  const long nb = (long)a.n * C::BANDS;
  const int grid = (int)(nb < ncu ? nb : ncu);
  hipLaunchKernelGGL((qcn::stem_fused_kernel<S, P>), dim3(grid), dim3(C::NTH), C::LDS, st, a);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}
}  // namespace

extern "C" int qcn_resnet_stem_fused(const float* x, int nimg, int h, int w, float in_scale,
                                     int in_zp, const int8_t* w_packed, int cout, const float* u,
                                     const float* v, const float* mult, const int32_t* corr,
                                     int y_zp, int relu, uint8_t* y, void* stream) {
  if (!x || !w_packed || !u || !v || !mult || !corr || !y) return QCN_ERR_ARG;
  if (nimg <= 0 || h <= 0 || w <= 0 || !(in_scale > 0.f) || in_zp < 0 || in_zp > 255 || y_zp < 0 ||
      y_zp > 255)
    return QCN_ERR_ARG;
  if (h != w || (h != 224 && h != 64) || cout != 64) return QCN_ERR_UNSUPPORTED;
  if ((long)nimg * 3 * h * w >= (1L << 31)) return QCN_ERR_UNSUPPORTED;
  qcn::StemArgs a{};
  a.x = x; a.n = nimg; a.inv = 1.0f / in_scale; a.zp = in_zp; a.w = w_packed;
  a.u = u; a.v = v; a.mult = mult; a.corr = corr; a.zp_y = y_zp; a.lo = relu ? y_zp : 0; a.y = y;
  hipStream_t st = (hipStream_t)stream;
  if (h == 64) return launch_stem<64>(a, st);
  // 4 pool rows per band at 224²: a band of 9 conv rows recomputes one shared
  // conv row per 8 instead of per 4 (2 pool rows) and passes its three
  // barriers half as often per image: 0.422 -> 0.329 ms, ResNet-50
  // 106.2-108.2 -> 108.3-109.0 K img/s same box (1 pool row, two workgroups
  // per CU at 128 VGPRs: 0.549 ms; profiles/r03_diag_resnet_stem_band_ab.txt)
  return launch_stem<224, 4>(a, st);
}
