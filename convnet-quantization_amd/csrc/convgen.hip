// Generic int8 convolution (any KH x KW, stride, padding; Cin % 32 == 0,
// Cout % 64 == 0) and the dequantize-add-ReLU-quantize residual join — the
// building blocks of the ResNet-style bottleneck blocks of SURVEY §8(f)2
// (custom_quantization_model.py:60-102: 1x1 / 3x3 (strided) / 1x1 convs, a 1x1
// strided downsample, and the residual add done in the float domain).
//
// Implicit GEMM on v_mfma_i32_32x32x32_i8: D[cout][pixel] = W'[cout][k] .
// X'[pixel][k], K = KH*KW*Cin ordered (r, s, c) in 32-byte chunks.  A
// workgroup (4 waves) owns 64*WCO output channels x (4/WCO)*64 output pixels;
// each wave 64 channels x 64 pixels (2 x 2 MFMA tiles).  Weights are packed
// chunk-major [K/32][Cout][32] so an A fragment is one contiguous 1 KB; a B
// fragment row is the 32 input channels of one tap of one pixel (32
// contiguous bytes of the NHWC input), or the zero point outside the image.
// Numerics: identical to conv3x3_u8s8 (FBGEMM requant, A6).
#include "common.hpp"
#include "qconvnet_abi.hpp"

namespace qcn {

struct GenEpi {
  const float *u, *v, *mult;
  const int* corr;   // (128 - zp_x) * sum_k w
  int zp_y, lo;
};

struct GenShape {
  int n, h, w, cin, oh, ow, cout, kh, kw, sy, sx, py, px;
};

template <int WCO>
__global__ __launch_bounds__(256) void conv_gen_kernel(const uint8_t* __restrict__ x, int x_zp,
                                                       const int8_t* __restrict__ wpk, GenShape sh,
                                                       GenEpi ep, uint8_t* __restrict__ y) {
  constexpr int WPX = 4 / WCO;                 // waves along pixels
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hi = lane >> 5;
  const int wc = wave % WCO, wp = wave / WCO;
  const long npix = (long)sh.n * sh.oh * sh.ow;
  const long p0 = (long)blockIdx.x * (WPX * 64) + wp * 64;
  const int co0 = blockIdx.y * (64 * WCO) + wc * 64;
  const int cpt = sh.cin / 32;                 // chunks per tap
  const int kcs = sh.kh * sh.kw * cpt;

  // this lane's two pixels (B rows), as input coordinates of tap (0, 0)
  long xb[2];
  int iy0[2], ix0[2];
  bool pv[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const long p = p0 + j * 32 + l32;
    pv[j] = p < npix;
    const long pc = pv[j] ? p : 0;
    const int ox = (int)(pc % sh.ow), oy = (int)((pc / sh.ow) % sh.oh);
    const int nn = (int)(pc / ((long)sh.ow * sh.oh));
    iy0[j] = oy * sh.sy - sh.py;
    ix0[j] = ox * sh.sx - sh.px;
    xb[j] = (long)nn * sh.h * sh.w;
  }
  const uint32_t padw = xor80(splat_u8(x_zp));
  const int8_t* wa = wpk + ((long)co0 + l32) * 32 + hi * 16;
  const long wstep = (long)sh.cout * 32;

  v16i acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    v16i c0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int4 c4 = *reinterpret_cast<const int4*>(ep.corr + co0 + i * 32 + 8 * g + 4 * hi);
      c0[4 * g] = c4.x; c0[4 * g + 1] = c4.y; c0[4 * g + 2] = c4.z; c0[4 * g + 3] = c4.w;
    }
    acc[i][0] = c0;
    acc[i][1] = c0;
  }

  constexpr int U = 4;
  for (int kc0 = 0; kc0 < kcs; kc0 += U) {
    v4i fa[U][2], fb[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kc = kc0 + u < kcs ? kc0 + u : kcs - 1;
      const bool live = kc0 + u < kcs;
      const int tap = kc / cpt, c0 = (kc % cpt) * 32;
      const int r = tap / sh.kw, s = tap % sh.kw;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        fa[u][i] = live ? *reinterpret_cast<const v4i*>(wa + kc * wstep + i * 32 * 32)
                        : (v4i){0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int iy = iy0[j] + r, ix = ix0[j] + s;
        const bool in = live && pv[j] && iy >= 0 && iy < sh.h && ix >= 0 && ix < sh.w;
        const long off = in ? ((xb[j] + (long)iy * sh.w + ix) * sh.cin + c0 + hi * 16) : 0;
        const uint4 q = *reinterpret_cast<const uint4*>(x + off);
        fb[u][j] = in ? (v4i){(int)xor80(q.x), (int)xor80(q.y), (int)xor80(q.z), (int)xor80(q.w)}
                      : (v4i){(int)padw, (int)padw, (int)padw, (int)padw};
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[u][i], fb[u][j], acc[i][j], 0, 0, 0);
  }

  // epilogue: per-channel requant, 16 consecutive channels per lane -> 16-B stores
  const float zpf = (float)ep.zp_y, lof = (float)ep.lo;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int cb = co0 + i * 32;
    float u[16], v[16], mu[16];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int co = cb + 8 * g + 4 * hi;
      const float4 a = *reinterpret_cast<const float4*>(ep.u + co);
      const float4 b = *reinterpret_cast<const float4*>(ep.v + co);
      const float4 c = *reinterpret_cast<const float4*>(ep.mult + co);
      u[4 * g] = a.x; u[4 * g + 1] = a.y; u[4 * g + 2] = a.z; u[4 * g + 3] = a.w;
      v[4 * g] = b.x; v[4 * g + 1] = b.y; v[4 * g + 2] = b.z; v[4 * g + 3] = b.w;
      mu[4 * g] = c.x; mu[4 * g + 1] = c.y; mu[4 * g + 2] = c.z; mu[4 * g + 3] = c.w;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      uint32_t wv[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint32_t wd = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rg = 4 * g + e;
          wd = __builtin_amdgcn_cvt_pk_u8_f32(requant_f(acc[i][j][rg], u[rg], v[rg], mu[rg], zpf, lof),
                                              e, wd);
        }
        wv[g] = wd;
      }
      auto s01 = __builtin_amdgcn_permlane32_swap(wv[0], wv[1], false, false);
      auto s23 = __builtin_amdgcn_permlane32_swap(wv[2], wv[3], false, false);
      wv[0] = s01[0]; wv[1] = s01[1]; wv[2] = s23[0]; wv[3] = s23[1];
      auto s02 = __builtin_amdgcn_permlane32_swap(wv[0], wv[2], false, false);
      auto s13 = __builtin_amdgcn_permlane32_swap(wv[1], wv[3], false, false);
      wv[0] = s02[0]; wv[2] = s02[1]; wv[1] = s13[0]; wv[3] = s13[1];
      const long p = p0 + j * 32 + l32;
      if (p < npix)
        *reinterpret_cast<uint4*>(y + p * sh.cout + cb + 16 * hi) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
    }
  }
}

// out = quantize(relu?(dequantize(a) + dequantize(b))) with aten op order:
// fp32(s) * (q - z) per operand, an IEEE fp32 add, max(., 0), then
// quantize_per_tensor (zp added after rint).  16 elements per thread.
__global__ void add_relu_u8_kernel(const uint8_t* __restrict__ a, float sa, int za,
                                   const uint8_t* __restrict__ b, float sb, int zb, long count,
                                   float inv_o, int zo, int relu, uint8_t* __restrict__ y) {
  const long i0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (i0 >= count) return;
  if (i0 + 16 <= count) {
    const uint4 va = *reinterpret_cast<const uint4*>(a + i0);
    const uint4 vb = *reinterpret_cast<const uint4*>(b + i0);
    const uint32_t wa[4] = {va.x, va.y, va.z, va.w}, wb[4] = {vb.x, vb.y, vb.z, vb.w};
    uint32_t wo[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint32_t o = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xa = sa * (float)((int)((wa[g] >> (8 * e)) & 0xff) - za);
        const float xb = sb * (float)((int)((wb[g] >> (8 * e)) & 0xff) - zb);
        float s = xa + xb;
        if (relu) s = s > 0.0f ? s : 0.0f;
        const float t = fminf(fmaxf(s * inv_o, -1.0e9f), 1.0e9f);
        int q = (int)__builtin_rintf(t) + zo;
        q = q < 0 ? 0 : (q > 255 ? 255 : q);
        o |= (uint32_t)q << (8 * e);
      }
      wo[g] = o;
    }
    *reinterpret_cast<uint4*>(y + i0) = make_uint4(wo[0], wo[1], wo[2], wo[3]);
  } else {
    for (long i = i0; i < count; ++i) {
      float s = sa * (float)((int)a[i] - za) + sb * (float)((int)b[i] - zb);
      if (relu) s = s > 0.0f ? s : 0.0f;
      const float t = fminf(fmaxf(s * inv_o, -1.0e9f), 1.0e9f);
      int q = (int)__builtin_rintf(t) + zo;
      y[i] = (uint8_t)(q < 0 ? 0 : (q > 255 ? 255 : q));
    }
  }
}

// Byte-wise max of 4 packed u8 (two packed-u16 maxes on the even/odd bytes).
__device__ __forceinline__ uint32_t max_u8x4(uint32_t a, uint32_t b) {
  typedef unsigned short us2 __attribute__((ext_vector_type(2)));
  const uint32_t m = 0x00ff00ffu;
  us2 a0 = __builtin_bit_cast(us2, a & m), b0 = __builtin_bit_cast(us2, b & m);
  us2 a1 = __builtin_bit_cast(us2, (a >> 8) & m), b1 = __builtin_bit_cast(us2, (b >> 8) & m);
  const uint32_t lo = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(a0, b0));
  const uint32_t hi = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(a1, b1));
  return lo | (hi << 8);
}

// nn.MaxPool2d(3, 2, padding=1) on u8 NHWC (torchvision ResNet stem).  Max
// commutes with the monotone dequantize, so the u8 result is exact; a window
// always holds at least one real pixel, so out-of-image taps are skipped.
__global__ void maxpool3x3s2_kernel(const uint8_t* __restrict__ x, int n, int h, int w, int c,
                                    int oh, int ow, uint8_t* __restrict__ y) {
  const int c16 = c / 16;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)n * oh * ow * c16) return;
  const int cb = (int)(e % c16);
  const long p = e / c16;
  const int ox = (int)(p % ow), oy = (int)((p / ow) % oh);
  const long img = p / ((long)ow * oh);
  uint4 r = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy) {
    const int iy = 2 * oy + dy;
    if (iy < 0 || iy >= h) continue;
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      const int ix = 2 * ox + dx;
      if (ix < 0 || ix >= w) continue;
      const uint4 q = *reinterpret_cast<const uint4*>(x + ((img * h + iy) * w + ix) * c + cb * 16);
      r.x = max_u8x4(r.x, q.x); r.y = max_u8x4(r.y, q.y);
      r.z = max_u8x4(r.z, q.z); r.w = max_u8x4(r.w, q.w);
    }
  }
  *reinterpret_cast<uint4*>(y + p * c + cb * 16) = r;
}

// QuantStub + the row im2col of the 7x7/stride-2/pad-3 stem conv on 3 input
// channels: out[n][iy][ox][32] holds, at byte 3*s + ch (s < 7, ch < 3), the
// quantized x[n][ch][iy][2*ox - 3 + s] (the zero point outside the image) and
// the zero point in bytes 21..31.  The stem is then a 7x1 conv with strides
// (2, 1) and padding (3, 0) over Cin = 32 — K = 224 instead of 49 * 32.
__global__ void stem_pack_kernel(const float* __restrict__ x, int n, int h, int w, int ow,
                                 float inv, int zp, uint8_t* __restrict__ y) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)n * h * ow) return;
  const int ox = (int)(e % ow);
  const int iy = (int)((e / ow) % h);
  const long img = e / ((long)ow * h);
  uint32_t wd[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) wd[i] = splat_u8(zp);
#pragma unroll
  for (int s = 0; s < 7; ++s) {
    const int ix = 2 * ox - 3 + s;
    if (ix < 0 || ix >= w) continue;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float v = x[((img * 3 + ch) * h + iy) * w + ix];
      const float t = fminf(fmaxf(v * inv, -1.0e9f), 1.0e9f);
      int q = (int)__builtin_rintf(t) + zp;
      q = q < 0 ? 0 : (q > 255 ? 255 : q);
      const int b = 3 * s + ch;
      wd[b >> 2] = (wd[b >> 2] & ~(0xffu << (8 * (b & 3)))) | ((uint32_t)q << (8 * (b & 3)));
    }
  }
  uint4* o = reinterpret_cast<uint4*>(y + e * 32);
  o[0] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
  o[1] = make_uint4(wd[4], wd[5], wd[6], wd[7]);
}

// Global average pool on u8 NHWC, quantization parameters kept (torch's
// quantized adaptive_avg_pool2d to 1x1, what a static-int8 ResNet runs before
// its fc): per (image, channel) acc = sum_q - hw * zp (exact), then
// q = clamp(zp + rne(fp32(acc) * fp32(1 / hw)), 0, 255) — probed bit-exact
// against torch 2.10 (fbgemm) at 2x2 and 7x7 with ties (oracle qref.avgpool_q).
// 4 channels per thread.
__global__ void avgpool_kernel(const uint8_t* __restrict__ x, int n, int hw, int c, int zp,
                               float inv_hw, uint8_t* __restrict__ y) {
  const int c4 = c / 4;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)n * c4) return;
  const int cb = (int)(e % c4);
  const long img = e / c4;
  const uint8_t* base = x + img * hw * c + cb * 4;
  int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  for (int p = 0; p < hw; ++p) {
    const uint32_t q = *reinterpret_cast<const uint32_t*>(base + (long)p * c);
    s0 += q & 0xff; s1 += (q >> 8) & 0xff; s2 += (q >> 16) & 0xff; s3 += q >> 24;
  }
  const int sums[4] = {s0, s1, s2, s3};
  const float zpf = (float)zp;
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float t = __builtin_rintf((float)(sums[i] - hw * zp) * inv_hw) + zpf;   // exact integer
    o = __builtin_amdgcn_cvt_pk_u8_f32(t, i, o);                                    // clamp [0, 255]
  }
  *reinterpret_cast<uint32_t*>(y + img * c + cb * 4) = o;
}

}  // namespace qcn

extern "C" {

int qcn_pack_conv_weight_kmajor(const int8_t* w_oihw, int cout, int cin, int kh, int kw,
                                int8_t* out, int32_t* wsum) {
  if (!w_oihw || !out || !wsum || cout <= 0 || cin <= 0 || kh <= 0 || kw <= 0 || cin % 32 != 0)
    return QCN_ERR_ARG;
  const int cpt = cin / 32;
  for (int co = 0; co < cout; ++co) {
    int32_t s = 0;
    for (int c = 0; c < cin; ++c)
      for (int r = 0; r < kh; ++r)
        for (int t = 0; t < kw; ++t) {
          const int8_t v = w_oihw[(((long)co * cin + c) * kh + r) * kw + t];
          s += v;
          const int kc = (r * kw + t) * cpt + c / 32;
          out[((long)kc * cout + co) * 32 + c % 32] = v;
        }
    wsum[co] = s;
  }
  return QCN_OK;
}

int qcn_conv_u8s8_nhwc(const uint8_t* x, int nimg, int h, int w, int cin, int x_zp,
                       const int8_t* w_packed, int cout, int kh, int kw, int stride_h,
                       int stride_w, int pad_h, int pad_w, const float* u, const float* v,
                       const float* mult, const int32_t* corr, int y_zp, int relu, uint8_t* y,
                       void* stream) {
  if (!x || !w_packed || !u || !v || !mult || !corr || !y) return QCN_ERR_ARG;
  if (nimg <= 0 || h <= 0 || w <= 0 || cin <= 0 || cout <= 0 || kh <= 0 || kw <= 0 ||
      stride_h <= 0 || stride_w <= 0 || pad_h < 0 || pad_w < 0 || x_zp < 0 || x_zp > 255 ||
      y_zp < 0 || y_zp > 255)
    return QCN_ERR_ARG;
  if (cin % 32 != 0 || cout % 64 != 0) return QCN_ERR_UNSUPPORTED;
  const int oh = (h + 2 * pad_h - kh) / stride_h + 1, ow = (w + 2 * pad_w - kw) / stride_w + 1;
  if (oh <= 0 || ow <= 0) return QCN_ERR_ARG;
  qcn::GenShape sh{nimg, h, w, cin, oh, ow, cout, kh, kw, stride_h, stride_w, pad_h, pad_w};
  qcn::GenEpi ep{u, v, mult, corr, y_zp, relu ? y_zp : 0};
  const long npix = (long)nimg * oh * ow;
  hipStream_t st = (hipStream_t)stream;
  if (cout % 128 == 0) {
    dim3 grid((unsigned)((npix + 127) / 128), cout / 128);
    hipLaunchKernelGGL(qcn::conv_gen_kernel<2>, grid, dim3(256), 0, st, x, x_zp, w_packed, sh, ep, y);
  } else {
    dim3 grid((unsigned)((npix + 255) / 256), cout / 64);
    hipLaunchKernelGGL(qcn::conv_gen_kernel<1>, grid, dim3(256), 0, st, x, x_zp, w_packed, sh, ep, y);
  }
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_maxpool3x3s2_u8_nhwc(const uint8_t* x, int nimg, int h, int w, int c, uint8_t* y,
                             void* stream) {
  if (!x || !y || nimg <= 0 || h <= 0 || w <= 0 || c <= 0) return QCN_ERR_ARG;
  if (c % 16 != 0) return QCN_ERR_UNSUPPORTED;
  const int oh = (h - 1) / 2 + 1, ow = (w - 1) / 2 + 1;
  const long total = (long)nimg * oh * ow * (c / 16);
  hipLaunchKernelGGL(qcn::maxpool3x3s2_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, x, nimg, h, w, c, oh, ow, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_stem_pack_f32_nchw(const float* x, int nimg, int h, int w, float scale, int zp, uint8_t* y,
                           void* stream) {
  if (!x || !y || nimg <= 0 || h <= 0 || w <= 0 || !(scale > 0.f) || zp < 0 || zp > 255)
    return QCN_ERR_ARG;
  const int ow = (w - 1) / 2 + 1;
  const long total = (long)nimg * h * ow;
  hipLaunchKernelGGL(qcn::stem_pack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, x, nimg, h, w, ow, 1.0f / scale, zp, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_avgpool_u8_nhwc(const uint8_t* x, int nimg, int hw, int c, int x_zp, uint8_t* y,
                        void* stream) {
  if (!x || !y || nimg <= 0 || hw <= 0 || c <= 0 || x_zp < 0 || x_zp > 255) return QCN_ERR_ARG;
  if (c % 4 != 0 || hw > (1 << 16)) return QCN_ERR_UNSUPPORTED;
  const long total = (long)nimg * (c / 4);
  hipLaunchKernelGGL(qcn::avgpool_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, x, nimg, hw, c, x_zp, 1.0f / (float)hw, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_add_relu_u8(const uint8_t* a, float sa, int za, const uint8_t* b, float sb, int zb,
                    long long count, float s_out, int z_out, int relu, uint8_t* y, void* stream) {
  if (!a || !b || !y || count < 0 || !(s_out > 0.f) || za < 0 || za > 255 || zb < 0 || zb > 255 ||
      z_out < 0 || z_out > 255)
    return QCN_ERR_ARG;
  if (count == 0) return QCN_OK;
  const long th = (count + 15) / 16;
  hipLaunchKernelGGL(qcn::add_relu_u8_kernel, dim3((unsigned)((th + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, a, sa, za, b, sb, zb, (long)count, 1.0f / s_out, z_out,
                     relu, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

}  // extern "C"
