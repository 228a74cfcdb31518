// ResNet bottleneck blocks in the reference's own semantics:
// CustomQuantizedBottleneck / CustomQuantizedResNet50
// (/root/reference/models/custom_quantization_model.py:60-143) with the
// per-layer stubs live.  Every conv is QuantStub -> int8 conv -> DeQuantStub
// (:34-45); BN, ReLU, the stem's max-pool, the residual add (:95-101) and the
// average pool stay fp32.  The int8 convs are the LDS-tiled implicit-GEMM
// kernel (convgemm.hip, requant to the conv's own output qparams, no ReLU);
// this file holds the fp32 hand-offs between them, each fused with the next
// stub's quantize so a conv's input is written once, as u8:
//
//   dq_bn_q_kernel          conv -> DeQuantStub -> BN -> [ReLU] -> next QuantStub
//   dq_bn_relu_maxpool      stem conv -> DeQuantStub -> BN -> ReLU -> max-pool
//                           3x3/2 (fp32 block input) + block 0's QuantStub
//   qdq_join_kernel         conv3 -> DeQuantStub -> BN3 (+ downsample conv ->
//                           DeQuantStub -> BN, or the fp32 identity) -> add ->
//                           ReLU (fp32 block output) + next block's QuantStub
//   avgpool_f32_kernel      AdaptiveAvgPool2d(1) on the fp32 map
//
// Numerics (oracle/qref.py resnet_qdq_forward, pinned to torch.ao by
// tests/golden/net_resnet_qdq.npz): dequantize fp32(q - z) * s; BN eval
// y = fmaf(x, alpha, beta) with alpha / beta from ATen's eval constants
// (host, qconvnet/quant.py bn_eval_affine); ReLU keeps -0.0 like
// torch.relu; quantize zp + rint(x * fp32(1/s)) clamped; avg-pool a
// sequential fp32 sum in row-major window order, then / (H*W).  All NHWC,
// channel innermost, 4 channels per lane (C % 4 == 0).
#include "common.hpp"
#include "qconvnet_abi.hpp"

namespace qcn {
namespace {

QCN_DEV float relu_keep_sign(float y) { return y < 0.f ? 0.f : y; }

QCN_DEV int quant_q(float x, float inv, int zp) {
  float t = x * inv;
  t = fminf(fmaxf(t, -1.0e9f), 1.0e9f);
  const int q = (int)__builtin_rintf(t) + zp;
  return q < 0 ? 0 : (q > 255 ? 255 : q);
}

QCN_DEV float dq_bn(uint32_t q, int z, float s, float a, float b) {
  return __builtin_fmaf((float)((int)q - z) * s, a, b);
}

int grid_of(long long work) {
  long long g = (work + 255) / 256;
  if (g < 1) g = 1;
  return (int)(g < 4096 ? g : 4096);
}

__global__ __launch_bounds__(256) void dq_bn_q_kernel(const uint8_t* __restrict__ y, long long n4,
                                                      int c, float s, int z,
                                                      const float* __restrict__ alpha,
                                                      const float* __restrict__ beta, int relu,
                                                      float inv_next, int z_next,
                                                      uint8_t* __restrict__ out) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const int c0 = (int)((i * 4) % c);
    const uint32_t v = reinterpret_cast<const uint32_t*>(y)[i];
    const float4 a = *reinterpret_cast<const float4*>(alpha + c0);
    const float4 b = *reinterpret_cast<const float4*>(beta + c0);
    const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
    uint32_t w = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float f = dq_bn((v >> (8 * j)) & 0xff, z, s, av[j], bv[j]);
      if (relu) f = relu_keep_sign(f);
      w |= (uint32_t)quant_q(f, inv_next, z_next) << (8 * j);
    }
    reinterpret_cast<uint32_t*>(out)[i] = w;
  }
}

// stem: u8 [n][h][w][c] -> fp32 max-pool 3x3/2 pad 1 of relu(bn(dq(.)))
// (each window element mapped first: BN may be decreasing) + its u8 quantize
__global__ __launch_bounds__(256) void dq_bn_relu_maxpool_kernel(
    const uint8_t* __restrict__ y, int n, int h, int w, int c, float s, int z,
    const float* __restrict__ alpha, const float* __restrict__ beta, float* __restrict__ out,
    float inv_next, int z_next, uint8_t* __restrict__ out_q) {
  const int oh = (h - 1) / 2 + 1, ow = (w - 1) / 2 + 1, c4 = c / 4;
  const long long total = (long long)n * oh * ow * c4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int cg = (int)(i % c4);
    const long long p = i / c4;
    const int ox = (int)(p % ow), oy = (int)((p / ow) % oh), img = (int)(p / ((long long)ow * oh));
    const float4 a = *reinterpret_cast<const float4*>(alpha + 4 * cg);
    const float4 b = *reinterpret_cast<const float4*>(beta + 4 * cg);
    const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
    float m[4] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    for (int r = 0; r < 3; ++r) {
      const int iy = 2 * oy - 1 + r;
      if (iy < 0 || iy >= h) continue;
      for (int t = 0; t < 3; ++t) {
        const int ix = 2 * ox - 1 + t;
        if (ix < 0 || ix >= w) continue;
        const uint32_t v = *reinterpret_cast<const uint32_t*>(y + (((long long)img * h + iy) * w + ix) * c + 4 * cg);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float f = relu_keep_sign(dq_bn((v >> (8 * j)) & 0xff, z, s, av[j], bv[j]));
          m[j] = f > m[j] ? f : m[j];   // nn.MaxPool2d keeps the first maximum
        }
      }
    }
    reinterpret_cast<float4*>(out)[i] = make_float4(m[0], m[1], m[2], m[3]);
    if (out_q) {
      uint32_t wq = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) wq |= (uint32_t)quant_q(m[j], inv_next, z_next) << (8 * j);
      reinterpret_cast<uint32_t*>(out_q)[i] = wq;
    }
  }
}

// out = relu(bn3(dq(y3)) + identity), identity = bn_d(dq(yd)) or idf (fp32)
__global__ __launch_bounds__(256) void qdq_join_kernel(
    const uint8_t* __restrict__ y3, float s3, int z3, const float* __restrict__ a3,
    const float* __restrict__ b3, const uint8_t* __restrict__ yd, float sd, int zd,
    const float* __restrict__ ad, const float* __restrict__ bd, const float* __restrict__ idf,
    long long n4, int c, float* __restrict__ out, float inv_next, int z_next,
    uint8_t* __restrict__ out_q) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const int c0 = (int)((i * 4) % c);
    const uint32_t v = reinterpret_cast<const uint32_t*>(y3)[i];
    const float4 a = *reinterpret_cast<const float4*>(a3 + c0);
    const float4 b = *reinterpret_cast<const float4*>(b3 + c0);
    const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
    float idv[4];
    if (yd) {
      const uint32_t u = reinterpret_cast<const uint32_t*>(yd)[i];
      const float4 a2 = *reinterpret_cast<const float4*>(ad + c0);
      const float4 b2 = *reinterpret_cast<const float4*>(bd + c0);
      const float av2[4] = {a2.x, a2.y, a2.z, a2.w}, bv2[4] = {b2.x, b2.y, b2.z, b2.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) idv[j] = dq_bn((u >> (8 * j)) & 0xff, zd, sd, av2[j], bv2[j]);
    } else {
      const float4 f = reinterpret_cast<const float4*>(idf)[i];
      idv[0] = f.x; idv[1] = f.y; idv[2] = f.z; idv[3] = f.w;
    }
    float o[4];
    uint32_t wq = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = relu_keep_sign(dq_bn((v >> (8 * j)) & 0xff, z3, s3, av[j], bv[j]) + idv[j]);
      wq |= (uint32_t)quant_q(o[j], inv_next, z_next) << (8 * j);
    }
    reinterpret_cast<float4*>(out)[i] = make_float4(o[0], o[1], o[2], o[3]);
    if (out_q) reinterpret_cast<uint32_t*>(out_q)[i] = wq;
  }
}

// [n][hw][c] fp32 -> [n][c]: one lane per (image, 4 channels), sequential sum
__global__ __launch_bounds__(256) void avgpool_f32_kernel(const float* __restrict__ x, int n, int hw,
                                                          int c, float* __restrict__ out) {
  const int c4 = c / 4;
  const long long total = (long long)n * c4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int cg = (int)(i % c4), img = (int)(i / c4);
    const float4* p = reinterpret_cast<const float4*>(x + (long long)img * hw * c) + cg;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 0; k < hw; ++k) {
      const float4 v = p[(long long)k * c4];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    const float d = (float)hw;
    reinterpret_cast<float4*>(out)[i] = make_float4(acc.x / d, acc.y / d, acc.z / d, acc.w / d);
  }
}

bool aligned(const void* p, int a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; }

}  // namespace
}  // namespace qcn

extern "C" {

int qcn_dq_bn_q_u8(const uint8_t* y, long long count, int c, float s, int z, const float* alpha,
                   const float* beta, int relu, float s_next, int z_next, uint8_t* out,
                   void* stream) {
  if (!y || !alpha || !beta || !out || count <= 0 || c <= 0 || c % 4 || count % c) return QCN_ERR_ARG;
  if (!(s > 0.f) || !(s_next > 0.f) || z < 0 || z > 255 || z_next < 0 || z_next > 255) return QCN_ERR_ARG;
  if (!qcn::aligned(y, 4) || !qcn::aligned(out, 4) || !qcn::aligned(alpha, 16) || !qcn::aligned(beta, 16))
    return QCN_ERR_ARG;
  const long long n4 = count / 4;
  hipLaunchKernelGGL(qcn::dq_bn_q_kernel, dim3(qcn::grid_of(n4)), dim3(256), 0, (hipStream_t)stream,
                     y, n4, c, s, z, alpha, beta, relu ? 1 : 0, 1.0f / s_next, z_next, out);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_dq_bn_relu_maxpool_f32(const uint8_t* y, int n, int h, int w, int c, float s, int z,
                               const float* alpha, const float* beta, float* out, float s_next,
                               int z_next, uint8_t* out_q, void* stream) {
  if (!y || !alpha || !beta || !out || n <= 0 || h <= 0 || w <= 0 || c <= 0 || c % 4) return QCN_ERR_ARG;
  if (!(s > 0.f) || z < 0 || z > 255 || (out_q && (!(s_next > 0.f) || z_next < 0 || z_next > 255)))
    return QCN_ERR_ARG;
  if (!qcn::aligned(y, 4) || !qcn::aligned(out, 16) || (out_q && !qcn::aligned(out_q, 4)) ||
      !qcn::aligned(alpha, 16) || !qcn::aligned(beta, 16))
    return QCN_ERR_ARG;
  const long long total = (long long)n * ((h - 1) / 2 + 1) * ((w - 1) / 2 + 1) * (c / 4);
  hipLaunchKernelGGL(qcn::dq_bn_relu_maxpool_kernel, dim3(qcn::grid_of(total)), dim3(256), 0,
                     (hipStream_t)stream, y, n, h, w, c, s, z, alpha, beta, out,
                     out_q ? 1.0f / s_next : 0.f, z_next, out_q);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_qdq_join_f32(const uint8_t* y3, float s3, int z3, const float* a3, const float* b3,
                     const uint8_t* yd, float sd, int zd, const float* ad, const float* bd,
                     const float* idf, long long count, int c, float* out, float s_next, int z_next,
                     uint8_t* out_q, void* stream) {
  if (!y3 || !a3 || !b3 || !out || count <= 0 || c <= 0 || c % 4 || count % c) return QCN_ERR_ARG;
  if ((yd == nullptr) == (idf == nullptr)) return QCN_ERR_ARG;   // exactly one identity operand
  if (yd && (!ad || !bd || !(sd > 0.f) || zd < 0 || zd > 255)) return QCN_ERR_ARG;
  if (!(s3 > 0.f) || z3 < 0 || z3 > 255 || (out_q && (!(s_next > 0.f) || z_next < 0 || z_next > 255)))
    return QCN_ERR_ARG;
  if (!qcn::aligned(y3, 4) || !qcn::aligned(out, 16) || (yd && !qcn::aligned(yd, 4)) ||
      (idf && !qcn::aligned(idf, 16)) || (out_q && !qcn::aligned(out_q, 4)) || !qcn::aligned(a3, 16) ||
      !qcn::aligned(b3, 16) || (yd && (!qcn::aligned(ad, 16) || !qcn::aligned(bd, 16))))
    return QCN_ERR_ARG;
  const long long n4 = count / 4;
  hipLaunchKernelGGL(qcn::qdq_join_kernel, dim3(qcn::grid_of(n4)), dim3(256), 0, (hipStream_t)stream,
                     y3, s3, z3, a3, b3, yd, sd, zd, ad, bd, idf, n4, c, out,
                     out_q ? 1.0f / s_next : 0.f, z_next, out_q);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_avgpool_f32_nhwc(const float* x, int n, int h, int w, int c, float* out, void* stream) {
  if (!x || !out || n <= 0 || h <= 0 || w <= 0 || c <= 0 || c % 4) return QCN_ERR_ARG;
  if (!qcn::aligned(x, 16) || !qcn::aligned(out, 16)) return QCN_ERR_ARG;
  hipLaunchKernelGGL(qcn::avgpool_f32_kernel, dim3(qcn::grid_of((long long)n * (c / 4))), dim3(256), 0,
                     (hipStream_t)stream, x, n, h * w, c, out);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

}  // extern "C"
