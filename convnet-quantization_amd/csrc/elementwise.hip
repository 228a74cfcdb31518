// HBM-bound helpers of the int8 ConvNet path:
// quantize / dequantize, the PTQ observer min/max, u8 max-pool, argmax.
// All loads/stores are 16 B per lane where the layout allows; grids are capped
// at 8 workgroups per CU (256 CUs) and grid-stride the remainder.
#include "common.hpp"
#include "qconvnet_abi.hpp"

namespace qcn {

constexpr int kMaxGrid = 2048;

static inline int grid_for(long long work, int per_block) {
  long long g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (int)(g < kMaxGrid ? g : kMaxGrid);
}

QCN_DEV int quant_u8(float x, float inv, int zp) {
  float t = x * inv;
  t = fminf(fmaxf(t, -1.0e9f), 1.0e9f);
  int q = (int)__builtin_rintf(t) + zp;
  return q < 0 ? 0 : (q > 255 ? 255 : q);
}

// NCHW fp32 -> NCHW u8, 4 elements per lane.
__global__ void quantize_flat_kernel(const float* __restrict__ x, uint8_t* __restrict__ q,
                                     long long count, float inv, int zp) {
  const long long n4 = count / 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    const uint32_t w = (uint32_t)quant_u8(v.x, inv, zp) | ((uint32_t)quant_u8(v.y, inv, zp) << 8) |
                       ((uint32_t)quant_u8(v.z, inv, zp) << 16) |
                       ((uint32_t)quant_u8(v.w, inv, zp) << 24);
    reinterpret_cast<uint32_t*>(q)[i] = w;
  }
  if (blockIdx.x == 0 && threadIdx.x < (count & 3)) {
    const long long i = n4 * 4 + threadIdx.x;
    q[i] = (uint8_t)quant_u8(x[i], inv, zp);
  }
}

// NCHW fp32 -> NHWC u8: one thread per (n, h, w) pixel, reads are coalesced
// along w for every channel plane.
__global__ void quantize_nchw_nhwc_kernel(const float* __restrict__ x, uint8_t* __restrict__ q,
                                          int n, int c, int hw, float inv, int zp) {
  const long long pix = (long long)n * hw;
  for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < pix;
       p += (long long)gridDim.x * blockDim.x) {
    const long long img = p / hw, off = p % hw;
    const float* src = x + img * c * hw + off;
    uint8_t* dst = q + p * c;
    for (int ch = 0; ch < c; ++ch) dst[ch] = (uint8_t)quant_u8(src[(long long)ch * hw], inv, zp);
  }
}

__global__ void dequantize_kernel(const uint8_t* __restrict__ q, float* __restrict__ x,
                                  long long count, float scale, int zp) {
  const long long n4 = count / 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    const uint32_t w = reinterpret_cast<const uint32_t*>(q)[i];
    float4 o;
    o.x = (float)((int)(w & 0xff) - zp) * scale;
    o.y = (float)((int)((w >> 8) & 0xff) - zp) * scale;
    o.z = (float)((int)((w >> 16) & 0xff) - zp) * scale;
    o.w = (float)((int)(w >> 24) - zp) * scale;
    reinterpret_cast<float4*>(x)[i] = o;
  }
  if (blockIdx.x == 0 && threadIdx.x < (count & 3)) {
    const long long i = n4 * 4 + threadIdx.x;
    x[i] = (float)((int)q[i] - zp) * scale;
  }
}

// ---- observer min/max: per-lane float4 sweep -> wave shuffle -> LDS -> one
// pair of order-preserving integer atomics per workgroup.
QCN_DEV void atomic_min_f32(float* addr, float v) {
  v = v + 0.0f;  // -0.0 -> +0.0 so the integer orderings below agree
  if (v >= 0.0f) atomicMin(reinterpret_cast<int*>(addr), __float_as_int(v));
  else atomicMax(reinterpret_cast<unsigned int*>(addr), __float_as_uint(v));
}
QCN_DEV void atomic_max_f32(float* addr, float v) {
  v = v + 0.0f;
  if (v >= 0.0f) atomicMax(reinterpret_cast<int*>(addr), __float_as_int(v));
  else atomicMin(reinterpret_cast<unsigned int*>(addr), __float_as_uint(v));
}

__global__ void minmax_reset_kernel(float* mm) {
  if (threadIdx.x == 0) {
    mm[0] = __int_as_float(0x7f800000);
    mm[1] = __int_as_float(0xff800000);
  }
}

__global__ __launch_bounds__(256) void minmax_kernel(const float* __restrict__ x,
                                                     long long count, float* mm) {
  float lo = __int_as_float(0x7f800000), hi = __int_as_float(0xff800000);
  const long long n4 = count / 4;
  const uintptr_t mis = (reinterpret_cast<uintptr_t>(x) & 15) ? 1 : 0;
  if (!mis) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
         i += (long long)gridDim.x * blockDim.x) {
      const float4 v = reinterpret_cast<const float4*>(x)[i];
      lo = fminf(lo, fminf(fminf(v.x, v.y), fminf(v.z, v.w)));
      hi = fmaxf(hi, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
    }
  }
  for (long long i = (mis ? 0 : n4 * 4) + blockIdx.x * (long long)blockDim.x + threadIdx.x;
       i < count; i += (long long)gridDim.x * blockDim.x) {
    lo = fminf(lo, x[i]);
    hi = fmaxf(hi, x[i]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, off));
    hi = fmaxf(hi, __shfl_xor(hi, off));
  }
  __shared__ float s_lo[4], s_hi[4];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_lo[wave] = lo;
    s_hi[wave] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      lo = fminf(lo, s_lo[w]);
      hi = fmaxf(hi, s_hi[w]);
    }
    atomic_min_f32(&mm[0], lo);
    atomic_max_f32(&mm[1], hi);
  }
}

// u8 NHWC 2x2 max-pool, 16 channels per lane.
__global__ void maxpool2x2_kernel(const uint8_t* __restrict__ x, int n, int h, int w, int c,
                                  uint8_t* __restrict__ y) {
  const int oh = h / 2, ow = w / 2, c16 = c / 16;
  const long long total = (long long)n * oh * ow * c16;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int cb = (int)(e % c16);
    const long long p = e / c16;
    const int ox = (int)(p % ow), oy = (int)((p / ow) % oh);
    const long long img = p / ((long long)ow * oh);
    const uint8_t* base = x + ((img * h + 2 * oy) * w + 2 * ox) * c + cb * 16;
    uint4 a = *reinterpret_cast<const uint4*>(base);
    uint4 b = *reinterpret_cast<const uint4*>(base + c);
    uint4 d = *reinterpret_cast<const uint4*>(base + (long long)w * c);
    uint4 f = *reinterpret_cast<const uint4*>(base + (long long)w * c + c);
    uint4 r;
    auto mx = [](uint32_t p, uint32_t q) {
      uint32_t o = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t u = (p >> (8 * k)) & 0xff, v = (q >> (8 * k)) & 0xff;
        o |= (u > v ? u : v) << (8 * k);
      }
      return o;
    };
    r.x = mx(mx(a.x, b.x), mx(d.x, f.x));
    r.y = mx(mx(a.y, b.y), mx(d.y, f.y));
    r.z = mx(mx(a.z, b.z), mx(d.z, f.z));
    r.w = mx(mx(a.w, b.w), mx(d.w, f.w));
    *reinterpret_cast<uint4*>(y + p * c + cb * 16) = r;
  }
}

__global__ void maxpool2x2_bytes_kernel(const uint8_t* __restrict__ x, int n, int h, int w, int c,
                                        uint8_t* __restrict__ y) {
  const int oh = h / 2, ow = w / 2;
  const long long total = (long long)n * oh * ow * c;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(e % c);
    const long long p = e / c;
    const int ox = (int)(p % ow), oy = (int)((p / ow) % oh);
    const long long img = p / ((long long)ow * oh);
    const uint8_t* base = x + ((img * h + 2 * oy) * w + 2 * ox) * c + ch;
    uint8_t m = base[0];
    m = base[c] > m ? base[c] : m;
    m = base[(long long)w * c] > m ? base[(long long)w * c] : m;
    m = base[(long long)w * c + c] > m ? base[(long long)w * c + c] : m;
    y[e] = m;
  }
}

// argmax over rows; one wave per row (cols <= a few thousand), ties -> lowest index.
__global__ void argmax_kernel(const float* __restrict__ x, int rows, int cols,
                              long long* __restrict__ idx) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= rows) return;
  const float* r = x + (long long)wave * cols;
  float best = __int_as_float(0xff800000);
  int bi = 0x7fffffff;
  for (int c = lane; c < cols; c += 64) {
    const float v = r[c];
    if (bi == 0x7fffffff || v > best) {  // c increases: ties keep the lowest index
      best = v;
      bi = c;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float ob = __shfl_xor(best, off);
    const int oi = __shfl_xor(bi, off);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  if (lane == 0) idx[wave] = bi;
}

// Inference BatchNorm1d (+ReLU) on [rows, cols] fp32, in ATen's CPU op order
// (probed bit-exact against F.batch_norm(training=False) on the host):
// y = fma(x, alpha[c], beta[c]) with alpha / beta precomputed on the host
// (qconvnet.quant.bn_eval_affine).  One float4 of a row per lane.
__global__ void channel_affine_kernel(const float* __restrict__ x, int rows, int cols,
                                      const float* __restrict__ alpha,
                                      const float* __restrict__ beta, int relu,
                                      float* __restrict__ y) {
  const int c4 = cols / 4;
  const long long total = (long long)rows * c4;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % c4) * 4;
    const float4 v = reinterpret_cast<const float4*>(x)[e];
    const float4 a = *reinterpret_cast<const float4*>(alpha + c);
    const float4 b = *reinterpret_cast<const float4*>(beta + c);
    float4 o = make_float4(__builtin_fmaf(v.x, a.x, b.x), __builtin_fmaf(v.y, a.y, b.y),
                           __builtin_fmaf(v.z, a.z, b.z), __builtin_fmaf(v.w, a.w, b.w));
    if (relu) {
      o.x = fmaxf(o.x, 0.f); o.y = fmaxf(o.y, 0.f); o.z = fmaxf(o.z, 0.f); o.w = fmaxf(o.w, 0.f);
    }
    reinterpret_cast<float4*>(y)[e] = o;
  }
}

}  // namespace qcn

extern "C" {

int qcn_version(void) { return 100; }

int qcn_quantize_f32_u8(const float* x, uint8_t* q, int n, int c, int h, int w, int nhwc_out,
                        float scale, int zero_point, void* stream) {
  if (!x || !q || n <= 0 || c <= 0 || h <= 0 || w <= 0) return QCN_ERR_ARG;
  if (!(scale > 0.f) || zero_point < 0 || zero_point > 255) return QCN_ERR_ARG;
  const float inv = 1.0f / scale;
  hipStream_t st = (hipStream_t)stream;
  if (nhwc_out && c > 1) {
    const long long pix = (long long)n * h * w;
    hipLaunchKernelGGL(qcn::quantize_nchw_nhwc_kernel, dim3(qcn::grid_for(pix, 256)), dim3(256),
                       0, st, x, q, n, c, h * w, inv, zero_point);
  } else {
    const long long cnt = (long long)n * c * h * w;
    if ((reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(q) & 3))
      return QCN_ERR_ARG;
    hipLaunchKernelGGL(qcn::quantize_flat_kernel, dim3(qcn::grid_for(cnt / 4 + 1, 256)),
                       dim3(256), 0, st, x, q, cnt, inv, zero_point);
  }
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_dequantize_u8_f32(const uint8_t* q, float* x, long long count, float scale,
                          int zero_point, void* stream) {
  if (!q || !x || count <= 0) return QCN_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(q) & 3))
    return QCN_ERR_ARG;
  hipLaunchKernelGGL(qcn::dequantize_kernel, dim3(qcn::grid_for(count / 4 + 1, 256)), dim3(256),
                     0, (hipStream_t)stream, q, x, count, scale, zero_point);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_minmax_reset(float* minmax, void* stream) {
  if (!minmax) return QCN_ERR_ARG;
  hipLaunchKernelGGL(qcn::minmax_reset_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, minmax);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_minmax_f32(const float* x, long long count, float* minmax, void* stream) {
  if (!x || !minmax || count < 0) return QCN_ERR_ARG;
  if (count == 0) return QCN_OK;  // observer.py:561 — empty input is a no-op
  hipLaunchKernelGGL(qcn::minmax_kernel, dim3(qcn::grid_for(count / 4 + 1, 256 * 4)), dim3(256),
                     0, (hipStream_t)stream, x, count, minmax);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_maxpool2x2_u8_nhwc(const uint8_t* x, int n, int h, int w, int c, uint8_t* y,
                           void* stream) {
  if (!x || !y || n <= 0 || h < 2 || w < 2 || c <= 0) return QCN_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (c % 16 == 0 && !(reinterpret_cast<uintptr_t>(x) & 15) &&
      !(reinterpret_cast<uintptr_t>(y) & 15)) {
    const long long work = (long long)n * (h / 2) * (w / 2) * (c / 16);
    hipLaunchKernelGGL(qcn::maxpool2x2_kernel, dim3(qcn::grid_for(work, 256)), dim3(256), 0, st,
                       x, n, h, w, c, y);
  } else {
    const long long work = (long long)n * (h / 2) * (w / 2) * c;
    hipLaunchKernelGGL(qcn::maxpool2x2_bytes_kernel, dim3(qcn::grid_for(work, 256)), dim3(256), 0,
                       st, x, n, h, w, c, y);
  }
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_argmax_f32(const float* x, int rows, int cols, long long* idx, void* stream) {
  if (!x || !idx || rows <= 0 || cols <= 0) return QCN_ERR_ARG;
  const int blocks = (rows + 3) / 4;
  hipLaunchKernelGGL(qcn::argmax_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, rows,
                     cols, idx);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_channel_affine_f32(const float* x, int rows, int cols, const float* alpha,
                           const float* beta, int relu, float* y, void* stream) {
  if (!x || !alpha || !beta || !y || rows <= 0 || cols <= 0 || cols % 4) return QCN_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) |
       reinterpret_cast<uintptr_t>(alpha) | reinterpret_cast<uintptr_t>(beta)) & 15)
    return QCN_ERR_ARG;
  const long long work = (long long)rows * (cols / 4);
  hipLaunchKernelGGL(qcn::channel_affine_kernel, dim3(qcn::grid_for(work, 256)), dim3(256), 0,
                     (hipStream_t)stream, x, rows, cols, alpha, beta, relu, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

}  // extern "C"
