// int8 Linear layers of the ConvNet path:
//  * static u8 x s8 -> u8 (QuantizedLinear / QuantizedLinearReLU, fbgemm),
//    optional fused DeQuantStub (fp32 logits);
//  * dynamic fp32 -> fp32 (quantized::linear_dynamic): device-side min/max,
//    ChooseQuantizationParams, LEGACY quantize, GEMM, fp32 epilogue;
//  * plain fp32 Linear (the fp32 fc2 of CustomQuantizedSimpleConvNet).
//
// GEMM shape: D[feature][row] = W[feature][k] * X[row][k]^T on
// v_mfma_i32_32x32x32_i8.  A workgroup (4 waves) owns 64 features x 32 rows
// and splits K four ways across its waves; partial accumulators are summed
// through LDS.  fc1 at batch 1024 -> 8 x 32 = 256 workgroups (one per CU).
#include "common.hpp"
#include "qconvnet_abi.hpp"

namespace qcn {

struct LinEpi {
  const float* u;
  const float* v;
  const float* mult;
  const int* corr;        // static: (128 - zx) * wsum; dynamic: wsum (zx from device)
  int zp_y, lo;
  float y_scale;          // dequant scale for y_deq
  // dynamic
  const float* w_scale;   // [1] or [n]
  int per_channel;
  const float* bias;      // may be null
  const float* dyn;       // device qparams: [scale, inv, zp(float), zp(int bits)]
};

template <bool DYN>
__global__ __launch_bounds__(256) void linear_u8s8_kernel(
    const uint8_t* __restrict__ x, int m, int k, int x_zp, const int8_t* __restrict__ w, int n,
    LinEpi ep, uint8_t* __restrict__ y, float* __restrict__ yf) {
  __shared__ __attribute__((aligned(16))) int part[3][2][16][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hi = lane >> 5;
  const int f0 = blockIdx.x * 64, r0 = blockIdx.y * 32;
  const int kq = k / 4;
  const int kb = wave * kq;

  const int row = r0 + l32;
  const bool row_ok = row < m;
  const uint8_t* xr = x + (long)(row_ok ? row : 0) * k + hi * 16;
  const int8_t* wr[2];
  bool f_ok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int f = f0 + i * 32 + l32;
    f_ok[i] = f < n;
    wr[i] = w + (long)(f_ok[i] ? f : 0) * k + hi * 16;
  }
  v16i acc[2] = {(v16i){0}, (v16i){0}};
  // 4 K-steps of loads in flight per batch (the loop is latency-bound otherwise)
  constexpr int U = 4;
  int kk = kb;
  for (; kk + 32 * U <= kb + kq; kk += 32 * U) {
    uint4 xb[U];
    v4i wa[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xb[u] = *reinterpret_cast<const uint4*>(xr + kk + 32 * u);
#pragma unroll
      for (int i = 0; i < 2; ++i) wa[u][i] = *reinterpret_cast<const v4i*>(wr[i] + kk + 32 * u);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const v4i b = (v4i){(int)xor80(xb[u].x), (int)xor80(xb[u].y), (int)xor80(xb[u].z),
                          (int)xor80(xb[u].w)};
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const v4i a = f_ok[i] ? wa[u][i] : (v4i){0, 0, 0, 0};
        acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
      }
    }
  }
  for (; kk < kb + kq; kk += 32) {
    uint4 xb = *reinterpret_cast<const uint4*>(xr + kk);
    const v4i b = (v4i){(int)xor80(xb.x), (int)xor80(xb.y), (int)xor80(xb.z), (int)xor80(xb.w)};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      v4i a = *reinterpret_cast<const v4i*>(wr[i] + kk);
      if (!f_ok[i]) a = (v4i){0, 0, 0, 0};
      acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
    }
  }
  if (wave > 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int rg = 0; rg < 16; ++rg) part[wave - 1][i][rg][lane] = acc[i][rg];
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int rg = 0; rg < 16; ++rg)
      acc[i][rg] += part[0][i][rg][lane] + part[1][i][rg][lane] + part[2][i][rg][lane];

  if (!row_ok) return;
  int zx = x_zp;
  float s_x = 0.f;
  if constexpr (DYN) {
    s_x = ep.dyn[0];
    zx = __float_as_int(ep.dyn[3]);
  }
  const bool vec_ok = (n % 4) == 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      int qv[4];
      float fv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rg = 4 * g + e;
        const int f = f0 + i * 32 + e + 8 * g + 4 * hi;
        if (f >= n) { qv[e] = 0; fv[e] = 0.f; continue; }
        if constexpr (DYN) {
          const int a = acc[i][rg] + (128 - zx) * ep.corr[f];
          const float sw = ep.per_channel ? ep.w_scale[f] : ep.w_scale[0];
          const float aws = s_x * sw;
          const float b = ep.bias ? ep.bias[f] : 0.0f;
          fv[e] = __builtin_fmaf((float)a, aws, b);
        } else {
          const int q = requant_one(acc[i][rg] + ep.corr[f], ep.u[f], ep.v[f], ep.mult[f],
                                    ep.zp_y, ep.lo);
          qv[e] = q;
          fv[e] = (float)(q - ep.zp_y) * ep.y_scale;
        }
      }
      const int fb = f0 + i * 32 + 8 * g + 4 * hi;
      if (fb >= n) continue;
      if constexpr (!DYN) {
        if (vec_ok && fb + 3 < n) {
          *reinterpret_cast<uint32_t*>(y + (long)row * n + fb) =
              (uint32_t)qv[0] | ((uint32_t)qv[1] << 8) | ((uint32_t)qv[2] << 16) |
              ((uint32_t)qv[3] << 24);
        } else {
          for (int e = 0; e < 4 && fb + e < n; ++e) y[(long)row * n + fb + e] = (uint8_t)qv[e];
        }
      }
      if (yf != nullptr) {
        if (vec_ok && fb + 3 < n) {
          *reinterpret_cast<float4*>(yf + (long)row * n + fb) = make_float4(fv[0], fv[1], fv[2], fv[3]);
        } else {
          for (int e = 0; e < 4 && fb + e < n; ++e) yf[(long)row * n + fb + e] = fv[e];
        }
      }
    }
  }
}

// Generic fallback for K not a multiple of 128: one thread per output.
template <bool DYN>
__global__ void linear_generic_kernel(const uint8_t* __restrict__ x, int m, int k, int x_zp,
                                      const int8_t* __restrict__ w, int n, LinEpi ep,
                                      uint8_t* __restrict__ y, float* __restrict__ yf) {
  const long total = (long)m * n;
  int zx = x_zp;
  float s_x = 0.f;
  if constexpr (DYN) {
    s_x = ep.dyn[0];
    zx = __float_as_int(ep.dyn[3]);
  }
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int f = (int)(e % n);
    const long row = e / n;
    int acc = 0;
    for (int kk = 0; kk < k; ++kk) acc += ((int)x[row * k + kk] - zx) * (int)w[(long)f * k + kk];
    if constexpr (DYN) {
      const float sw = ep.per_channel ? ep.w_scale[f] : ep.w_scale[0];
      yf[e] = __builtin_fmaf((float)acc, s_x * sw, ep.bias ? ep.bias[f] : 0.0f);
    } else {
      const int q = requant_one(acc, ep.u[f], ep.v[f], ep.mult[f], ep.zp_y, ep.lo);
      y[e] = (uint8_t)q;
      if (yf) yf[e] = (float)(q - ep.zp_y) * ep.y_scale;
    }
  }
}

// ATen ChooseQuantizationParams (torch/include/ATen/native/quantized/cpu/
// QuantUtils.h:70-185) on the device, preserve_sparsity = false,
// force_scale_power_of_two = false.  dyn = [scale, inv, zp_f, zp_i(bits)].
__global__ void choose_qparams_kernel(const float* __restrict__ mm, int reduce_range, float* dyn) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int qmin = 0, qmax = 255;
  if (reduce_range) { qmin = qmin / 2; qmax = qmax / 2; }
  float mn = fminf(mm[0], 0.f), mx = fmaxf(mm[1], 0.f);
  double scale = ((double)mx - (double)mn) / (double)(qmax - qmin);
  if ((float)scale == 0.0f || __builtin_isinf(1.0f / (float)scale)) scale = 0.1;
  const float kSmall = 6.1e-5f;
  if (scale < (double)kSmall) {
    const float org = (float)scale;
    scale = (double)kSmall;
    if (mn == 0.0f) mx = kSmall * (float)(qmax - qmin);
    else if (mx == 0.0f) mn = -kSmall * (float)(qmax - qmin);
    else {
      const float amp = kSmall / org;
      mn *= amp;
      mx *= amp;
    }
  }
  const double zfm = (double)qmin - (double)mn / scale;
  const double zfx = (double)qmax - (double)mx / scale;
  const double efm = fabs((double)qmin) - fabs((double)mn / scale);
  const double efx = fabs((double)qmax) - fabs((double)mx / scale);
  const double z0 = efm < efx ? zfm : zfx;
  int zp;
  if (z0 < qmin) zp = qmin;
  else if (z0 > qmax) zp = qmax;
  else zp = (int)rint(z0);
  const float sf = (float)scale;
  dyn[0] = sf;
  dyn[1] = 1.0f / sf;
  dyn[2] = (float)zp;
  dyn[3] = __int_as_float(zp);
}

// fbgemm::QuantizeAvx2<uint8_t, LEGACY=true>: q = clamp(rne(min(fmaf(x, inv, zp), 255)), 0, 255).
__global__ void quantize_legacy_kernel(const float* __restrict__ x, long long count,
                                       const float* __restrict__ dyn, uint8_t* __restrict__ q) {
  const float inv = dyn[1], zpf = dyn[2];
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < count;
       i += (long long)gridDim.x * blockDim.x) {
    float t = __builtin_fmaf(x[i], inv, zpf);
    t = fminf(t, 255.0f);
    t = __builtin_rintf(t);
    t = fmaxf(t, 0.0f);
    q[i] = (uint8_t)(int)t;
  }
}

// One wave per row: lane l takes k-elements l, l + 64, ...; up to 16 outputs
// per pass (fma chains per lane, then a wave reduction by xor shuffles).
__global__ __launch_bounds__(256) void linear_f32_kernel(const float* __restrict__ x, int m, int k,
                                                         const float* __restrict__ w, int n,
                                                         const float* __restrict__ b, int relu_in,
                                                         float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= m) return;
  const float* xr = x + row * k;
  for (int f0 = 0; f0 < n; f0 += 16) {
    float acc[16];
#pragma unroll
    for (int o = 0; o < 16; ++o) acc[o] = 0.f;
    for (int kk = lane; kk < k; kk += 64) {
      float xv = xr[kk];
      if (relu_in) xv = xv > 0.f ? xv : 0.f;
#pragma unroll
      for (int o = 0; o < 16; ++o)
        if (f0 + o < n) acc[o] = __builtin_fmaf(xv, w[(long)(f0 + o) * k + kk], acc[o]);
    }
#pragma unroll
    for (int o = 0; o < 16; ++o) {
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) acc[o] += __shfl_xor(acc[o], d);
    }
    float mine = 0.f;
#pragma unroll
    for (int o = 0; o < 16; ++o)
      if (lane == o) mine = acc[o];
    if (lane < 16 && f0 + lane < n) y[row * n + f0 + lane] = mine + (b ? b[f0 + lane] : 0.f);
  }
}

}  // namespace qcn

// minmax kernels live in elementwise.hip
extern "C" int qcn_minmax_reset(float* minmax, void* stream);
extern "C" int qcn_minmax_f32(const float* x, long long count, float* minmax, void* stream);

extern "C" {

int qcn_linear_u8s8(const uint8_t* x, int m, int k, int x_zp, const int8_t* w, int n,
                    const float* u, const float* v, const float* mult, const int32_t* corr,
                    int y_zp, int relu, uint8_t* y, float* y_deq, float y_scale, void* stream) {
  if (!x || !w || !u || !v || !mult || !corr || !y) return QCN_ERR_ARG;
  if (m <= 0 || k <= 0 || n <= 0 || x_zp < 0 || x_zp > 255 || y_zp < 0 || y_zp > 255)
    return QCN_ERR_ARG;
  qcn::LinEpi ep{u, v, mult, corr, y_zp, relu ? y_zp : 0, y_scale, nullptr, 0, nullptr, nullptr};
  hipStream_t st = (hipStream_t)stream;
  if (k % 128 == 0) {
    dim3 grid((n + 63) / 64, (m + 31) / 32);
    hipLaunchKernelGGL(qcn::linear_u8s8_kernel<false>, grid, dim3(256), 0, st, x, m, k, x_zp, w, n,
                       ep, y, y_deq);
  } else {
    // generic path takes the raw zero point, not the (128 - zp) * wsum correction
    const long total = (long)m * n;
    const int grid = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(qcn::linear_generic_kernel<false>, dim3(grid), dim3(256), 0, st, x, m, k,
                       x_zp, w, n, ep, y, y_deq);
  }
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

long long qcn_linear_dynamic_workspace_size(int m, int k) { return 64 + (long long)m * k; }

static int linear_dynamic_impl(const float* x, int m, int k, const int8_t* w, int n,
                               const float* w_scale, int per_channel, const int32_t* wsum,
                               const float* bias, int reduce_range, const float* ext_minmax,
                               float* y, void* workspace, void* stream) {
  if (!x || !w || !w_scale || !wsum || !y || !workspace) return QCN_ERR_ARG;
  if (m <= 0 || k <= 0 || n <= 0) return QCN_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  float* mm = reinterpret_cast<float*>(workspace);
  float* dyn = mm + 4;
  uint8_t* qx = reinterpret_cast<uint8_t*>(workspace) + 64;
  const float* range = ext_minmax;
  if (!range) {   // this batch's own [min, max]
    int rc = qcn_minmax_reset(mm, stream);
    if (rc) return rc;
    rc = qcn_minmax_f32(x, (long long)m * k, mm, stream);
    if (rc) return rc;
    range = mm;
  }
  hipLaunchKernelGGL(qcn::choose_qparams_kernel, dim3(1), dim3(64), 0, st, range, reduce_range, dyn);
  const long long cnt = (long long)m * k;
  int g = (int)((cnt + 255) / 256 < 2048 ? (cnt + 255) / 256 : 2048);
  hipLaunchKernelGGL(qcn::quantize_legacy_kernel, dim3(g), dim3(256), 0, st, x, cnt, dyn, qx);
  qcn::LinEpi ep{nullptr, nullptr, nullptr, wsum, 0, 0, 0.f, w_scale, per_channel, bias, dyn};
  if (k % 128 == 0) {
    dim3 grid((n + 63) / 64, (m + 31) / 32);
    hipLaunchKernelGGL(qcn::linear_u8s8_kernel<true>, grid, dim3(256), 0, st, qx, m, k, 0, w, n,
                       ep, nullptr, y);
  } else {
    const long total = (long)m * n;
    const int grid = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(qcn::linear_generic_kernel<true>, dim3(grid), dim3(256), 0, st, qx, m, k, 0,
                       w, n, ep, nullptr, y);
  }
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_linear_dynamic_f32(const float* x, int m, int k, const int8_t* w, int n,
                           const float* w_scale, int per_channel, const int32_t* wsum,
                           const float* bias, int reduce_range, float* y, void* workspace,
                           void* stream) {
  return linear_dynamic_impl(x, m, k, w, n, w_scale, per_channel, wsum, bias, reduce_range,
                             nullptr, y, workspace, stream);
}

int qcn_linear_dynamic_range_f32(const float* x, int m, int k, const int8_t* w, int n,
                                 const float* w_scale, int per_channel, const int32_t* wsum,
                                 const float* bias, int reduce_range, const float* minmax,
                                 float* y, void* workspace, void* stream) {
  if (!minmax) return QCN_ERR_ARG;
  return linear_dynamic_impl(x, m, k, w, n, w_scale, per_channel, wsum, bias, reduce_range,
                             minmax, y, workspace, stream);
}

int qcn_linear_f32(const float* x, int m, int k, const float* w, int n, const float* b,
                   int relu_in, float* y, void* stream) {
  if (!x || !w || !y || m <= 0 || k <= 0 || n <= 0) return QCN_ERR_ARG;
  hipLaunchKernelGGL(qcn::linear_f32_kernel, dim3((m + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     x, m, k, w, n, b, relu_in, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

}  // extern "C"
