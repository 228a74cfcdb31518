// Classifier head of the static int8 SimpleConvNet (baseline_model.py:38-40,
// QuantizedLinearReLU fc1 -> QuantizedLinear fc2 -> DeQuantStub), in two
// launches instead of two full GEMM kernels:
//
//  1. fc_splitk_kernel: fc1's u8 x s8 GEMM (M = batch, K = 4096, N = 512) split
//     four ways along K.  From 1024 rows up a workgroup owns a 128 (rows) x 64
//     (features) tile of one K quarter and its four waves each compute 64 x 32
//     (fc_splitk_kernel<64>); below 1024 rows workgroups own 64 x 64 tiles and
//     each wave 32 x 32 (fc_splitk_kernel<32>: twice the workgroups, so a
//     small batch still fills the CUs).  Both on v_mfma_i32_32x32x32_i8
//     straight from global memory.  Both operands are
//     chunk-major ([K/32][rows][32]: conv6 writes its output that way, the
//     weights are packed so at upload), so every fragment load is one
//     contiguous 1 KB — row-major operands (4 KB row stride) ran 2-3x slower.
//     Each XCD takes one K quarter and half of the output tiles, so its L2
//     holds a quarter of W and half of X's quarter.  int32 partial sums go to a
//     workspace (4 x M x 512 x 4 B = 8 MB at batch 1024).
//  2. fc_finish_kernel: one wave per row sums the partials, adds the
//     zero-point correction, requantizes fc1 (+ReLU), writes the u8 fc1 row,
//     then computes fc2 (512 -> n2 <= 16) from the row it holds in registers
//     (exact integer dot products, wave reduction), requantizes and
//     dequantizes the logits.  Numerics are those of linear_u8s8_kernel (A9).
#include "common.hpp"
#include "qconvnet_abi.hpp"

namespace qcn {

constexpr int FC_S = 4;      // K split
constexpr int FC_N1 = 512;   // fc1 features handled by the finisher (64 lanes x 8)
constexpr int FC_N2 = 16;    // max fc2 outputs
// workspace: the split-K partials, [FC_S][m][n1] int32

// X' [K/32][m][32], W' [K/32][n][32] (chunk-major: a 32-row MFMA fragment of
// one 32-byte K chunk is one contiguous 1 KB, every wave-load fully coalesced).
// RW: rows per wave — 64 (two MFMA row blocks, 128-row workgroups) or 32
// (one block, 64-row workgroups: twice the workgroups at the same partial
// traffic, for batches too small to fill the CUs with 128-row tiles).
// fc1's split-K partial tile of workgroup blockIdx.x; returns its (row
// block, feature block, K quarter)
template <int RW>
QCN_DEV void fc_splitk_tile(const uint8_t* __restrict__ x, int m, int k, const int8_t* __restrict__ w, int n,
                            int* __restrict__ part) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int MB = m / (2 * RW), NB = n / 64, T = MB * NB * FC_S;
  int mb, nb, s;
  if (T % 8 == 0 && (MB * NB) % 2 == 0) {
    // K-quarter-major over the XCDs (workgroup b runs on XCD b % 8): XCD x
    // takes K quarter x % 4 and half (x / 4) of the (row block, feature
    // block) tiles, so it fetches a quarter of W and half of X's K quarter:
    // 1 MB per XCD at batch 1024 instead of 2.5 MB with row-block-major
    // order (FETCH_SIZE 20.6 -> 8.3 MB, 9.27 -> 8.87 us)
    const int x = blockIdx.x % 8, l = blockIdx.x / 8;
    s = x % FC_S;
    const int v = (x / FC_S) * (MB * NB / 2) + l;
    mb = v / NB;
    nb = v % NB;
  } else {
    int t = blockIdx.x;
    if (T % 8 == 0) t = (t % 8) * (T / 8) + t / 8;   // row-block-major per XCD
    mb = t / (NB * FC_S);
    const int rem = t % (NB * FC_S);
    nb = rem / FC_S;
    s = rem % FC_S;
  }
  const int mi = wave & 1, ni = wave >> 1;
  const int row0 = mb * 2 * RW + mi * RW, col0 = nb * 64 + ni * 32;
  const int kcs = (k / 32) / FC_S, kc0 = s * kcs;
  // fragment lane (l32, hi): row l32, bytes [16 hi, 16 hi + 16) of the chunk
  const int frag = (lane & 31) * 32 + (lane >> 5) * 16;
  const uint8_t* xa = x + ((long)kc0 * m + row0) * 32 + frag;
  const int8_t* wa = w + ((long)kc0 * n + col0) * 32 + frag;
  const long xs = (long)m * 32, ws = (long)n * 32;   // bytes per K chunk

  v16i acc0 = (v16i){0}, acc1 = (v16i){0};
  constexpr int U = 4;   // K chunks per load batch of the split-K loop; two batches in flight
  v4i fw[2][U];
  uint4 f0[2][U], f1[2][U];
  auto load = [&](int buf, int c) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      fw[buf][u] = *reinterpret_cast<const v4i*>(wa + (c + u) * ws);
      f0[buf][u] = *reinterpret_cast<const uint4*>(xa + (c + u) * xs);
      if constexpr (RW == 64) f1[buf][u] = *reinterpret_cast<const uint4*>(xa + (c + u) * xs + 1024);
    }
  };
  auto mm = [&](int buf) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint4 a = f0[buf][u];
      const v4i b0 = (v4i){(int)xor80(a.x), (int)xor80(a.y), (int)xor80(a.z), (int)xor80(a.w)};
      acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fw[buf][u], b0, acc0, 0, 0, 0);
      if constexpr (RW == 64) {
        const uint4 b = f1[buf][u];
        const v4i b1 = (v4i){(int)xor80(b.x), (int)xor80(b.y), (int)xor80(b.z), (int)xor80(b.w)};
        acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fw[buf][u], b1, acc1, 0, 0, 0);
      }
    }
  };
  load(0, 0);
  for (int c = 0; c < kcs; c += 2 * U) {
    if (c + U < kcs) load(1, c + U);
    mm(0);
    if (c + 2 * U < kcs) load(0, c + 2 * U);
    if (c + U < kcs) mm(1);
  }
  // D[feature][row]: lane (l32 = row, hi) holds features 8g + 4hi + e
  const int l32 = lane & 31, hi = lane >> 5;
  // plain stores: write-through partials measured slower (split-K 15.3 -> 16.1 us
  // with the finisher, profiles/r02_diag_write_through_ab.txt)
  int* pp = part + (long)s * m * n + col0 + 4 * hi;
  const int r = row0 + l32;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    *reinterpret_cast<int4*>(pp + (long)r * n + 8 * g) =
        make_int4(acc0[4 * g], acc0[4 * g + 1], acc0[4 * g + 2], acc0[4 * g + 3]);
    if constexpr (RW == 64)
      *reinterpret_cast<int4*>(pp + (long)(r + 32) * n + 8 * g) =
          make_int4(acc1[4 * g], acc1[4 * g + 1], acc1[4 * g + 2], acc1[4 * g + 3]);
  }
}

template <int RW>
__global__ __launch_bounds__(256) void fc_splitk_kernel(const uint8_t* __restrict__ x, int m, int k,
                                                        const int8_t* __restrict__ w, int n,
                                                        int* __restrict__ part) {
  fc_splitk_tile<RW>(x, m, k, w, n, part);
}

// 64-row tiles below 1024 rows (batch 256: 128 workgroups instead of 64)
inline void launch_fc_splitk(const uint8_t* x, int m, int k, const int8_t* w1, int n1, int* part,
                             hipStream_t st) {
  if (m < 1024) {
    const int tiles = (m / 64) * (n1 / 64) * FC_S;
    hipLaunchKernelGGL(fc_splitk_kernel<32>, dim3(tiles), dim3(256), 0, st, x, m, k, w1, n1, part);
  } else {
    const int tiles = (m / 128) * (n1 / 64) * FC_S;
    hipLaunchKernelGGL(fc_splitk_kernel<64>, dim3(tiles), dim3(256), 0, st, x, m, k, w1, n1, part);
  }
}

struct FcHead {
  const float *u1, *v1, *m1;
  const int* corr1;     // (128 - zx1) * wsum1 (the GEMM saw q ^ 0x80)
  int z1, lo1;          // fc1 output zero point = fc2 input zero point
  const int8_t* w2;
  int n2;
  const float *u2, *v2, *m2;
  int z2, lo2;
  float y2_scale;
};

__global__ __launch_bounds__(256) void fc_finish_kernel(const int* __restrict__ part, int m,
                                                        FcHead hd, uint8_t* __restrict__ y1,
                                                        uint8_t* __restrict__ y2,
                                                        float* __restrict__ y2f) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + wave;
  if (row >= m) return;
  const int f0 = lane * 8;
  // every load up front (one wave per row: nothing else hides their latency)
  int4 pv[FC_S][2];
#pragma unroll
  for (int s = 0; s < FC_S; ++s) {
    const int* p = part + ((long)s * m + row) * FC_N1 + f0;
    pv[s][0] = *reinterpret_cast<const int4*>(p);
    pv[s][1] = *reinterpret_cast<const int4*>(p + 4);
  }
  const int4 c0 = *reinterpret_cast<const int4*>(hd.corr1 + f0), c1 = *reinterpret_cast<const int4*>(hd.corr1 + f0 + 4);
  const float4 u0 = *reinterpret_cast<const float4*>(hd.u1 + f0), u4 = *reinterpret_cast<const float4*>(hd.u1 + f0 + 4);
  const float4 v0 = *reinterpret_cast<const float4*>(hd.v1 + f0), v4 = *reinterpret_cast<const float4*>(hd.v1 + f0 + 4);
  const float4 m0 = *reinterpret_cast<const float4*>(hd.m1 + f0), m4 = *reinterpret_cast<const float4*>(hd.m1 + f0 + 4);
  uint2 wv[FC_N2];
#pragma unroll
  for (int o = 0; o < FC_N2; ++o)
    wv[o] = *reinterpret_cast<const uint2*>(hd.w2 + (long)(o < hd.n2 ? o : 0) * FC_N1 + f0);

  int a[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
  for (int s = 0; s < FC_S; ++s) {
    a[0] += pv[s][0].x; a[1] += pv[s][0].y; a[2] += pv[s][0].z; a[3] += pv[s][0].w;
    a[4] += pv[s][1].x; a[5] += pv[s][1].y; a[6] += pv[s][1].z; a[7] += pv[s][1].w;
  }
  const float uu[8] = {u0.x, u0.y, u0.z, u0.w, u4.x, u4.y, u4.z, u4.w};
  const float vv[8] = {v0.x, v0.y, v0.z, v0.w, v4.x, v4.y, v4.z, v4.w};
  const float mm[8] = {m0.x, m0.y, m0.z, m0.w, m4.x, m4.y, m4.z, m4.w};
  int q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) q[e] = requant_one(a[e], uu[e], vv[e], mm[e], hd.z1, hd.lo1);
  const uint32_t lo = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
  const uint32_t hw = (uint32_t)q[4] | ((uint32_t)q[5] << 8) | ((uint32_t)q[6] << 16) | ((uint32_t)q[7] << 24);
  *reinterpret_cast<uint2*>(y1 + (long)row * FC_N1 + f0) = make_uint2(lo, hw);

  // fc2: exact sum_k (q1 - z1) * w2[o][k] over this lane's 8 k, for all
  // outputs at once: (q1 - z1) w = s8(q1 ^ 0x80) w + (128 - z1) w, so two
  // v_dot4_i32_i8 on the xor'd fc1 bytes plus (128 - z1) * sum(w) (two more
  // dot4 against 0x01010101) — no 32-bit multiplies
  const int ql = (int)(lo ^ 0x80808080u), qh = (int)(hw ^ 0x80808080u);
  const int zc = 128 - hd.z1;
  int sacc[FC_N2];
#pragma unroll
  for (int o = 0; o < FC_N2; ++o) {
    const int wx = (int)wv[o].x, wy = (int)wv[o].y;
    const int ws = __builtin_amdgcn_sdot4(wx, 0x01010101, __builtin_amdgcn_sdot4(wy, 0x01010101, 0, false), false);
    sacc[o] = __builtin_amdgcn_sdot4(ql, wx, __builtin_amdgcn_sdot4(qh, wy, zc * ws, false), false);
  }
  // wave sums by DPP (quad xor 1 / 2, half-row and row mirrors, row
  // broadcasts 15 / 31): the total lands in lane 63; 16 independent chains
  // interleave (ds_bpermute-based shuffles cost an LDS round trip each)
#pragma unroll
  for (int o = 0; o < FC_N2; ++o) sacc[o] += __builtin_amdgcn_update_dpp(0, sacc[o], 0xB1, 0xF, 0xF, false);
#pragma unroll
  for (int o = 0; o < FC_N2; ++o) sacc[o] += __builtin_amdgcn_update_dpp(0, sacc[o], 0x4E, 0xF, 0xF, false);
#pragma unroll
  for (int o = 0; o < FC_N2; ++o) sacc[o] += __builtin_amdgcn_update_dpp(0, sacc[o], 0x141, 0xF, 0xF, false);
#pragma unroll
  for (int o = 0; o < FC_N2; ++o) sacc[o] += __builtin_amdgcn_update_dpp(0, sacc[o], 0x140, 0xF, 0xF, false);
#pragma unroll
  for (int o = 0; o < FC_N2; ++o) sacc[o] += __builtin_amdgcn_update_dpp(0, sacc[o], 0x142, 0xA, 0xF, false);
#pragma unroll
  for (int o = 0; o < FC_N2; ++o) sacc[o] += __builtin_amdgcn_update_dpp(0, sacc[o], 0x143, 0xC, 0xF, false);
  int mine = 0;
#pragma unroll
  for (int o = 0; o < FC_N2; ++o) {
    const int tot = __builtin_amdgcn_readlane(sacc[o], 63);
    if (lane == o) mine = tot;
  }
  if (lane < hd.n2) {
    const int o = lane;
    const int q2 = requant_one(mine, hd.u2[o], hd.v2[o], hd.m2[o], hd.z2, hd.lo2);
    y2[(long)row * hd.n2 + o] = (uint8_t)q2;
    y2f[(long)row * hd.n2 + o] = (float)(q2 - hd.z2) * hd.y2_scale;
  }
}

// Wave sum of v over the 64 lanes by DPP (quad xor 1 / 2, half-row and row
// mirrors, row broadcasts 15 / 31); the total lands in lane 63.
QCN_DEV float wave_sum_dpp(float v) {
#define QCN_DPP_ADD(CTL, RM) \
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTL, RM, 0xF, false))
  QCN_DPP_ADD(0xB1, 0xF);
  QCN_DPP_ADD(0x4E, 0xF);
  QCN_DPP_ADD(0x141, 0xF);
  QCN_DPP_ADD(0x140, 0xF);
  QCN_DPP_ADD(0x142, 0xA);
  QCN_DPP_ADD(0x143, 0xC);
#undef QCN_DPP_ADD
  return v;
}

// QDQ variant of the finisher (CustomQuantizedSimpleConvNet,
// custom_quantization_model.py:256-258): fc1's stub chain requantizes to its
// own output qparams (no ReLU in the int8 op), DeQuantStub ->
// fp32(s1) * (q1 - z1), F.relu in fp32, then fc2 stays an fp32 nn.Linear:
// y = x @ w2^T + b2.  Each lane holds 8 of the 512 fc1 features; fc2's dot
// products are lane-local fma chains summed over the wave (fp32, a different
// summation order from MKL's sgemm: the QDQ tests bound it).
struct FcHeadQdq {
  const float *u1, *v1, *m1;
  const int* corr1;
  int z1, lo1;
  float s1;
  const float* w2;   // [n2][512] fp32
  const float* b2;   // [n2] or nullptr
  int n2;
};

__global__ __launch_bounds__(256) void fc_finish_qdq_kernel(const int* __restrict__ part, int m,
                                                            FcHeadQdq hd, uint8_t* __restrict__ y1,
                                                            float* __restrict__ y2f) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + wave;
  if (row >= m) return;
  const int f0 = lane * 8;
  int4 pv[FC_S][2];
#pragma unroll
  for (int s = 0; s < FC_S; ++s) {
    const int* p = part + ((long)s * m + row) * FC_N1 + f0;
    pv[s][0] = *reinterpret_cast<const int4*>(p);
    pv[s][1] = *reinterpret_cast<const int4*>(p + 4);
  }
  const int4 c0 = *reinterpret_cast<const int4*>(hd.corr1 + f0), c1 = *reinterpret_cast<const int4*>(hd.corr1 + f0 + 4);
  const float4 u0 = *reinterpret_cast<const float4*>(hd.u1 + f0), u4 = *reinterpret_cast<const float4*>(hd.u1 + f0 + 4);
  const float4 v0 = *reinterpret_cast<const float4*>(hd.v1 + f0), v4 = *reinterpret_cast<const float4*>(hd.v1 + f0 + 4);
  const float4 m0 = *reinterpret_cast<const float4*>(hd.m1 + f0), m4 = *reinterpret_cast<const float4*>(hd.m1 + f0 + 4);
  int a[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
  for (int s = 0; s < FC_S; ++s) {
    a[0] += pv[s][0].x; a[1] += pv[s][0].y; a[2] += pv[s][0].z; a[3] += pv[s][0].w;
    a[4] += pv[s][1].x; a[5] += pv[s][1].y; a[6] += pv[s][1].z; a[7] += pv[s][1].w;
  }
  const float uu[8] = {u0.x, u0.y, u0.z, u0.w, u4.x, u4.y, u4.z, u4.w};
  const float vv[8] = {v0.x, v0.y, v0.z, v0.w, v4.x, v4.y, v4.z, v4.w};
  const float mm[8] = {m0.x, m0.y, m0.z, m0.w, m4.x, m4.y, m4.z, m4.w};
  int q[8];
  float xf[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    q[e] = requant_one(a[e], uu[e], vv[e], mm[e], hd.z1, hd.lo1);
    const float d = (float)(q[e] - hd.z1) * hd.s1;   // aten::dequantize
    xf[e] = d > 0.f ? d : 0.f;                       // F.relu
  }
  if (y1) {
    const uint32_t lo = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
    const uint32_t hw = (uint32_t)q[4] | ((uint32_t)q[5] << 8) | ((uint32_t)q[6] << 16) | ((uint32_t)q[7] << 24);
    *reinterpret_cast<uint2*>(y1 + (long)row * FC_N1 + f0) = make_uint2(lo, hw);
  }
  float acc[FC_N2];
#pragma unroll
  for (int o = 0; o < FC_N2; ++o) {
    acc[o] = 0.f;
    if (o < hd.n2) {
      const float4 wa = *reinterpret_cast<const float4*>(hd.w2 + (long)o * FC_N1 + f0);
      const float4 wb = *reinterpret_cast<const float4*>(hd.w2 + (long)o * FC_N1 + f0 + 4);
      float t = xf[0] * wa.x;
      t = __builtin_fmaf(xf[1], wa.y, t);
      t = __builtin_fmaf(xf[2], wa.z, t);
      t = __builtin_fmaf(xf[3], wa.w, t);
      t = __builtin_fmaf(xf[4], wb.x, t);
      t = __builtin_fmaf(xf[5], wb.y, t);
      t = __builtin_fmaf(xf[6], wb.z, t);
      t = __builtin_fmaf(xf[7], wb.w, t);
      acc[o] = t;
    }
  }
#pragma unroll
  for (int o = 0; o < FC_N2; ++o) acc[o] = wave_sum_dpp(acc[o]);
  float mine = 0.f;
#pragma unroll
  for (int o = 0; o < FC_N2; ++o) {
    const float tot = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, acc[o]), 63));
    if (lane == o) mine = tot;
  }
  if (lane < hd.n2) y2f[(long)row * hd.n2 + lane] = mine + (hd.b2 ? hd.b2[lane] : 0.f);
}

}  // namespace qcn

extern "C" {

int qcn_pack_fc_kmajor(const int8_t* w, int n, int k, int8_t* out) {
  if (!w || !out || n <= 0 || k <= 0 || k % 32 != 0) return QCN_ERR_ARG;
  for (int o = 0; o < n; ++o)
    for (int kk = 0; kk < k; ++kk)
      out[((long)(kk / 32) * n + o) * 32 + kk % 32] = w[(long)o * k + kk];
  return QCN_OK;
}

long long qcn_classifier_workspace_size(int m, int n1) {
  if (m <= 0 || n1 <= 0) return 0;
  return (long long)qcn::FC_S * m * n1 * 4;   // the split-K partials
}

int qcn_classifier_u8s8(const uint8_t* x, int m, int k, const int8_t* w1, int n1, const float* u1,
                        const float* v1, const float* mult1, const int32_t* corr1, int y1_zp,
                        int relu1, const int8_t* w2, int n2, const float* u2, const float* v2,
                        const float* mult2, int y2_zp, int relu2, float y2_scale, void* workspace,
                        uint8_t* y1, uint8_t* y2, float* y2f, void* stream) {
  if (!x || !w1 || !u1 || !v1 || !mult1 || !corr1 || !w2 || !u2 || !v2 || !mult2 || !workspace ||
      !y1 || !y2 || !y2f)
    return QCN_ERR_ARG;
  if (m <= 0 || k <= 0 || n1 <= 0 || n2 <= 0 || y1_zp < 0 || y1_zp > 255 || y2_zp < 0 || y2_zp > 255)
    return QCN_ERR_ARG;
  if (m % 128 != 0 || n1 != qcn::FC_N1 || k % (32 * qcn::FC_S * 8) != 0 ||
      n2 > qcn::FC_N2)
    return QCN_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  int* part = static_cast<int*>(workspace);
  qcn::FcHead hd{u1, v1, mult1, corr1, y1_zp, relu1 ? y1_zp : 0, w2, n2, u2, v2, mult2,
                 y2_zp, relu2 ? y2_zp : 0, y2_scale};
  qcn::launch_fc_splitk(x, m, k, w1, n1, part, st);
  hipLaunchKernelGGL(qcn::fc_finish_kernel, dim3((m + 3) / 4), dim3(256), 0, st, part, m, hd, y1,
                     y2, y2f);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

int qcn_classifier_qdq_u8s8(const uint8_t* x, int m, int k, const int8_t* w1, int n1,
                            const float* u1, const float* v1, const float* mult1,
                            const int32_t* corr1, int y1_zp, float y1_scale, const float* w2,
                            int n2, const float* b2, void* workspace, uint8_t* y1, float* y2,
                            void* stream) {
  if (!x || !w1 || !u1 || !v1 || !mult1 || !corr1 || !w2 || !workspace || !y2) return QCN_ERR_ARG;
  if (m <= 0 || k <= 0 || n1 <= 0 || n2 <= 0 || y1_zp < 0 || y1_zp > 255 || !(y1_scale > 0.f))
    return QCN_ERR_ARG;
  if (m % 128 != 0 || n1 != qcn::FC_N1 || k % (32 * qcn::FC_S * 8) != 0 ||
      n2 > qcn::FC_N2)
    return QCN_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  int* part = static_cast<int*>(workspace);
  qcn::FcHeadQdq hd{u1, v1, mult1, corr1, y1_zp, 0, y1_scale, w2, b2, n2};
  qcn::launch_fc_splitk(x, m, k, w1, n1, part, st);
  hipLaunchKernelGGL(qcn::fc_finish_qdq_kernel, dim3((m + 3) / 4), dim3(256), 0, st, part, m, hd,
                     y1, y2);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

}  // extern "C"
