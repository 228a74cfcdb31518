// Conv epilogue parameters and the per-element requant forms shared by the
// 3x3 conv kernels (conv3x3.hip) and the one-wave-per-SIMD conv3..conv6
// launch (convs36.hip).  Numerics: FBGEMM's ReQuantizeOutput as restated in
// oracle/qref.py, see common.hpp.
#pragma once
#include "common.hpp"
#include "qconvnet_abi.hpp"
#include <utility>

namespace qcn {

struct ConvEpi {
  const float* u;      // [COUT]
  const float* v;      // [COUT]
  const float* mult;   // [COUT]
  const int* corr;     // [COUT] (128 - zp_x) * sum_k w[k]
  int zp_y, lo;        // output zero point, lower clamp (zp_y if relu else 0)
  int qdq;             // 0: write requantized u8; 1: apply qdq_next; 2: as 1, with the
                       // exact one-fma form below (qdq_affine, set on the host)
  float s1; int z1; float inv2; int z2;
  int kmajor;          // 1: write y as [f / 32][image][32] (f = NHWC flatten index)
  // qdq == 2: requant + QDQ hand-off of an accumulator with ab = (acc + u v) m is
  // cvt_pk(med3(fma(rint(ab), qa, qb), glo, ghi)) — zp_y, lo, the dequantize,
  // ReLU and the next stub's quantize folded into one fma and one med3
  float qa, qb, glo, ghi;
};

// the QDQ hand-off after the requant, in the one-fma form (qdq == 2)
QCN_DEV float qdq_aff_f(float ab, const ConvEpi& ep) {
  return __builtin_amdgcn_fmed3f(__builtin_fmaf(__builtin_rintf(ab), ep.qa, ep.qb), ep.glo, ep.ghi);
}

__host__ __device__ inline bool epi_fast(const ConvEpi& ep) { return ep.zp_y == 0 && ep.lo == 0 && ep.qdq == 0; }
inline int epi_mode(const ConvEpi& ep) { return ep.qdq == 2 ? 2 : (epi_fast(ep) ? 1 : 0); }

// The QDQ hand-off of qcn_qdq_t q into ep (ep.zp_y / ep.lo already set):
// qdq = 2 with the one-fma constants when an exact form exists, else 1
// (host; conv3x3.hip).
void set_qdq(ConvEpi& ep, const qcn_qdq_t* q);

// Epilogue constants of 4 consecutive output channels from an LDS copy
// (u | v | mult, cout floats each).
struct EpiG {
  float4 u, v, m;
};
QCN_DEV EpiG load_epig(const float* ek, int cout, int co) {
  return {*reinterpret_cast<const float4*>(ek + co), *reinterpret_cast<const float4*>(ek + cout + co),
          *reinterpret_cast<const float4*>(ek + 2 * cout + co)};
}
QCN_DEV float f4e(const float4& f, int e) { return e == 0 ? f.x : (e == 1 ? f.y : (e == 2 ? f.z : f.w)); }

// Compile-time loop: f(std::integral_constant<int, i>) for i = 0 .. N-1 (a
// guaranteed unroll, so every register-array index below is a constant).
template <class F, int... I>
QCN_DEV void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
QCN_DEV void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// One requantized output into byte e of wd.  EM 1 — FAST: zp_y == 0, lo == 0
// and no QDQ hand-off (every post-ReLU layer of the static net): then
// clamp(rne(ab) + zp, lo, 255) == v_cvt_pk_u8_f32(ab), which rounds half to
// even and saturates to [0, 255] (probed exhaustively on gfx950,
// tools/micro/cvt_probe.hip).  EM 2: the QDQ hand-off in its one-fma form.
// EM 0: the general requant (+ qdq_next_f).
template <int EM>
QCN_DEV uint32_t rq_elem(int a, const EpiG& K, int e, const ConvEpi& ep, uint32_t wd) {
  const float u = f4e(K.u, e), v = f4e(K.v, e), m = f4e(K.m, e);
  if constexpr (EM != 0) {
    float f = __builtin_fmaf(u, v, (float)a);
    f = f * m;
    if constexpr (EM == 2) f = qdq_aff_f(f, ep);
    return __builtin_amdgcn_cvt_pk_u8_f32(f, e, wd);
  } else {
    float q = requant_f(a, u, v, m, (float)ep.zp_y, (float)ep.lo);
    if (ep.qdq) q = qdq_next_f(q, ep.s1, (float)ep.z1, ep.inv2, (float)ep.z2);
    return __builtin_amdgcn_cvt_pk_u8_f32(q, e, wd);
  }
}

// LDS writes of this wave complete, then the workgroup barrier (global stores
// stay in flight: no vmcnt drain, unlike __syncthreads).
QCN_DEV void lds_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

}  // namespace qcn
