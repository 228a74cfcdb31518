// Shared device helpers for the gfx950 int8 ConvNet kernels.
//
// Numerics follow FBGEMM's vector epilogue exactly (see oracle/qref.py for the
// CPU restatement and the torch-wheel disassembly it was read from):
//   t  = fmaf(u_k, v_k, fp32(acc))          (per-tensor: u=b, v=fp32(1/aws);
//                                            per-channel: u=fp32(b/aws), v=1)
//   ab = fp32(t * mult_k)
//   y  = clamp(rne(ab) + zp, relu ? zp : 0, 255)
// Every kernel is compiled with -ffp-contract=off so that no other
// multiply/add pair is fused behind our back.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v2f __attribute__((ext_vector_type(2)));

#define QCN_DEV __device__ __forceinline__

// Host-side, once per device: the dynamic-LDS limit of a kernel.  Launchers
// run on the caller's current device (the Python side enters the model's
// device first), so a flag per device id keeps a second GPU from launching
// with an attribute only set on the first.
constexpr int QCN_MAX_DEV = 64;
inline int qcn_current_device() {
  int d = 0;
  return (hipGetDevice(&d) == hipSuccess && d >= 0 && d < QCN_MAX_DEV) ? d : -1;
}
// Compute units of the current device (cached per device); 0 on error.
inline int qcn_cu_count() {
  static int ncu_dev[QCN_MAX_DEV] = {};
  const int d = qcn_current_device();
  if (d < 0) return 0;
  int& ncu = ncu_dev[d];
  if (!ncu && (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess ||
               ncu <= 0))
    ncu = 0;
  return ncu;
}
inline bool qcn_set_lds_once(const void* kernel, int lds_bytes, bool (&done)[QCN_MAX_DEV]) {
  const int d = qcn_current_device();
  if (d < 0) return false;
  if (!done[d]) {
    if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes) !=
        hipSuccess)
      return false;
    done[d] = true;
  }
  return true;
}

QCN_DEV int requant_one(int acc, float u, float v, float mult, int zp, int lo) {
  float a = (float)acc;                      // v_cvt_f32_i32: RNE, like cvtdq2ps
  float t = __builtin_fmaf(u, v, a);
  float ab = t * mult;
  ab = __builtin_rintf(ab);                  // v_rndne_f32: ties to even
  ab = fminf(fmaxf(ab, -65536.0f), 65536.0f);  // keep the int conversion defined
  int r = (int)ab + zp;
  r = r < lo ? lo : r;
  r = r > 255 ? 255 : r;
  return r;
}

// Per-layer QDQ second stage (reference CustomQuantizedConv2d chain,
// custom_quantization_model.py:41-45 + F.relu at :237-250): the u8 output q of
// this layer (scale s1, zero point z1) is dequantized, ReLU'd, and quantized
// with the NEXT layer's input qparams (inv = fp32(1/s2), z2), in the same fp32
// op order as aten dequantize / quantize_per_tensor (oracle qref A1/A7).
QCN_DEV int qdq_next(int q, float s1, int z1, float inv2, int z2) {
  float x = (float)(q - z1) * s1;
  x = x > 0.0f ? x : 0.0f;
  float t = x * inv2;
  t = fminf(t, 1.0e9f);
  t = __builtin_rintf(t);
  int r = (int)t + z2;
  r = r < 0 ? 0 : r;
  r = r > 255 ? 255 : r;
  return r;
}

// Float form of requant_one for the MFMA epilogues: returns the requantized
// value as an integral float in [lo, 255].  rint(ab) + zp is exact while
// |ab| < 2^24; beyond that the sum keeps its sign and the clamp saturates to
// the same bound, so no separate range clamp is needed.  7 VALU per element
// (cvt, fma, mul, rndne, add, med3 + the pack) instead of ~15.
QCN_DEV float requant_f(int acc, float u, float v, float mult, float zpf, float lof) {
  const float t = __builtin_fmaf(u, v, (float)acc);
  const float ab = t * mult;
  return __builtin_amdgcn_fmed3f(__builtin_rintf(ab) + zpf, lof, 255.0f);
}

// qdq_next on the float form (q integral in [0,255]): (q - z1) is exact in fp32.
QCN_DEV float qdq_next_f(float q, float s1, float z1f, float inv2, float z2f) {
  float x = (q - z1f) * s1;
  x = x > 0.0f ? x : 0.0f;
  const float t = fminf(x * inv2, 1.0e9f);
  return __builtin_amdgcn_fmed3f(__builtin_rintf(t) + z2f, 0.0f, 255.0f);
}

QCN_DEV uint32_t xor80(uint32_t v) { return v ^ 0x80808080u; }

// Write-through (sc1) global stores for activations the NEXT launch reads:
// the bytes go to memory as they are produced instead of sitting dirty in
// this XCD's L2 until the kernel boundary's release writes them back
// (MI355X_MICROARCH 'boundary': + bytes / 6 TB/s per dirty predecessor).
// `base` must be wave-uniform; byte offsets < 2^31.
typedef __amdgpu_buffer_rsrc_t wt_rsrc_t;
QCN_DEV wt_rsrc_t wt_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
QCN_DEV void store_wt16(wt_rsrc_t r, uint32_t off, uint4 v) {
  __builtin_amdgcn_raw_buffer_store_b128((v4i){(int)v.x, (int)v.y, (int)v.z, (int)v.w}, r, (int)off, 0,
                                         16);
}

QCN_DEV uint32_t splat_u8(int b) {
  uint32_t x = (uint32_t)(b & 0xff);
  return x | (x << 8) | (x << 16) | (x << 24);
}

// 16-B-per-lane LDS-DMA (global_load_lds_dwordx4) issued from inline asm.
// The compiler's wait-count model treats an in-flight builtin LDS-DMA as an
// LDS event of unknown order and then guards every later ds_read use with
// lgkmcnt(0), which serialises a software-pipelined MFMA loop.  Callers of
// this form track completion themselves with explicit s_waitcnt vmcnt.
// lds_dst: the wave's 1-KiB destination (lane i writes lds_dst + 16 i).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"   // m0 is ours for the two instructions
QCN_DEV void glds16(const void* gsrc, void* lds_dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds_dst);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :: "v"(gsrc), "s"(m0) : "memory", "m0");
}
#pragma clang diagnostic pop
