// LDS-tiled implicit-GEMM int8 convolution for the ResNet bottleneck path
// (SURVEY §8(f)2), with the residual join fused into the epilogue.
//
// D[cout][pixel] = W'[cout][k] . X'[pixel][k] on v_mfma_i32_32x32x32_i8,
// K = (r, s, c) in 32-byte chunks.  Workgroup tile: 256 output pixels x BN
// output channels (BN = 128, or 64 for the 64-channel convs); 4 waves, each
// 128 x 64 (JT = 4 pixel tiles x 2 channel tiles) or 64 x 64.  K advances 64
// bytes (two chunks) per stage through a 3-deep LDS ring filled by LDS-DMA
// (global_load_lds_dwordx4).  Every 1-KiB piece of a stage is one fragment in
// MFMA operand order (lane L <-> row L%32, k half L/32), so the DMA source
// address carries the im2col gather (pixel row, tap, channel chunk) and the
// MFMA reads are lane-linear ds_read_b128 with no bank conflicts.  Out-of-image
// taps read a constant line of the input zero point (g_zp_lines), so padding
// costs nothing.  Activations are biased by 0x80 after the read (u8 -> s8).
//
// Epilogue: FBGEMM requant (A6) per output channel, and for the last 1x1 conv
// of a bottleneck optionally the residual join of
// custom_quantization_model.py:94-101 in registers: y3 = requant(acc) (u8,
// s3/z3), out = quantize(relu(s3*(y3-z3) + s_r*(r-z_r)), s_o, z_o) — the same
// fp32 ops as qcn_add_relu_u8 on the materialised y3, so bit-identical.
#include "common.hpp"
#include "qconvnet_abi.hpp"

#include <algorithm>
#include <cmath>
#include <type_traits>

namespace qcn {

// fp32(fp32(acc) + u*v) * mult for two channels (FBGEMM requant before the
// rounding) as one packed fma and one packed mul: in these epilogue-bound
// convs no MFMA stream competes with the packed issue (the SimpleConvNet ring
// kernels keep scalar fp32 beside their partner waves' MFMAs).
QCN_DEV v2f requant2(int a0, int a1, v2f u, v2f v, v2f m) {
  return __builtin_elementwise_fma(u, v, (v2f){(float)a0, (float)a1}) * m;
}

// floor(a / d) for 0 <= a < 2^22 and d >= 1 from an fp32 reciprocal estimate
// (off by at most one) and one correction each way.
QCN_DEV int div_small(int a, int d, float rd) {
  int q = (int)((float)a * rd);
  q -= (q * d > a) ? 1 : 0;
  q += ((q + 1) * d <= a) ? 1 : 0;
  return q;
}


struct ZpLines {
  uint8_t b[256][32];
};
constexpr ZpLines make_zp_lines() {
  ZpLines z{};
  for (int i = 0; i < 256; ++i)
    for (int j = 0; j < 32; ++j) z.b[i][j] = (uint8_t)i;
  return z;
}
// row z = 32 bytes of value z (row 0 doubles as the zero weight line)
__device__ const ZpLines g_zp_lines = make_zp_lines();

struct GemmArgs {
  const uint8_t* x;
  const int8_t* w;
  int n, h, w_, cin, oh, ow, cout, kh, kw, sy, sx, py, px, x_zp;
  long npix;
  int kcs;     // K chunks of 32
  int mt, nt;  // tiles along pixels / channels
  const float *u, *v, *mult;
  const int* corr;
  int zp_y, lo;
  // fused residual join (RESID): identity r (u8, s_r/z_r), y3 scale s3 (z3 = zp_y)
  const uint8_t* r;
  float s3, s_r, inv_o;
  int z_r, z_o;
  uint8_t* y;
  // streaming 1x1 kernel: 32-pixel strips, chunks of `per` strips, `cg`
  // channel groups of NW x 32 output channels
  int nstrip, nchunk, per, cg;
  // fused next-block reduce (CR > 0): 1x1 conv of the joined output y (its
  // input zero point z_o), k-major weights [K/32][CR][32], FBGEMM requant
  // (u2, v2, mult2, corr2, zp2, lo2) into y2 [pixel][CR]
  const int8_t* w2;
  const float *u2, *v2, *mult2;
  const int* corr2;
  int zp2, lo2;
  uint8_t* y2;
};

template <int BN, int BM_ = 256>
struct GemmCfg {
  // BM_ = 128 (thin convs, K <= 256): half the pixels per tile, 64 accumulators
  // per wave and a third of the LDS, so three workgroups share a CU
  static constexpr int BM = BM_;
  static constexpr int NW = BN == 256 ? 8 : 4;   // waves (BN = 256: 512 threads, one per CU)
  static constexpr int NT = 64 * NW;
  static constexpr int WN = BN / 64;          // waves along channels
  static constexpr int WM = NW / WN;          // waves along pixels
  static constexpr int JT = BM / (32 * WM);   // pixel tiles per wave (4 or 2)
  static constexpr int FA = 2 * BN / 32;      // A fragments (1 KiB) per stage
  static constexpr int AREG = FA * 1024;      // A region of a stage
  static constexpr int STAGE = AREG + BM * 64;
  static constexpr int DA = FA / NW;          // A DMA instructions per wave per stage
  static constexpr int NB = BM * 64 / 1024 / NW;   // B DMA instructions (16 rows x 64 B) per wave
  static constexpr int D = DA + NB;
  static constexpr int OS = BN + 16;          // output staging row stride (bytes)
  static constexpr int LDS = 3 * STAGE;
  static constexpr int MINW = BM == 128 ? 3 : 512 / NT;   // waves per SIMD the registers allow
  static_assert(FA % NW == 0, "A fragments split evenly over the waves");
  static_assert(BM * OS <= LDS, "output staging fits in the ring");
};

// one K chunk (32 channels of one tap) forward in (r, s, c) order
struct KCursor {
  int r, s, c;
  QCN_DEV void adv(int cin, int kw) {
    c += 32;
    if (c == cin) {
      c = 0;
      if (++s == kw) { s = 0; ++r; }
    }
  }
};

template <int BN, bool RESID, int BM = 256>
__global__ __launch_bounds__((GemmCfg<BN, BM>::NT), (GemmCfg<BN, BM>::MINW)) void conv_gemm_kernel(GemmArgs a) {
  using C = GemmCfg<BN, BM>;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, hi = lane >> 5;

  // XCD-aware tile order: consecutive tiles (same pixels, all channel tiles
  // first) stay on one XCD's L2.
  const int T = a.mt * a.nt;
  const int bid = blockIdx.x, xcd = bid & 7, k8 = bid >> 3;
  const int q = T >> 3, rm = T & 7;
  const int t = xcd < rm ? xcd * (q + 1) + k8 : rm * (q + 1) + (xcd - rm) * q + k8;
  const int mtile = t / a.nt, ntile = t % a.nt;
  const long m0 = (long)mtile * C::BM;
  const int n0 = ntile * BN;

  // B (pixel) rows: a stage holds BM rows x 64 B (two K chunks); row r's 16-B
  // piece pc sits at slot pc ^ ((r >> 2) & 3) (conflict-free MFMA reads).  DMA
  // instruction ib covers rows 16 ib .. 16 ib + 15, lane L -> row L/4, slot L%4,
  // so every lane loads the same piece (chunk c, half h) of its 4 rows.
  const int bslot = lane & 3, bswz = (lane >> 4) & 3, bpc = bslot ^ bswz;
  const int bc = bpc >> 1, bh = bpc & 1;
  long pbase[C::NB];
  int iy0[C::NB], ix0[C::NB];
  bool pv[C::NB];
  // pixel -> (image, oy, ox): the tile's first pixel is split once (uniform;
  // npix < 2^31 is checked at launch), each lane's offset (< 256) is carried
  // through ox and oy with small fp32-reciprocal divisions — no 64-bit
  // divisions per lane (they were ~half the VALU of the thin 1x1 convs)
  // A 1x1 stride-1 unpadded conv reads input pixel = output pixel: no
  // decomposition and no bounds checks (uniform branch).
  const bool flat = a.kh == 1 && a.kw == 1 && a.sy == 1 && a.sx == 1 && a.py == 0 && a.px == 0;
  const int ohw = a.oh * a.ow;
  const int m0i = (int)m0;
  const int img0 = m0i / ohw, rem0 = m0i - img0 * ohw;
  const int oy00 = rem0 / a.ow, ox00 = rem0 - oy00 * a.ow;
  const float rw = 1.0f / (float)a.ow, rh = 1.0f / (float)a.oh;
#pragma unroll
  for (int e = 0; e < C::NB; ++e) {
    const int off = (wave + C::NW * e) * 16 + (lane >> 2);
    pv[e] = m0 + off < a.npix;
    if (flat) {
      iy0[e] = ix0[e] = 0;
      pbase[e] = (m0 + off) * (long)a.cin + bh * 16;
      continue;
    }
    const int tx = ox00 + off;
    const int qx = div_small(tx, a.ow, rw);
    const int ty = oy00 + qx;
    const int qy = div_small(ty, a.oh, rh);
    const int ox = tx - qx * a.ow, oy = ty - qy * a.oh;
    const long img = pv[e] ? img0 + qy : 0;
    iy0[e] = oy * a.sy - a.py;
    ix0[e] = ox * a.sx - a.px;
    pbase[e] = ((img * a.h + iy0[e]) * a.w_ + ix0[e]) * (long)a.cin + bh * 16;
  }
  const uint8_t* zpl = &g_zp_lines.b[a.x_zp][bh * 16];
  const uint8_t* zero = &g_zp_lines.b[0][hi * 16];
  const int8_t* wl = a.w + ((long)n0 + l32) * 32 + hi * 16;
  const long wstep = (long)a.cout * 32;

  // uniform cursors of the even and odd chunk of the next stage to load
  KCursor cur0{0, 0, 0}, cur1{0, 0, 0};
  cur1.adv(a.cin, a.kw);
  const int nst = (a.kcs + 1) / 2;
  auto issue = [&](int st) {
    uint8_t* buf = lds + (st % 3) * C::STAGE;
#pragma unroll
    for (int tt = 0; tt < C::DA; ++tt) {   // A: fragment f = wave + NW tt
      const int f = wave + C::NW * tt, c = f / (BN / 32), g = f % (BN / 32);
      const int kc = 2 * st + c;
      const void* src = kc < a.kcs ? (const void*)(wl + kc * wstep + g * 32 * 32) : (const void*)zero;
      glds16(src, buf + f * 1024);
    }
    const int lr = bc ? cur1.r : cur0.r, ls = bc ? cur1.s : cur0.s, lc = bc ? cur1.c : cur0.c;
    const bool live = 2 * st + bc < a.kcs;
    const long toff = ((long)lr * a.w_ + ls) * a.cin + lc;
#pragma unroll
    for (int e = 0; e < C::NB; ++e) {      // B: instruction wave + NW e
      const int iy = iy0[e] + lr, ix = ix0[e] + ls;
      const bool in = live && pv[e] && (flat || (iy >= 0 && iy < a.h && ix >= 0 && ix < a.w_));
      const void* src = in ? (const void*)(a.x + pbase[e] + toff) : (const void*)zpl;
      glds16(src, buf + C::AREG + (wave + C::NW * e) * 1024);
    }
    cur0.adv(a.cin, a.kw); cur0.adv(a.cin, a.kw);
    cur1.adv(a.cin, a.kw); cur1.adv(a.cin, a.kw);
  };

  const int wc = wave % C::WN, wm = wave / C::WN;
  // accumulators: the first half-stage's MFMAs take the zero-point
  // correction cinit[i] as their C operand (no copies into 2 x JT tiles:
  // those v_movs were ~10 % of a K = 64 conv's VALU)
  v16i acc[2][C::JT];
  v16i cinit[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int4 c4 = *reinterpret_cast<const int4*>(a.corr + n0 + wc * 64 + i * 32 + 8 * g + 4 * hi);
      cinit[i][4 * g] = c4.x; cinit[i][4 * g + 1] = c4.y; cinit[i][4 * g + 2] = c4.z; cinit[i][4 * g + 3] = c4.w;
    }
  }
  // Residual join (RESID): the identity bytes each thread's join rows need
  // (thread (rr, cq): 16 channels of rows rr + R_RPI it, see the epilogue).
  // With at most two stages (conv3 with K <= 128) they are loaded right
  // behind the stage DMAs, so their HBM latency overlaps the DMA wait and the
  // MFMAs instead of following them; longer K loads them before the join.
  // Rows past npix load the last pixel's bytes (unused) so every wave issues
  // the same count.
  constexpr int R_TPR = BN / 16, R_RPI = C::NT / R_TPR, NIT = C::BM / R_RPI;
  constexpr int NIDL = NIT;                    // identity loads per thread
  const int rr = tid / R_TPR, cq = tid % R_TPR;
  const int ch2 = n0 + cq * 16;
  uint4 rid[NIT];
  auto load_id = [&]() {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      long pp = m0 + it * R_RPI + rr;
      pp = pp < a.npix ? pp : a.npix - 1;
      rid[it] = *reinterpret_cast<const uint4*>(a.r + pp * a.cout + ch2);
    }
  };
  const bool early = RESID && nst <= 2;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  issue(0);
  if (nst > 1) issue(1);
  if constexpr (RESID) {
    if (early) load_id();
  }

  // MFMA read offsets: A lane-linear; B row (wm*JT + j)*32 + l32, piece 2c+hi
  const int swz = (l32 >> 2) & 3;
  const int boff0 = C::AREG + (wm * C::JT) * 2048 + l32 * 64 + ((hi ^ swz) << 4);
  const int boff1 = C::AREG + (wm * C::JT) * 2048 + l32 * 64 + (((2 + hi) ^ swz) << 4);
  auto rd_a = [&](int st, int c, int i) {
    return *reinterpret_cast<const v4i*>(lds + (st % 3) * C::STAGE + (c * (BN / 32) + wc * 2 + i) * 1024 +
                                         lane * 16);
  };
  auto rd_b = [&](int st, int c, int j) {
    return *reinterpret_cast<const v4i*>(lds + (st % 3) * C::STAGE + (c ? boff1 : boff0) + j * 2048);
  };
  // Software pipeline over half-stages (one 32-byte K chunk each): the
  // fragments of the next half-stage are read one per MFMA of this one.  The
  // ring's one barrier per stage sits between its two halves: it certifies
  // stage st+1 landed (its reads start in the second half) and that every
  // wave is done with stage st-1, whose buffer stage st+2's DMA then reuses.
  auto seg = [&](auto first, const v4i (&fa)[2], v4i (&fb)[C::JT], v4i (&na)[2], v4i (&nb)[C::JT],
                 int rst, int rc, bool rd) {
#pragma unroll
    for (int j = 0; j < C::JT; ++j)
#pragma unroll
      for (int d = 0; d < 4; ++d) fb[j][d] ^= (int)0x80808080u;   // u8 -> s8 (q - 128)
#pragma unroll
    for (int m = 0; m < 2 * C::JT; ++m) {
      if (rd) {
        if (m < 2) na[m] = rd_a(rst, rc, m);
        else if (m < 2 + C::JT) nb[m - 2] = rd_b(rst, rc, m - 2);
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (decltype(first)::value)
        acc[m / C::JT][m % C::JT] =
            __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[m / C::JT], fb[m % C::JT], cinit[m / C::JT], 0, 0, 0);
      else
        acc[m / C::JT][m % C::JT] =
            __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[m / C::JT], fb[m % C::JT], acc[m / C::JT][m % C::JT], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  v4i fa0[2], fb0[C::JT], fa1[2], fb1[C::JT];
  // (early identity loads are the youngest NIDL vector-memory operations)
  if (early) {
    if (nst > 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(C::D + NIDL) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NIDL) : "memory");
  } else {
    if (nst > 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(C::D) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 2; ++i) fa0[i] = rd_a(0, 0, i);
#pragma unroll
  for (int j = 0; j < C::JT; ++j) fb0[j] = rd_b(0, 0, j);
  // stage st: first half multiplies (st, 0) and reads (st, 1); the stage
  // barrier; second half multiplies (st, 1) and reads (st+1, 0).  Stage 0's
  // first half is peeled (its MFMAs start from cinit).
  auto mid = [&](int st) {
    __builtin_amdgcn_sched_barrier(0);
    const bool more = st + 1 < nst;
    if (more) {
      // stage st+1 (the only DMA in flight; behind it only early identity loads)
      if (early) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NIDL) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (st + 2 < nst) issue(st + 2);
      __builtin_amdgcn_sched_barrier(0);
    }
    seg(std::false_type{}, fa1, fb1, fa0, fb0, st + 1, 0, more);
  };
  seg(std::true_type{}, fa0, fb0, fa1, fb1, 0, 1, true);
  mid(0);
  for (int st = 1; st < nst; ++st) {
    seg(std::false_type{}, fa0, fb0, fa1, fb1, st, 1, true);
    mid(st);
  }
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();   // every wave is done with the ring: reuse it
  __builtin_amdgcn_sched_barrier(0);


  // Epilogue phase 1 (accumulator layout: lane (l32, hi) of tile (i, j) holds
  // pixel l32, channels 8g + 4hi + e): FBGEMM requant to u8 — scalar fma / mul
  // (requant2), v_cvt_pk_u8_f32 (RNE + saturate) standing in for
  // rint/+zp/clamp when zp == 0 — and dword writes into the LDS tile
  // [BM][OS] (no lane transposes).
  const bool fast = a.zp_y == 0;
  const float zpf = (float)a.zp_y, lof = (float)a.lo;
  const v2f zpv = {zpf, zpf};
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int cl = wc * 64 + i * 32;   // tile's first channel within the workgroup
    v2f u[8], v[8], mu[8];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int co = n0 + cl + 8 * g + 4 * hi;
      const float4 x4 = *reinterpret_cast<const float4*>(a.u + co);
      const float4 y4 = *reinterpret_cast<const float4*>(a.v + co);
      const float4 z4 = *reinterpret_cast<const float4*>(a.mult + co);
      u[2 * g] = (v2f){x4.x, x4.y}; u[2 * g + 1] = (v2f){x4.z, x4.w};
      v[2 * g] = (v2f){y4.x, y4.y}; v[2 * g + 1] = (v2f){y4.z, y4.w};
      mu[2 * g] = (v2f){z4.x, z4.y}; mu[2 * g + 1] = (v2f){z4.z, z4.w};
    }
#pragma unroll
    for (int j = 0; j < C::JT; ++j) {
      v2f ab[8];
#pragma unroll
      for (int h2 = 0; h2 < 8; ++h2) {
        ab[h2] = requant2(acc[i][j][2 * h2], acc[i][j][2 * h2 + 1], u[h2], v[h2], mu[h2]);
      }
      uint32_t* od = reinterpret_cast<uint32_t*>(lds + ((wm * C::JT + j) * 32 + l32) * C::OS + cl) + hi;
      if (fast) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          uint32_t wd = __builtin_amdgcn_cvt_pk_u8_f32(ab[2 * g].x, 0, 0u);
          wd = __builtin_amdgcn_cvt_pk_u8_f32(ab[2 * g].y, 1, wd);
          wd = __builtin_amdgcn_cvt_pk_u8_f32(ab[2 * g + 1].x, 2, wd);
          od[2 * g] = __builtin_amdgcn_cvt_pk_u8_f32(ab[2 * g + 1].y, 3, wd);
        }
      } else if (a.lo == 0) {
        // clamp(rint + zp, 0, 255): v_cvt_pk_u8_f32 saturates to [0, 255] and
        // rint + zp is integer-valued, so no med3
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const v2f r0 = (v2f){__builtin_rintf(ab[2 * g].x), __builtin_rintf(ab[2 * g].y)} + zpv;
          const v2f r1 = (v2f){__builtin_rintf(ab[2 * g + 1].x), __builtin_rintf(ab[2 * g + 1].y)} + zpv;
          uint32_t wd = __builtin_amdgcn_cvt_pk_u8_f32(r0.x, 0, 0u);
          wd = __builtin_amdgcn_cvt_pk_u8_f32(r0.y, 1, wd);
          wd = __builtin_amdgcn_cvt_pk_u8_f32(r1.x, 2, wd);
          od[2 * g] = __builtin_amdgcn_cvt_pk_u8_f32(r1.y, 3, wd);
        }
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          uint32_t wd = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x = e & 1 ? ab[2 * g + (e >> 1)].y : ab[2 * g + (e >> 1)].x;
            wd = __builtin_amdgcn_cvt_pk_u8_f32(
                __builtin_amdgcn_fmed3f(__builtin_rintf(x) + zpf, lof, 255.0f), e, wd);
          }
          od[2 * g] = wd;
        }
      }
    }
  }
  __syncthreads();

  if constexpr (RESID) {
    // Residual join on the staged u8 conv3 output y3 (phase 1 above, zp z3, no
    // ReLU): out = quantize(relu(s3*(y3 - z3) + s_r*(r - z_r))) with the
    // identity r loaded earlier (rid) — (float)y3 - z3 is exact, so this is
    // the same fp32 op sequence as qcn_add_relu_u8 on the materialised y3.
    // Row-contiguous: thread (rr, cq) takes 16 channels of rows rr + R_RPI it.
    if (!early) load_id();
    const v2f z3v = {(float)a.zp_y, (float)a.zp_y}, s3v = {a.s3, a.s3};
    const v2f zr = {(float)a.z_r, (float)a.z_r}, sr = {a.s_r, a.s_r}, io = {a.inv_o, a.inv_o};
    const float zof = (float)a.z_o;
    auto join = [&](auto zo0) {
      constexpr bool ZO0 = decltype(zo0)::value;   // z_o == 0: ReLU = saturation at 0
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int row = it * R_RPI + rr;
        const long px = m0 + row;
        if (px >= a.npix) break;
        const uint4 yv = *reinterpret_cast<const uint4*>(lds + row * C::OS + cq * 16);
        const uint4 rv = rid[it];
        const uint32_t yw[4] = {yv.x, yv.y, yv.z, yv.w}, rw[4] = {rv.x, rv.y, rv.z, rv.w};
        uint32_t ow[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          uint32_t o = 0;
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const v2f yf = {(float)((yw[g] >> (8 * e)) & 0xff), (float)((yw[g] >> (8 * e + 8)) & 0xff)};
            const v2f rf = {(float)((rw[g] >> (8 * e)) & 0xff), (float)((rw[g] >> (8 * e + 8)) & 0xff)};
            const v2f sm = ((yf - z3v) * s3v + (rf - zr) * sr) * io;
            if constexpr (ZO0) {
              o = __builtin_amdgcn_cvt_pk_u8_f32(sm.x, e, o);
              o = __builtin_amdgcn_cvt_pk_u8_f32(sm.y, e + 1, o);
            } else {   // relu(s) * inv == max(s * inv, 0) since inv > 0
              o = __builtin_amdgcn_cvt_pk_u8_f32(
                  __builtin_amdgcn_fmed3f(__builtin_rintf(__builtin_fmaxf(sm.x, 0.0f)) + zof, 0.0f, 255.0f),
                  e, o);
              o = __builtin_amdgcn_cvt_pk_u8_f32(
                  __builtin_amdgcn_fmed3f(__builtin_rintf(__builtin_fmaxf(sm.y, 0.0f)) + zof, 0.0f, 255.0f),
                  e + 1, o);
            }
          }
          ow[g] = o;
        }
        *reinterpret_cast<uint4*>(a.y + px * a.cout + ch2) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
      }
    };
    if (a.z_o == 0) join(std::true_type{});
    else join(std::false_type{});
    return;
  }

  // Epilogue phase 2 (row-contiguous): 16 B per thread, whole 64/128-B row
  // segments per store instruction.
  constexpr int TPR = BN / 16;            // threads per row
  constexpr int RPI = C::NT / TPR;        // rows per iteration
  const int orr = tid / TPR, cc = (tid % TPR) * 16;
#pragma unroll 2
  for (int r0 = 0; r0 < C::BM; r0 += RPI) {
    const int row = r0 + orr;
    const long p = m0 + row;
    if (p >= a.npix) break;
    *reinterpret_cast<uint4*>(a.y + p * a.cout + n0 + cc) =
        *reinterpret_cast<const uint4*>(lds + row * C::OS + cc);
  }
}

template <int BN, bool RESID, int BM = 256>
int launch_gemm(GemmArgs& a, hipStream_t st) {
  using C = GemmCfg<BN, BM>;
  a.mt = (int)((a.npix + C::BM - 1) / C::BM);
  a.nt = a.cout / BN;
  static bool attr_done[QCN_MAX_DEV] = {};
  if (!qcn_set_lds_once((const void*)conv_gemm_kernel<BN, RESID, BM>, C::LDS, attr_done))
    return QCN_ERR_HIP;
  hipLaunchKernelGGL((conv_gemm_kernel<BN, RESID, BM>), dim3(a.mt * a.nt), dim3(C::NT), C::LDS, st, a);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

// compile-time loop: f(integral_constant<int, I>) for I in [B, E)
template <int B, int E, class F>
QCN_DEV void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// raw buffer descriptor (wave-uniform base, 2 GiB range, no stride)
QCN_DEV v4i buf_rsrc(const void* base) {
  const uint64_t p = (uint64_t)(uintptr_t)base;
  return (v4i){(int)(uint32_t)p, (int)((uint32_t)(p >> 32) & 0xffff), 0x7fffffff, 0x00020000};
}
// 16-B buffer load / store issued from inline asm: invisible to the
// compiler's wait-count pass, so the caller counts vmcnt itself
QCN_DEV v4i asm_bload(v4i rs, int voff) {
  v4i r;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(r) : "v"(voff), "s"(rs) : "memory");
  return r;
}
QCN_DEV void asm_bstore(v4i rs, int voff, v4i d) {
  // s_nop: a VALU write of a >8-byte store's data VGPR right behind the store
  // needs a wait state (the hazard recognizer does not see inside asm)
  asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen\n\ts_nop 1" :: "v"(d), "v"(voff), "s"(rs) : "memory");
}

// ---------------------------------------------------------------------------
// Streaming 1x1 conv (stride 1, no padding, K = Cin <= 512): the bottleneck's
// thin expand / reduce convs move 16-32 output bytes (plus 16 identity bytes
// for the join) per 64-256 MACs, so they are HBM-bound, and the tiled kernel
// above — load a stage, multiply, requantize, store, one tile per workgroup
// residency — leaves HBM idle during each tile's epilogue.  Here every wave
// owns one 32-channel output tile for good: its A fragments (the channel
// tile's weights, K/32 x 16 B per lane) and epilogue constants stay in
// registers, and it walks a chunk of 32-pixel strips with the next P strips'
// activations and identity bytes already in flight.  The NW waves of a
// workgroup (and the cg workgroups of a chunk, all placed on one XCD) read the
// same strips, so each activation byte leaves HBM once.
//
// Activations (B fragments) come either straight into registers (BL = false:
// K/32 16-B loads per lane and strip), or (BL = true, K = 256: eight 1-KiB
// pieces per strip that every wave would otherwise fetch itself) through an
// LDS ring filled by LDS-DMA, each wave loading K/32/NW pieces of whole pixel
// rows; the row's 16-B chunks are XOR-swizzled by pixel so the MFMA's
// lane-linear fragment reads are conflict-free.
//
// Per strip: K/32 MFMAs, the FBGEMM requant of 16 values per lane, two rounds
// of v_permlane32_swap (MFMA layout -> 16 consecutive channels per lane), and
// an LDS transpose of the workgroup's NW x 32 channels: a store of the MFMA
// layout is 32 rows x 32 B per instruction, which runs the address path at
// ~3x the work per byte of whole lines (3.8 vs 5.8 TB/s on this conv's
// traffic, tools/micro/stream_shape.hip; 1.5x fetch and 1.3x write
// amplification), so each wave moves 32/NW whole row segments of NW x 32 B
// instead.  With RESID the join of custom_quantization_model.py:94-101 runs on
// those row segments with the same fp32 op sequence as the tiled kernel's
// join (bit-identical).
//
// Epilogue modes (uniform per launch, so compiled in): RQ 0 = zp_y 0 and no
// ReLU floor (v_cvt_pk_u8_f32 alone rounds and saturates), 1 = no ReLU floor
// (rint + zp, then the saturating pack), 2 = general clamp; ZO (RESID) = the
// join's output zero point is 0 (ReLU = saturation at 0).

// vmcnt bound at a wait of the strip loop, from the issue order: prologue
// B(j) x NB, I(j) for j < P; step t issues S(t), B(t+P) x NB, I(t+P) after its
// waits.  BL = false waits at the head of step t for B(t), I(t); BL = true
// waits before step t's barrier for B(t+1), I(t) (t = -1: the prologue's wait
// for B(0)).  NS: stores per step (2 with the fused reduce: its previous
// strip's output is stored after the step's first barrier), NS0 at a chunk's
// first step.  The steady-state bound (t = P) is modelled on a first round, so
// with NS0 < NS it is one op conservative.  Returns the number of younger
// operations that may stay in flight.
constexpr int stream_vmcnt(int P, int NB, bool RESID, bool BL, int t, int NS = 1, int NS0 = 1) {
  int pos = 0, last = -1;
  auto issue_b = [&](int strip) {
    for (int i = 0; i < NB; ++i) {
      if (strip == (BL ? t + 1 : t)) last = pos;
      ++pos;
    }
  };
  auto issue_i = [&](int strip) {
    if (!RESID) return;
    if (strip == t && !(BL && t < 0)) last = pos;
    ++pos;
  };
  for (int j = 0; j < P; ++j) { issue_b(j); issue_i(j); }
  for (int u = 0; u < t; ++u) { pos += u == 0 ? NS0 : NS; issue_b(u + P); issue_i(u + P); }
  return pos - 1 - last;
}

template <int K, int NW, bool RESID, int P, int RQ, int ZO, bool BL, bool S2 = false, int CR = 0>
__global__ __launch_bounds__(NW * 64, (CR > 0 ? 1 : (K == 64 ? 3 : 2))) void conv1x1_stream_kernel(GemmArgs a) {
  static_assert(!S2 || BL, "stride 2 reads its rows through the LDS ring");
  static_assert(CR == 0 || (RESID && K == 64 && NW == 8 && !BL && (CR == 64 || CR == 128)),
                "the fused reduce follows a 64 -> 256 expand + join (one workgroup holds a strip's 256 channels)");
  constexpr int KC = K / 32;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l32 = lane & 31, hi = lane >> 5;
  // block -> (chunk, channel group); the cg groups of a chunk share blockIdx % 8
  const int b = blockIdx.x, x8 = b & 7, kq = b >> 3;
  const int cgi = kq % a.cg, c = (kq / a.cg) * 8 + x8;
  if (c >= a.nchunk) return;
  const int s0 = c * a.per, s1 = min(s0 + a.per, a.nstrip);
  const int cout = a.cout, co0 = (cgi * NW + wave) * 32;

  v4i wa[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc)
    wa[kc] = *reinterpret_cast<const v4i*>(a.w + ((long)kc * cout + co0 + l32) * 32 + hi * 16);
  // constants of the lane's channels co0 + 8g + 4hi + e
  v16i corr;
  v2f u[8], v[8], m[8];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int co = co0 + 8 * g + 4 * hi;
    const int4 c4 = *reinterpret_cast<const int4*>(a.corr + co);
    corr[4 * g] = c4.x; corr[4 * g + 1] = c4.y; corr[4 * g + 2] = c4.z; corr[4 * g + 3] = c4.w;
    const float4 x4 = *reinterpret_cast<const float4*>(a.u + co);
    const float4 y4 = *reinterpret_cast<const float4*>(a.v + co);
    const float4 z4 = *reinterpret_cast<const float4*>(a.mult + co);
    u[2 * g] = (v2f){x4.x, x4.y}; u[2 * g + 1] = (v2f){x4.z, x4.w};
    v[2 * g] = (v2f){y4.x, y4.y}; v[2 * g + 1] = (v2f){y4.z, y4.w};
    m[2 * g] = (v2f){z4.x, z4.y}; m[2 * g + 1] = (v2f){z4.z, z4.w};
  }
  // the constants land before the strip loop (otherwise the compiler's wait
  // for them sits inside the loop as a vmcnt(0) that drains the prefetch)
#pragma unroll
  for (int h = 0; h < 8; ++h) asm volatile("" :: "v"(u[h]), "v"(v[h]), "v"(m[h]));
  asm volatile("" :: "v"(corr));
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) asm volatile("" :: "v"(wa[kc]));
  const float zpf = (float)a.zp_y, lof = (float)a.lo;
  const v2f zpv = {zpf, zpf};
  const v2f s3v = {a.s3, a.s3};
  const v2f zr = {(float)a.z_r, (float)a.z_r}, sr = {a.s_r, a.s_r}, io = {a.inv_o, a.inv_o};
  const float zof = (float)a.z_o;
  // ZO == 2: the join's one-form constants (ja, jb, jc) travel in s3, s_r, inv_o
  const v2f jav = {a.s3, a.s3}, jbv = {a.s_r, a.s_r}, jcv = {a.inv_o, a.inv_o};
  const int lastp = (int)(a.npix - 1);   // npix < 2^31 - 256 (checked at the ABI)

  // Fused reduce (CR > 0): the next bottleneck's 1x1 conv (K = 256 -> CR) on
  // the strip's joined bytes, which never leave the chip for it.  The joined
  // 32 x 256 tile goes to LDS (q ^ 0x80, pixel stride 288 B: 16 B x (2 mod 4),
  // conflict-free for the 16x16 B reads); the (CR / 16) x 2 jobs of 16 couts x
  // 16 pixels on v_mfma_i32_16x16x64_i8 spread over the 8 waves (NJ per wave),
  // their A fragments (4 K-steps x 16 B per lane) and requant constants
  // resident in registers.  Lane (p, g) of a job holds couts 4g .. 4g + 3 of
  // its pixel p: one dword per lane and job into an LDS [32][CR] tile, which
  // the next strip stores as whole 16-B row pieces after its first barrier
  // (dword stores of the MFMA layout cost the CR = 128 form ~0.1 ms).
  constexpr int NJ = CR > 0 ? CR / 64 : 1, RS2 = 288;
  const int p16 = lane & 15, g16 = lane >> 4;
  v4i wr2[NJ][4];
  float4 ru[NJ], rv[NJ], rm[NJ];
  int4 rc[NJ];
  if constexpr (CR > 0) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int job = wave + 8 * j, c16 = job % (CR / 16);
#pragma unroll
      for (int s = 0; s < 4; ++s)
        wr2[j][s] = *reinterpret_cast<const v4i*>(a.w2 + ((long)(2 * s + (g16 >> 1)) * CR + c16 * 16 + p16) * 32 +
                                                  16 * (g16 & 1));
      const int co = c16 * 16 + 4 * g16;
      ru[j] = *reinterpret_cast<const float4*>(a.u2 + co);
      rv[j] = *reinterpret_cast<const float4*>(a.v2 + co);
      rm[j] = *reinterpret_cast<const float4*>(a.mult2 + co);
      rc[j] = *reinterpret_cast<const int4*>(a.corr2 + co);
      asm volatile("" :: "v"(wr2[j][0]), "v"(wr2[j][1]), "v"(wr2[j][2]), "v"(wr2[j][3]));
      asm volatile("" :: "v"(ru[j].x), "v"(ru[j].y), "v"(ru[j].z), "v"(ru[j].w), "v"(rv[j].x), "v"(rv[j].y),
                   "v"(rv[j].z), "v"(rv[j].w));
      asm volatile("" :: "v"(rm[j].x), "v"(rm[j].y), "v"(rm[j].z), "v"(rm[j].w), "v"(rc[j].x), "v"(rc[j].y),
                   "v"(rc[j].z), "v"(rc[j].w));
    }
  }
  const float zp2f = (float)a.zp2, lo2f = (float)a.lo2;

  // 32-bit buffer offsets (activations, identity and output are < 2 GiB:
  // checked at launch).  Every memory operation is unconditional: pixel rows
  // past the end (and strips past s1) are clamped to the last pixel, whose
  // output they recompute bit for bit, so the duplicate stores write the same
  // bytes.  The strip loads and stores are issued from inline asm with the
  // waits counted here (stream_vmcnt): on a runtime-trip-count loop the
  // compiler's own bookkeeping falls back to vmcnt(0) at the loop head, which
  // drains the prefetch every round.
  const v4i xr = buf_rsrc(a.x), rr = buf_rsrc(a.r), yr = buf_rsrc(a.y);
  const v4i y2r = buf_rsrc(CR > 0 ? a.y2 : a.y);
  auto pix = [&](int st, int row) {
    st = st < s1 ? st : s1 - 1;
    const int p = st * 32 + row;
    return p < lastp ? p : lastp;
  };
  constexpr int ROWB = NW * 32, RS = ROWB + 16, LPR = ROWB / 16, RPW = 64 / LPR;
  static_assert(RPW * NW == 32, "each wave moves 32 / NW rows of a strip");
  // B ring (BL): 1-KiB pieces of RPB pixel rows, CPR 16-B chunks per row
  // NDMA pieces per wave; with fewer pieces than waves (K = 64) the spare
  // waves repeat a piece into a scratch slot, so every wave issues the same
  // vector-memory ops (the vmcnt bounds are per wave)
  constexpr int CPR = K / 16, RPB = 1024 / K, NDMA = (KC + NW - 1) / NW;
  constexpr int RING = BL ? P * 32 * K + (NDMA * NW > KC ? 1024 : 0) : 16;
  static_assert(!BL || NDMA * NW == KC || NDMA == 1, "pieces split evenly, or one per wave");
  __shared__ __attribute__((aligned(16))) uint8_t tile[2][32 * RS];
  __shared__ __attribute__((aligned(16))) uint8_t tile2[CR > 0 ? 2 : 1][CR > 0 ? 32 * RS2 : 16];
  // the reduce's strip output [32][CR] (row stride RS3), stored as whole 16-B
  // row pieces in the NEXT strip, after its first barrier
  constexpr int RS3 = CR + 16;
  __shared__ __attribute__((aligned(16))) uint8_t tile3[CR > 0 ? 2 : 1][CR > 0 ? 32 * RS3 : 16];
  int last_st = 0;
  auto store_reduced = [&](int sp) {   // strip sp's reduce output: CR / 4 pieces per wave
    if constexpr (CR > 0) {
      if (lane < CR / 4) {
        const int piece = wave * (CR / 4) + lane, row = piece / (CR / 16), c = piece % (CR / 16);
        const v4i v = *reinterpret_cast<const v4i*>(tile3[sp & 1] + row * RS3 + 16 * c);
        asm_bstore(y2r, pix(sp, row) * CR + 16 * c, v);
      }
    }
  };
  __shared__ __attribute__((aligned(16))) uint8_t ring[RING];
  const int rrow = wave * RPW + lane / LPR, rcol = (lane % LPR) * 16;
  const int cb0 = cgi * ROWB;
  // XOR swizzle of a row's 16-B chunks: the 16 lanes of a ds_read_b128 group
  // (distinct pixel rows) land on distinct 16-B bank slots
  constexpr int SD = CPR >= 16 ? 1 : 16 / CPR;
  auto swz = [](int row) { return (row / SD) % CPR; };
  // S2 (the stride-2 downsample 1x1): output pixel (n, oy, ox) reads input
  // pixel (n, 2 oy, 2 ox); p < 2^22 for the fp32-reciprocal divisions
  const int ohw = a.oh * a.ow;
  const float rohw = 1.0f / (float)ohw, rw = 1.0f / (float)a.ow;
  auto in_pix = [&](int p) {
    if constexpr (!S2) return p;
    const int n = div_small(p, ohw, rohw), rem = p - n * ohw;
    const int oy = div_small(rem, a.ow, rw), ox = rem - oy * a.ow;
    return (n * a.h + 2 * oy) * a.w_ + 2 * ox;
  };
  constexpr int NB = BL ? NDMA : KC;   // B vector-memory ops per strip and wave

  v4i bq[BL ? 1 : P][KC];
  v4i rq[P];
  auto load = [&](int q, int st) {
    if constexpr (BL) {
      const int row = lane / CPR;   // row within the piece
#pragma unroll
      for (int j = 0; j < NDMA; ++j) {
        const int i = wave + NW * j, ip = i < KC ? i : i % KC, r = ip * RPB + row;
        uint8_t* dst = i < KC ? ring + q * 32 * K + i * 1024 : ring + P * 32 * K;
        glds16(a.x + (long)in_pix(pix(st, r)) * K + ((lane % CPR) ^ swz(r)) * 16, dst);
      }
    } else {
      const int xo = pix(st, l32) * K + hi * 16;
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) bq[q][kc] = asm_bload(xr, xo + kc * 32);
    }
    if constexpr (RESID) rq[q] = asm_bload(rr, pix(st, rrow) * cout + cb0 + rcol);
  };
  // wait at step t (slot q): the asm ties the slot's registers, so no use of
  // them moves above it
  auto wait_vm = [&](auto tc, int q) {
    constexpr int N = stream_vmcnt(P, NB, RESID, BL, decltype(tc)::value, CR > 0 ? 2 : 1, 1);
    if constexpr (!BL) {
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) asm volatile("" : "+v"(bq[q][kc]));
    }
    if constexpr (RESID) asm volatile("s_waitcnt vmcnt(%1)" : "+v"(rq[q]) : "n"(N) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
    if constexpr (!BL) {
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) asm volatile("" : "+v"(bq[q][kc]));
    }
  };
  auto strip = [&](auto tc, int q, int st) {
    if constexpr (!BL) wait_vm(tc, q);
    v16i acc;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      v4i bx;
      if constexpr (BL)
        bx = *reinterpret_cast<const v4i*>(ring + q * 32 * K + (l32 / RPB) * 1024 +
                                           ((l32 % RPB) * CPR + ((2 * kc + hi) ^ swz(l32))) * 16);
      else
        bx = bq[q][kc];
#pragma unroll
      for (int d = 0; d < 4; ++d) bx[d] ^= (int)0x80808080u;   // u8 -> s8
      acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(wa[kc], bx, kc == 0 ? corr : acc, 0, 0, 0);
    }
    // FBGEMM requant (A6) of the lane's 16 channels, packed as bytes per
    // 4-channel group g (channels 8g + 4hi + 0..3)
    uint32_t w[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const v2f t0 = requant2(acc[4 * g], acc[4 * g + 1], u[2 * g], v[2 * g], m[2 * g]);
      const v2f t1 = requant2(acc[4 * g + 2], acc[4 * g + 3], u[2 * g + 1], v[2 * g + 1], m[2 * g + 1]);
      uint32_t wd;
      if constexpr (RQ == 0) {
        wd = __builtin_amdgcn_cvt_pk_u8_f32(t0.x, 0, 0u);
        wd = __builtin_amdgcn_cvt_pk_u8_f32(t0.y, 1, wd);
        wd = __builtin_amdgcn_cvt_pk_u8_f32(t1.x, 2, wd);
        wd = __builtin_amdgcn_cvt_pk_u8_f32(t1.y, 3, wd);
      } else if constexpr (RQ == 1) {
        const v2f r0 = (v2f){__builtin_rintf(t0.x), __builtin_rintf(t0.y)} + zpv;
        const v2f r1 = (v2f){__builtin_rintf(t1.x), __builtin_rintf(t1.y)} + zpv;
        wd = __builtin_amdgcn_cvt_pk_u8_f32(r0.x, 0, 0u);
        wd = __builtin_amdgcn_cvt_pk_u8_f32(r0.y, 1, wd);
        wd = __builtin_amdgcn_cvt_pk_u8_f32(r1.x, 2, wd);
        wd = __builtin_amdgcn_cvt_pk_u8_f32(r1.y, 3, wd);
      } else {
        wd = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_amdgcn_fmed3f(__builtin_rintf(t0.x) + zpf, lof, 255.0f), 0, 0u);
        wd = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_amdgcn_fmed3f(__builtin_rintf(t0.y) + zpf, lof, 255.0f), 1, wd);
        wd = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_amdgcn_fmed3f(__builtin_rintf(t1.x) + zpf, lof, 255.0f), 2, wd);
        wd = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_amdgcn_fmed3f(__builtin_rintf(t1.y) + zpf, lof, 255.0f), 3, wd);
      }
      w[g] = wd;
    }
    // low lanes: c0-3 | c8-11 | c16-19 | c24-27 ; high lanes: c4-7 | c12-15 | ...
    auto s01 = __builtin_amdgcn_permlane32_swap(w[0], w[1], false, false);
    auto s23 = __builtin_amdgcn_permlane32_swap(w[2], w[3], false, false);
    w[0] = s01[0]; w[1] = s01[1]; w[2] = s23[0]; w[3] = s23[1];
    auto s02 = __builtin_amdgcn_permlane32_swap(w[0], w[2], false, false);
    auto s13 = __builtin_amdgcn_permlane32_swap(w[1], w[3], false, false);
    w[0] = s02[0]; w[2] = s02[1]; w[1] = s13[0]; w[3] = s13[1];
    // now low lanes hold channels co0 + 0..15, high lanes co0 + 16..31
    uint8_t* tb = tile[st & 1];
    *reinterpret_cast<v4i*>(tb + l32 * RS + wave * 32 + 16 * hi) = (v4i){(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
    if constexpr (BL) wait_vm(tc, q);
    // the tile of strip st is complete (and, BL, strip st+1's B pieces and
    // every wave's reads of strip st's); the other tile buffer's readers
    // (strip st-1) passed this barrier only after their reads
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if constexpr (CR > 0) {
      // strip st - 1's reduce output (complete in tile3: every wave wrote its
      // part before this barrier); a chunk's first strip has none
      if (st != s0) store_reduced(st - 1);
      last_st = st;
    }
    {
      const v4i yv = *reinterpret_cast<const v4i*>(tb + rrow * RS + rcol);
#pragma unroll
      for (int g = 0; g < 4; ++g) w[g] = (uint32_t)yv[g];
    }
    if constexpr (RESID) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint32_t rw = (uint32_t)rq[q][g];
        uint32_t o = 0;
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const v2f yf = {(float)((w[g] >> (8 * e)) & 0xff), (float)((w[g] >> (8 * e + 8)) & 0xff)};
          const v2f rf = {(float)((rw >> (8 * e)) & 0xff), (float)((rw >> (8 * e + 8)) & 0xff)};
          if constexpr (ZO != 0) {
            // ZO == 2: the one-form join, 2 packed fma per 2 outputs instead of 6 packed ops
            v2f sm;
            if constexpr (ZO == 2) sm = __builtin_elementwise_fma(yf, jav, __builtin_elementwise_fma(rf, jbv, jcv));
            else sm = ((yf - zpv) * s3v + (rf - zr) * sr) * io;
            o = __builtin_amdgcn_cvt_pk_u8_f32(sm.x, e, o);
            o = __builtin_amdgcn_cvt_pk_u8_f32(sm.y, e + 1, o);
          } else {
            const v2f sm = ((yf - zpv) * s3v + (rf - zr) * sr) * io;   // relu(s) * inv == max(s * inv, 0) since inv > 0
            o = __builtin_amdgcn_cvt_pk_u8_f32(
                __builtin_amdgcn_fmed3f(__builtin_rintf(__builtin_fmaxf(sm.x, 0.0f)) + zof, 0.0f, 255.0f), e, o);
            o = __builtin_amdgcn_cvt_pk_u8_f32(
                __builtin_amdgcn_fmed3f(__builtin_rintf(__builtin_fmaxf(sm.y, 0.0f)) + zof, 0.0f, 255.0f), e + 1,
                o);
          }
        }
        w[g] = o;
      }
    }
    if constexpr (CR > 0) {
      uint8_t* t2 = tile2[st & 1];
      *reinterpret_cast<v4i*>(t2 + rrow * RS2 + rcol) =
          (v4i){(int)(w[0] ^ 0x80808080u), (int)(w[1] ^ 0x80808080u), (int)(w[2] ^ 0x80808080u),
                (int)(w[3] ^ 0x80808080u)};
      // every row of the strip is in tile2; tile2[st & 1]'s previous readers
      // (strip st - 2) passed this strip's first barrier after their reads
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int job = wave + 8 * j, pb = job / (CR / 16);
        const uint8_t* bp = t2 + (pb * 16 + p16) * RS2 + 16 * g16;
        v4i acc2 = (v4i){rc[j].x, rc[j].y, rc[j].z, rc[j].w};
#pragma unroll
        for (int s = 0; s < 4; ++s)
          acc2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(wr2[j][s], *reinterpret_cast<const v4i*>(bp + 64 * s), acc2,
                                                       0, 0, 0);
        const float uu[4] = {ru[j].x, ru[j].y, ru[j].z, ru[j].w}, vv[4] = {rv[j].x, rv[j].y, rv[j].z, rv[j].w};
        const float mm[4] = {rm[j].x, rm[j].y, rm[j].z, rm[j].w};
        uint32_t wd = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float f = __builtin_fmaf(uu[e], vv[e], (float)acc2[e]) * mm[e];
          wd = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_amdgcn_fmed3f(__builtin_rintf(f) + zp2f, lo2f, 255.0f), e, wd);
        }
        const int c16 = job % (CR / 16);
        *reinterpret_cast<uint32_t*>(tile3[st & 1] + (pb * 16 + p16) * RS3 + c16 * 16 + 4 * g16) = wd;
      }
    }
    asm_bstore(yr, pix(st, rrow) * cout + cb0 + rcol, (v4i){(int)w[0], (int)w[1], (int)w[2], (int)w[3]});
    load(q, st + P);   // refill the slot
  };
#pragma unroll
  for (int q = 0; q < P; ++q) load(q, s0 + q);
  if constexpr (BL) {
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" :: "n"(stream_vmcnt(P, NB, RESID, BL, -1)) : "memory");
  }
  // first round (its own wait counts), then steady rounds
  static_for<0, P>([&](auto q) { strip(q, q, s0 + q); });
  for (int s = s0 + P; s < s1; s += P) {
    static_for<0, P>([&](auto q) { strip(std::integral_constant<int, P>{}, q, s + q); });
  }
  if constexpr (CR > 0) {   // the last strip's reduce output
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    store_reduced(last_st);
  }
  // drain: the last refills are never consumed; keep their registers live
  // until they landed
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int q = 0; q < P; ++q) {
    if constexpr (!BL) {
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) asm volatile("" :: "v"(bq[q][kc]));
    }
    if constexpr (RESID) asm volatile("" :: "v"(rq[q]));
  }
}

template <int K, int NW, bool RESID, int P, int RQ, int ZO, bool BL, bool S2 = false, int CR = 0>
int launch_stream(GemmArgs& a, hipStream_t st) {
  const auto kern = conv1x1_stream_kernel<K, NW, RESID, P, RQ, ZO, BL, S2, CR>;
  static int occ_dev[QCN_MAX_DEV] = {};
  const int d = qcn_current_device(), ncu = qcn_cu_count();
  if (d < 0 || ncu <= 0) return QCN_ERR_HIP;
  int& occ = occ_dev[d];
  if (!occ && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, NW * 64, 0) != hipSuccess || occ <= 0))
    return QCN_ERR_HIP;
  a.cg = a.cout / (32 * NW);
  a.nstrip = (int)((a.npix + 31) / 32);
  // one resident wave of workgroups: cg x nchunk ~ CUs x occupancy, chunks a
  // multiple of 8 (the XCD interleave of blockIdx)
  int nchunk = (ncu * occ) / a.cg;
  nchunk = nchunk < 8 ? 8 : nchunk & ~7;
  if (nchunk > a.nstrip) nchunk = a.nstrip;
  a.per = (a.nstrip + nchunk - 1) / nchunk;
  a.nchunk = (a.nstrip + a.per - 1) / a.per;
  const int grid = (a.nchunk + 7) / 8 * 8 * a.cg;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NW * 64), 0, st, a);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

// ---- host: the residual join in one form (the streaming kernel's ZO == 2)
//
// With ZO (output zero point 0: ReLU = saturation at 0) the streaming
// kernel's join is out = sat(rne(((y - z3) s3 + (r - zr) sr) * inv_o)) over the
// byte pair (y3, identity), in that fp32 op order.  It is replaced by
// sat(rne(fma(y, ja, fma(r, jb, jc)))) when candidate constants near
// (s3 inv_o, sr inv_o, -(z3 s3 + zr sr) inv_o) reproduce it for all 65536
// pairs (an interval for jc per (ja, jb) candidate, then an exact fp32 check);
// otherwise the kernel keeps the op sequence.  Cached per qparam set.
namespace {

float join_ref_host(int y, int r, float z3f, float s3, float zrf, float sr, float io) {
  const float t1 = ((float)y - z3f) * s3;
  const float t2 = ((float)r - zrf) * sr;
  const float sm = (t1 + t2) * io;
  return std::fmin(std::fmax(std::nearbyint(sm), 0.0f), 255.0f);
}

bool join_affine_solve(const GemmArgs& a, float* j) {
  struct Entry { float s3, sr, io; int z3, zr; bool ok; float ja, jb, jc; };
  static thread_local Entry cache[32];
  static thread_local int ncache = 0, next = 0;
  for (int i = 0; i < ncache; ++i) {
    const Entry& e = cache[i];
    if (e.s3 == a.s3 && e.sr == a.s_r && e.io == a.inv_o && e.z3 == a.zp_y && e.zr == a.z_r) {
      j[0] = e.ja; j[1] = e.jb; j[2] = e.jc;
      return e.ok;
    }
  }
  const float z3f = (float)a.zp_y, zrf = (float)a.z_r;
  static thread_local float ref[256 * 256];
  for (int y = 0; y < 256; ++y)
    for (int r = 0; r < 256; ++r) ref[y * 256 + r] = join_ref_host(y, r, z3f, a.s3, zrf, a.s_r, a.inv_o);
  const double A0 = (double)a.s3 * a.inv_o, B0 = (double)a.s_r * a.inv_o;
  const float fa0 = (float)A0, fb0 = (float)B0;
  bool ok = false;
  float ja = 0.f, jb = 0.f, jc = 0.f;
  for (int k = 0; k < 25 && !ok; ++k) {   // ja, jb within +-2 ulp of the products
    const float A = std::nextafter(fa0, (k % 5) < 2 ? 0.f : 1e9f), B = std::nextafter(fb0, (k / 5) < 2 ? 0.f : 1e9f);
    const float Ac = (k % 5) == 2 ? fa0 : ((k % 5) == 4 ? std::nextafter(A, 1e9f) : ((k % 5) == 0 ? A : std::nextafter(A, 0.f)));
    const float Bc = (k / 5) == 2 ? fb0 : ((k / 5) == 4 ? std::nextafter(B, 1e9f) : ((k / 5) == 0 ? B : std::nextafter(B, 0.f)));
    if (!(Ac > 0.f) || !(Bc > 0.f)) continue;
    double lb = -1e30, ub = 1e30;
    for (int y = 0; y < 256; ++y)
      for (int r = 0; r < 256; ++r) {
        const double g = ref[y * 256 + r], base = (double)y * Ac + (double)r * Bc;
        if (g > 0.0) lb = std::max(lb, g - 0.5 - base);
        if (g < 255.0) ub = std::min(ub, g + 0.5 - base);
      }
    if (!(lb < ub)) continue;
    const float C = (float)(lb > -1e29 && ub < 1e29 ? 0.5 * (lb + ub) : (lb > -1e29 ? lb + 0.25 : ub - 0.25));
    bool exact = true;
    for (int y = 0; y < 256 && exact; ++y)
      for (int r = 0; r < 256; ++r) {
        const float v = std::fma((float)y, Ac, std::fma((float)r, Bc, C));
        if (std::fmin(std::fmax(std::nearbyint(v), 0.0f), 255.0f) != ref[y * 256 + r]) { exact = false; break; }
      }
    if (exact) { ok = true; ja = Ac; jb = Bc; jc = C; }
  }
  j[0] = ja; j[1] = jb; j[2] = jc;
  cache[next] = Entry{a.s3, a.s_r, a.inv_o, a.zp_y, a.z_r, ok, ja, jb, jc};
  next = (next + 1) % 32;
  if (ncache < 32) ++ncache;
  return ok;
}

}  // namespace

template <int K, int NW, bool RESID, int P, bool BL, bool S2 = false>
int stream_modes(GemmArgs& a, hipStream_t st) {
  if constexpr (S2) {   // the downsample conv: no ReLU, no join
    if (a.lo != 0) return -1;
    return a.zp_y == 0 ? launch_stream<K, NW, false, P, 0, true, true, true>(a, st)
                       : launch_stream<K, NW, false, P, 1, true, true, true>(a, st);
  } else if constexpr (RESID) {   // the join's conv has no ReLU (lo == 0)
    // ZO: 0 general output zero point, 1 zero (ReLU = saturation), 2 zero with
    // the join in its exact one form (join_affine_solve), whose constants
    // replace s3 / s_r / inv_o in this launch's copy of the arguments
    float j[3];
    if (a.z_o == 0 && join_affine_solve(a, j)) {
      GemmArgs b = a;
      b.s3 = j[0]; b.s_r = j[1]; b.inv_o = j[2];
      return a.zp_y == 0 ? launch_stream<K, NW, true, P, 0, 2, BL>(b, st) : launch_stream<K, NW, true, P, 1, 2, BL>(b, st);
    }
    const int zo = a.z_o == 0 ? 1 : 0;
    if (a.zp_y == 0)
      return zo ? launch_stream<K, NW, true, P, 0, 1, BL>(a, st) : launch_stream<K, NW, true, P, 0, 0, BL>(a, st);
    return zo ? launch_stream<K, NW, true, P, 1, 1, BL>(a, st) : launch_stream<K, NW, true, P, 1, 0, BL>(a, st);
  } else {
    if (a.lo == 0) return a.zp_y == 0 ? launch_stream<K, NW, false, P, 0, true, BL>(a, st)
                                      : launch_stream<K, NW, false, P, 1, true, BL>(a, st);
    return launch_stream<K, NW, false, P, 2, true, BL>(a, st);
  }
}

// The layer-1 expand + join (K = 64 -> 256) with the next block's reduce
// (256 -> CR) fused: 8 waves per workgroup so one holds a strip's 256 joined
// channels; the join's forms as stream_modes.
template <int CR>
int join_reduce_modes(GemmArgs& a, hipStream_t st) {
  float j[3];
  if (a.z_o == 0 && join_affine_solve(a, j)) {
    GemmArgs b = a;
    b.s3 = j[0]; b.s_r = j[1]; b.inv_o = j[2];
    return a.zp_y == 0 ? launch_stream<64, 8, true, 4, 0, 2, false, false, CR>(b, st)
                       : launch_stream<64, 8, true, 4, 1, 2, false, false, CR>(b, st);
  }
  const int zo = a.z_o == 0 ? 1 : 0;
  if (a.zp_y == 0)
    return zo ? launch_stream<64, 8, true, 4, 0, 1, false, false, CR>(a, st)
              : launch_stream<64, 8, true, 4, 0, 0, false, false, CR>(a, st);
  return zo ? launch_stream<64, 8, true, 4, 1, 1, false, false, CR>(a, st)
            : launch_stream<64, 8, true, 4, 1, 0, false, false, CR>(a, st);
}

// K in {64, 128, 256, 512}; Cout % 128 == 0 (4 waves per workgroup), or
// Cout % 64 == 0 without the join (2 waves, K <= 256); -1 when the shape has
// no streaming form.  Activations through the LDS ring for K >= 128 with 4
// waves (QCN_STREAM_BL128=0: K = 128 into registers; the layer-2 expand convs
// 0.126 -> 0.108 ms through the ring, profiles/r03_diag_resnet_stream_ab.txt).
// ---------------------------------------------------------------------------
// Whole-image 3x3 stride-1 conv for the small deep maps (layer 3: 14x14, 256
// channels; layer 4: 7x7, 512): the implicit GEMM above gathers a 64-B im2col
// row per output pixel and tap (nine per input byte), and at these shapes it
// is bound by that gather (0.09-0.10 ms per conv at batch 512; 0.065 / 0.073
// ms here).  Here one
// 8-wave workgroup takes one image and 256 output channels: the image is
// staged once in LDS (q ^ 0x80, zero-point halo), wave w owns channel tile w
// for ALL of the image's pixel tiles (NPT = ceil(HW^2 / 32), 7 or 2), its A
// fragments stream from L2 into registers D K-steps ahead, and every tap of a
// pixel tile is an immediate offset from the lane's patch address.  The patch
// row stride is padded so a 16-lane ds_read_b128 group (16 consecutive
// pixels) lands on 16 distinct 16-B bank slots across the row wraps.
// Epilogue: FBGEMM requant (+ReLU floor), permlane swaps, an LDS [pixel][256]
// tile and whole-row 16-B stores.
template <int HW, int CIN, int NS = 1>
struct ImgCfg {
  static constexpr int COUT = 256;                   // channels per workgroup
  // NS waves per channel tile, each taking JW of the image's pixel tiles
  static constexpr int NW = 8 * NS, NT = NW * 64;
  static constexpr int NPX = HW * HW, NPT = (NPX + 31) / 32, JW = (NPT + NS - 1) / NS;
  static constexpr int KC = 9 * CIN / 32;            // K-steps (r, s, 32-channel chunk)
  static constexpr int PW = HW + 2;
  static constexpr int PS = CIN + 16;                // pixel stride: 1 slot (mod 16) per pixel
  static constexpr int RS0 = PW * PS;
  // row stride with (RS / 16) % 16 == HW % 16: slot(pixel) = pixel index mod 16
  static constexpr int RS = RS0 + ((HW - RS0 / 16) % 16 + 16) % 16 * 16;
  static constexpr int PATCH = PW * RS;
  static constexpr int OS = COUT + 16;
  static constexpr int OUT = NPX * OS;
  static constexpr int LDS = (PATCH > OUT ? PATCH : OUT);
  static_assert(PS % 256 == 16 && (RS / 16) % 16 == HW % 16, "conflict-free patch reads");
  static_assert(CIN % 64 == 0, "whole 64-channel chunks");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

template <int HW, int CIN, int D, int NS>
__global__ __launch_bounds__((ImgCfg<HW, CIN, NS>::NT), 1) void conv3x3_img_kernel(GemmArgs a) {
  using C = ImgCfg<HW, CIN, NS>;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, hi = lane >> 5;
  const int ncg = a.cout / C::COUT;
  const int img = blockIdx.x / ncg, cg = blockIdx.x % ncg;
  const int ct = wave % 8, jg = wave / 8;             // channel tile, pixel-tile group
  const int co0 = cg * C::COUT + ct * 32;            // this wave's channel tile

  // ---- stage the image: 16-B pieces, q ^ 0x80; halo = zp ^ 0x80
  const uint8_t* xi = a.x + (long)img * C::NPX * CIN;
  constexpr int PPP = CIN / 16;                      // pieces per pixel
  constexpr int NPC = C::NPX * PPP;
  constexpr int PPT = (NPC + C::NT - 1) / C::NT;
  uint4 pc[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int e = tid + C::NT * i;
    pc[i] = e < NPC ? *reinterpret_cast<const uint4*>(xi + (long)e * 16) : make_uint4(0, 0, 0, 0);
  }
  // weights: A fragment of K-step kc for this wave's channel tile
  const int8_t* wl = a.w + ((long)co0 + l32) * 32 + hi * 16;
  const long wstep = (long)a.cout * 32;
  v4i wq[D];
#pragma unroll
  for (int d = 0; d < D; ++d) wq[d] = *reinterpret_cast<const v4i*>(wl + d * wstep);
  v16i corr;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int4 c4 = *reinterpret_cast<const int4*>(a.corr + co0 + 8 * g + 4 * hi);
    corr[4 * g] = c4.x; corr[4 * g + 1] = c4.y; corr[4 * g + 2] = c4.z; corr[4 * g + 3] = c4.w;
  }
  const uint32_t zq = xor80(splat_u8(a.x_zp));
  {
    // halo pixels: rows 0 and HW+1, columns 0 and HW+1 of the patch
    constexpr int NH = 2 * C::PW + 2 * HW;
    for (int e = tid; e < NH * PPP; e += C::NT) {
      const int hp = e / PPP, k = e % PPP;
      int py, px;
      if (hp < C::PW) { py = 0; px = hp; }
      else if (hp < 2 * C::PW) { py = HW + 1; px = hp - C::PW; }
      else { py = 1 + (hp - 2 * C::PW) / 2; px = (hp - 2 * C::PW) % 2 ? HW + 1 : 0; }
      *reinterpret_cast<uint4*>(lds + py * C::RS + px * C::PS + 16 * k) = make_uint4(zq, zq, zq, zq);
    }
  }
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int e = tid + C::NT * i;
    if (e < NPC) {
      const int p = e / PPP, k = e % PPP, y = p / HW, x = p % HW;
      const uint4 v = pc[i];
      *reinterpret_cast<uint4*>(lds + (y + 1) * C::RS + (x + 1) * C::PS + 16 * k) =
          make_uint4(xor80(v.x), xor80(v.y), xor80(v.z), xor80(v.w));
    }
  }
  __syncthreads();

  // ---- main loop: lane (l32, hi) of pixel tile j reads pixel j*32 + l32
  // (clamped; its outputs are never stored), channels 16 hi of the chunk
  int pb[C::JW];
#pragma unroll
  for (int j = 0; j < C::JW; ++j) {
    int p = (jg * C::JW + j) * 32 + l32;
    p = p < C::NPX ? p : C::NPX - 1;
    pb[j] = (p / HW) * C::RS + (p % HW) * C::PS + hi * 16;
  }
  v16i acc[C::JW];
  // software pipeline (sched_barrier fences keep it: left alone, the
  // scheduler sank every load next to its use, one vmcnt(0) / lgkmcnt(0) per
  // MFMA): the next K-step's B fragments are read during this step's MFMAs,
  // and the A fragment D steps ahead is loaded right after this step's use
  auto koff = [](int kc) {
    const int tap = kc / (CIN / 32), ch = kc % (CIN / 32);
    return (tap / 3) * C::RS + (tap % 3) * C::PS + ch * 32;
  };
  v4i bb[2][C::JW];
#pragma unroll
  for (int j = 0; j < C::JW; ++j) bb[0][j] = *reinterpret_cast<const v4i*>(lds + pb[j] + koff(0));
#pragma unroll
  for (int kc = 0; kc < C::KC; ++kc) {
    __builtin_amdgcn_sched_barrier(0);
    if (kc + 1 < C::KC) {
#pragma unroll
      for (int j = 0; j < C::JW; ++j)
        bb[(kc + 1) & 1][j] = *reinterpret_cast<const v4i*>(lds + pb[j] + koff(kc + 1));
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < C::JW; ++j)
      acc[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wq[kc % D], bb[kc & 1][j], kc == 0 ? corr : acc[j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (kc + D < C::KC) wq[kc % D] = *reinterpret_cast<const v4i*>(wl + (kc + D) * wstep);
  }
  __syncthreads();   // the patch is dead: its space becomes the output tile

  // ---- epilogue: requant (+ReLU floor) -> bytes -> 16 consecutive channels
  // per lane -> LDS [pixel][OS] -> whole-row stores
  {
    float u[16], v[16], m[16];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int co = co0 + 8 * g + 4 * hi;
      const float4 x4 = *reinterpret_cast<const float4*>(a.u + co);
      const float4 y4 = *reinterpret_cast<const float4*>(a.v + co);
      const float4 z4 = *reinterpret_cast<const float4*>(a.mult + co);
      u[4 * g] = x4.x; u[4 * g + 1] = x4.y; u[4 * g + 2] = x4.z; u[4 * g + 3] = x4.w;
      v[4 * g] = y4.x; v[4 * g + 1] = y4.y; v[4 * g + 2] = y4.z; v[4 * g + 3] = y4.w;
      m[4 * g] = z4.x; m[4 * g + 1] = z4.y; m[4 * g + 2] = z4.z; m[4 * g + 3] = z4.w;
    }
    const float zpf = (float)a.zp_y, lof = (float)a.lo;
#pragma unroll
    for (int j = 0; j < C::JW; ++j) {
      uint32_t w[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint32_t wd = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e;
          wd = __builtin_amdgcn_cvt_pk_u8_f32(requant_f(acc[j][r], u[r], v[r], m[r], zpf, lof), e, wd);
        }
        w[g] = wd;
      }
      auto s01 = __builtin_amdgcn_permlane32_swap(w[0], w[1], false, false);
      auto s23 = __builtin_amdgcn_permlane32_swap(w[2], w[3], false, false);
      w[0] = s01[0]; w[1] = s01[1]; w[2] = s23[0]; w[3] = s23[1];
      auto s02 = __builtin_amdgcn_permlane32_swap(w[0], w[2], false, false);
      auto s13 = __builtin_amdgcn_permlane32_swap(w[1], w[3], false, false);
      w[0] = s02[0]; w[2] = s02[1]; w[1] = s13[0]; w[3] = s13[1];
      const int p = (jg * C::JW + j) * 32 + l32;
      if (p < C::NPX)
        *reinterpret_cast<uint4*>(lds + p * C::OS + ct * 32 + 16 * hi) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
  __syncthreads();
  constexpr int TPR = C::COUT / 16;                  // threads per pixel row
  uint8_t* yo = a.y + (long)img * C::NPX * a.cout + cg * C::COUT;
  for (int e = tid; e < C::NPX * TPR; e += C::NT) {
    const int p = e / TPR, k = e % TPR;
    *reinterpret_cast<uint4*>(yo + (long)p * a.cout + 16 * k) =
        *reinterpret_cast<const uint4*>(lds + p * C::OS + 16 * k);
  }
}

template <int HW, int CIN, int D, int NS>
int launch_img(GemmArgs& a, hipStream_t st) {
  using C = ImgCfg<HW, CIN, NS>;
  static bool attr_done[QCN_MAX_DEV] = {};
  if (!qcn_set_lds_once((const void*)conv3x3_img_kernel<HW, CIN, D, NS>, C::LDS, attr_done)) return QCN_ERR_HIP;
  hipLaunchKernelGGL((conv3x3_img_kernel<HW, CIN, D, NS>), dim3(a.n * (a.cout / C::COUT)), dim3(C::NT), C::LDS, st,
                     a);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

// the stride-2 downsample 1x1 (no padding, K in {256, 512}, Cout % 128 == 0)
inline int dispatch_stream_s2(GemmArgs& a, hipStream_t st) {
  if (a.npix * (long)a.cout >= (1L << 31) - 4096 || (long)a.n * a.h * a.w_ * a.cin >= (1L << 31) - 4096 ||
      a.npix >= (1L << 22) || a.cout % 128 != 0)
    return -1;
  switch (a.cin) {
    case 256: return stream_modes<256, 4, false, 4, true, true>(a, st);
    case 512: return stream_modes<512, 4, false, 3, true, true>(a, st);
    default: return -1;
  }
}

template <bool RESID>
int dispatch_stream(GemmArgs& a, hipStream_t st) {
  // 32-bit buffer offsets
  if (a.npix * (long)(a.cin > a.cout ? a.cin : a.cout) >= (1L << 31) - 4096) return -1;
  if (a.cout % 128 != 0) {
    if (RESID || a.cout % 64 != 0) return -1;
    switch (a.cin) {
      case 64: return stream_modes<64, 2, false, 4, false>(a, st);
      case 128: return stream_modes<128, 2, false, 3, false>(a, st);
      case 256: return stream_modes<256, 2, false, 4, true>(a, st);
      default: return -1;
    }
  }
  switch (a.cin) {
    // K = 64 keeps its activations in registers (through the LDS-DMA ring it
    // measured slower); K >= 128 streams them through the ring
    case 64: return stream_modes<64, 4, RESID, 4, false>(a, st);
    case 128: return stream_modes<128, 4, RESID, 4, true>(a, st);
    case 256: return stream_modes<256, 4, RESID, 4, true>(a, st);
    case 512: return stream_modes<512, 4, RESID, 3, true>(a, st);
    default: return -1;
  }
}

}  // namespace qcn

extern "C" int qcn_join_affine(float y_scale, int y_zp, float r_scale, int r_zp, float out_scale, float* out) {
  if (!out || !(y_scale > 0.f) || !(r_scale > 0.f) || !(out_scale > 0.f) || y_zp < 0 || y_zp > 255 ||
      r_zp < 0 || r_zp > 255)
    return QCN_ERR_ARG;
  qcn::GemmArgs a{};
  a.s3 = y_scale; a.zp_y = y_zp; a.s_r = r_scale; a.z_r = r_zp; a.inv_o = 1.0f / out_scale;
  return qcn::join_affine_solve(a, out) ? 1 : 0;
}

extern "C" int qcn_conv1x1_join_reduce_u8s8_nhwc(
    const uint8_t* x, int nimg, int h, int w, int cin, int x_zp, const int8_t* w_packed, int cout,
    const float* u, const float* v, const float* mult, const int32_t* corr, int y_zp, const uint8_t* resid,
    float y_scale, float r_scale, int r_zp, float out_scale, int out_zp, uint8_t* y, const int8_t* w2_packed,
    int cout2, const float* u2, const float* v2, const float* mult2, const int32_t* corr2, int y2_zp, int relu2,
    uint8_t* y2, void* stream) {
  if (!x || !w_packed || !u || !v || !mult || !corr || !resid || !y || !w2_packed || !u2 || !v2 || !mult2 ||
      !corr2 || !y2)
    return QCN_ERR_ARG;
  if (nimg <= 0 || h <= 0 || w <= 0 || x_zp < 0 || x_zp > 255 || y_zp < 0 || y_zp > 255 || r_zp < 0 ||
      r_zp > 255 || out_zp < 0 || out_zp > 255 || y2_zp < 0 || y2_zp > 255 || !(y_scale > 0.f) ||
      !(r_scale > 0.f) || !(out_scale > 0.f))
    return QCN_ERR_ARG;
  if (cin != 64 || cout != 256 || (cout2 != 64 && cout2 != 128)) return QCN_ERR_UNSUPPORTED;
  qcn::GemmArgs a{};
  a.x = x; a.w = w_packed;
  a.n = nimg; a.h = h; a.w_ = w; a.cin = cin; a.oh = h; a.ow = w; a.cout = cout;
  a.kh = 1; a.kw = 1; a.sy = 1; a.sx = 1; a.py = 0; a.px = 0;
  a.x_zp = x_zp;
  a.npix = (long)nimg * h * w;
  a.kcs = cin / 32;
  a.u = u; a.v = v; a.mult = mult; a.corr = corr;
  a.zp_y = y_zp; a.lo = 0;
  a.r = resid; a.s3 = y_scale; a.s_r = r_scale; a.inv_o = 1.0f / out_scale;
  a.z_r = r_zp; a.z_o = out_zp; a.y = y;
  a.w2 = w2_packed; a.u2 = u2; a.v2 = v2; a.mult2 = mult2; a.corr2 = corr2;
  a.zp2 = y2_zp; a.lo2 = relu2 ? y2_zp : 0; a.y2 = y2;
  // 32-bit buffer offsets and pixel indices in the kernel
  if (a.npix * (long)cout >= (1L << 31) - 4096) return QCN_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  return cout2 == 64 ? qcn::join_reduce_modes<64>(a, st) : qcn::join_reduce_modes<128>(a, st);
}

extern "C" int qcn_conv_gemm_u8s8_nhwc(const uint8_t* x, int nimg, int h, int w, int cin, int x_zp,
                                       const int8_t* w_packed, int cout, int kh, int kw,
                                       int stride_h, int stride_w, int pad_h, int pad_w,
                                       const float* u, const float* v, const float* mult,
                                       const int32_t* corr, int y_zp, int relu,
                                       const uint8_t* resid, float y_scale, float r_scale,
                                       int r_zp, float out_scale, int out_zp, uint8_t* y,
                                       void* stream) {
  if (!x || !w_packed || !u || !v || !mult || !corr || !y) return QCN_ERR_ARG;
  if (nimg <= 0 || h <= 0 || w <= 0 || cin <= 0 || cout <= 0 || kh <= 0 || kw <= 0 ||
      stride_h <= 0 || stride_w <= 0 || pad_h < 0 || pad_w < 0 || x_zp < 0 || x_zp > 255 ||
      y_zp < 0 || y_zp > 255)
    return QCN_ERR_ARG;
  if (resid && (!(y_scale > 0.f) || !(r_scale > 0.f) || !(out_scale > 0.f) || r_zp < 0 ||
                r_zp > 255 || out_zp < 0 || out_zp > 255 || relu))
    return QCN_ERR_ARG;
  if (cin % 32 != 0 || cout % 64 != 0) return QCN_ERR_UNSUPPORTED;
  const int oh = (h + 2 * pad_h - kh) / stride_h + 1, ow = (w + 2 * pad_w - kw) / stride_w + 1;
  if (oh <= 0 || ow <= 0) return QCN_ERR_ARG;
  qcn::GemmArgs a{};
  a.x = x; a.w = w_packed;
  a.n = nimg; a.h = h; a.w_ = w; a.cin = cin; a.oh = oh; a.ow = ow; a.cout = cout;
  a.kh = kh; a.kw = kw; a.sy = stride_h; a.sx = stride_w; a.py = pad_h; a.px = pad_w;
  a.x_zp = x_zp;
  a.npix = (long)nimg * oh * ow;
  a.kcs = kh * kw * (cin / 32);
  a.u = u; a.v = v; a.mult = mult; a.corr = corr;
  a.zp_y = y_zp; a.lo = relu ? y_zp : 0;
  a.r = resid; a.s3 = y_scale; a.s_r = r_scale; a.inv_o = resid ? 1.0f / out_scale : 0.f;
  a.z_r = r_zp; a.z_o = out_zp; a.y = y;
  if ((long)((a.npix + 255) / 256) * (cout / 64) >= (1L << 31)) return QCN_ERR_UNSUPPORTED;
  if (a.npix >= (1L << 31) - 256) return QCN_ERR_UNSUPPORTED;   // 32-bit pixel indices in the kernel
  hipStream_t st = (hipStream_t)stream;
  // thin 1x1 stride-1 convs (K = Cin <= 512) stream: ResNet-50 98.3-99.0 ->
  // 102.9-104.1 K img/s (K <= 256) and 104.0-105.4 -> 105.9-108.3 K (K <= 512)
  // on two boxes (profiles/r03_diag_resnet_stream_ab.txt)
  constexpr int stream_k = 512;
  if (cin <= stream_k && kh == 1 && kw == 1 && stride_h == 1 && stride_w == 1 && pad_h == 0 && pad_w == 0) {
    const int rc = resid ? qcn::dispatch_stream<true>(a, st) : qcn::dispatch_stream<false>(a, st);
    if (rc >= 0) return rc;
  }
  // whole-image 3x3 for the 14x14x256 and 7x7x512 maps.  Same box: layer-3
  // 3x3 0.101 -> 0.065 ms, layer-4 0.094 -> 0.073 ms, ResNet-50 108.6-109.3
  // -> 114.5-114.6 K img/s (profiles/r03_diag_resnet_img3_ab.txt)
  if (!resid && kh == 3 && kw == 3 && stride_h == 1 && stride_w == 1 && pad_h == 1 && pad_w == 1 &&
      h == w && cout % 256 == 0) {
    if (h == 14 && cin == 256) return qcn::launch_img<14, 256, 8, 1>(a, st);
    if (h == 7 && cin == 512) return qcn::launch_img<7, 512, 8, 1>(a, st);
  }
  // the stride-2 downsample 1x1 streams too
  if (cin <= stream_k && !resid && kh == 1 && kw == 1 && stride_h == 2 && stride_w == 2 &&
      pad_h == 0 && pad_w == 0) {
    const int rc = qcn::dispatch_stream_s2(a, st);
    if (rc >= 0) return rc;
  }
  // 256-channel tiles (8 waves; every gathered B row serves 256 output
  // channels) where they measured faster: the 3x3 convs and the deepest 1x1
  // (-5..8 %); the residual-join convs lose 30-40 % at one workgroup per CU
  // (profiles/r02_diag_resnet_bn256_layers.txt)
  if (cout % 256 == 0 && !resid && (kh * kw > 1 || cin >= 2048))
    return qcn::launch_gemm<256, false>(a, st);
  if (cout % 128 == 0)
    return resid ? qcn::launch_gemm<128, true>(a, st) : qcn::launch_gemm<128, false>(a, st);
  return resid ? qcn::launch_gemm<64, true>(a, st) : qcn::launch_gemm<64, false>(a, st);
}
