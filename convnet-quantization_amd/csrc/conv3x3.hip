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
#include "conv_epi.hpp"
#include <type_traits>
#include <utility>
#include <algorithm>
#include <cmath>
#include "qconvnet_abi.hpp"

namespace qcn {

// weight-prefetch depth (K-steps) of the 32x32 wave-specialised pair kernels;
// D + 1 must divide 18
constexpr int kPipeD = 2;
// K-step prefetch depth of the one-image conv5+6 (convnet_convs_sm_kernel)
constexpr int kSm56D = 4;
// conv12 producer waves' issue priority (swept: 1-3 within noise, 2 best;
// 0 is ~20 % slower, profiles/r01_diag_conv12_prio_sweep_v16.txt)
constexpr int kProdPrio = 2;

// Patch layout knobs (chosen per layer by an offline bank-conflict search so
// that every ds_read_b128 of an MFMA operand is conflict-free):
//   PSP  bytes of padding per staged pixel (pixel stride PS = CIN + PSP)
//   RPAD bytes of padding per staged row,  SPAD per staged image segment
//   SPLIT store even patch columns before odd ones (pooled layers read stride-2)
template <int CIN, int COUT, int HW, bool POOL, int WPX, int PSP = 16, int RPAD = 0,
          int SPAD = 0, bool SPLIT = false, int WI_ = 2, int JT_ = 4, int RB_ = 0>
struct ConvCfg {
  static constexpr int kCin = CIN, kCout = COUT;
  static constexpr bool kPool = POOL, kSplit = SPLIT;
  static constexpr int W = HW, H = HW;
  // wave tile: WI 32-channel blocks (64 or 128 couts) x 128 pixels.  WI = 4
  // reads 8 fragments per 16 MFMAs instead of 6 per 8 (LDS bytes per MFMA
  // -33 %) and holds 256 accumulators, so one wave per SIMD
  static constexpr int WI = WI_;
  // JT 32-pixel blocks per wave: 4 (128 pixels; pooled layers need the four
  // 2x2 quadrants) or 2 (64 pixels: row bands of the 56-wide ResNet maps)
  static constexpr int JT = JT_;
  static constexpr int MPS = JT * WI;            // MFMAs per K-step
  static constexpr int kWpx = WPX;               // waves along the pixels
  static constexpr int WCO = COUT / (32 * WI);   // waves along cout
  static constexpr int NWAVES = WCO * WPX;
  static constexpr int NT = NWAVES * 64;         // threads
  static constexpr int PXB = WPX * 32 * JT;      // output pixels per workgroup (pre-pool)
  static constexpr int OPX = POOL ? PXB / 4 : PXB;  // output pixels written
  static constexpr int IMG = H * W;
  // RB_ > 0: BAND tiles — RB_ consecutive rows of the flattened (image, row)
  // space, which may run across image boundaries; each image's part of the
  // band gets its own halo rows in the patch (BandAddr / stage_band), so any
  // H works without padded rows.  SEGS is then the most images a band touches.
  static constexpr bool kBand = RB_ > 0;
  static constexpr int SEGS = kBand ? 1 + (RB_ - 1 + H - 1) / H : (PXB >= IMG ? PXB / IMG : 1);
  static constexpr int R = kBand ? RB_ : (PXB >= IMG ? H : PXB / W);   // rows per segment (band)
  static constexpr int PS = CIN + PSP;
  static constexpr int PROWS = R + 2, PCOLS = W + 2;
  static constexpr int HALF = (PCOLS + 1) / 2;
  static constexpr int RS = PCOLS * PS + RPAD;
  static constexpr int SS = PROWS * RS + SPAD;
  static constexpr int PATCH = kBand ? (RB_ + 2 * SEGS) * RS : SEGS * SS;
  static constexpr int WBUF = COUT * 64;         // one K-chunk of weights (XOR-swizzled rows)
  static constexpr int NPC = WBUF / 1024;        // 1-KiB LDS-DMA pieces per chunk
  static constexpr int NG = (NPC + NWAVES - 1) / NWAVES;  // global_load_lds per wave per chunk (at most)
  static constexpr int NCH = 9 * CIN / 64;       // K chunks
  static constexpr int OS = COUT + 16;           // output staging row stride
  static constexpr int MAIN = PATCH + 3 * WBUF;  // patch + 3-deep weight ring
  static constexpr int OUT = OPX * OS;
  static constexpr int EPI = MAIN > OUT ? MAIN : OUT;  // u | v | mult (fp32 x COUT each)
  static constexpr int LDS = EPI + 12 * COUT;
  static_assert(CIN % 64 == 0 && COUT % (32 * WI) == 0, "channel multiples");
  // WI = 1 (32 couts x 128 pixels): the cout-split conv6 of small batches
  static_assert(WI == 1 || WI == 2 || WI == 4, "wave tile of 32, 64 or 128 couts");
  static_assert(PSP % 16 == 0 && RPAD % 16 == 0 && SPAD % 16 == 0, "16-B aligned layout");
  static_assert(PXB % W == 0, "workgroup covers whole rows");
  static_assert(kBand ? (PXB == RB_ * W && !POOL)
                      : (PXB >= IMG ? (PXB % IMG == 0) : (H % R == 0)), "rows tile the image");
  static_assert(!POOL || (R % 2 == 0), "pooled rows come in pairs");
  static_assert(NG >= 1 && WBUF % 1024 == 0, "weight ring split");
  // pooled tiles: the four 2x2 quadrants as four 32-pixel blocks (JT = 4), or
  // one 8x8 image on 64-pixel tiles (JT = 2, "lane-pooled"): block j holds the
  // column-parity-j quadrants, lanes 0-15 / 16-31 the two row parities of the
  // 16 pooled pixels, and the row max is a v_permlane16_swap
  static constexpr bool kLanePool = POOL && JT == 2;
  static_assert(!POOL || JT == 4 || (HW == 8 && WPX == 1 && !RB_), "pooled tiles are the four quadrants");
  static_assert(JT == 2 || JT == 4, "64- or 128-pixel wave tiles");
  static_assert(LDS <= 160 * 1024, "LDS budget");
  __device__ static constexpr int slot(int seg, int prow, int pcol) {
    const int cpos = SPLIT ? ((pcol & 1) * HALF + (pcol >> 1)) : pcol;
    return seg * SS + prow * RS + cpos * PS;
  }
};

// Requantize one 32(cout) x 32(pixel) accumulator tile (optionally the max of
// four quadrant tiles) and write it to the LDS output image [pixel][cout]:
// two rounds of v_permlane32_swap turn the MFMA layout (4 couts per register,
// lane halves interleaved every 4 couts) into 16 contiguous couts per lane,
// so each lane issues ONE conflict-free ds_write_b128.
// fp32 epilogue constants of the 16 output channels a lane owns in one
// 32-channel accumulator tile (channels co_base + 8g + 4hi + e).
struct EpiK {
  float u[16], v[16], m[16];
};
QCN_DEV EpiK load_epik(const ConvEpi& ep, int co_base, int hi) {
  EpiK k;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int co = co_base + 8 * g + 4 * hi;
    const float4 u4 = *reinterpret_cast<const float4*>(ep.u + co);
    const float4 v4 = *reinterpret_cast<const float4*>(ep.v + co);
    const float4 m4 = *reinterpret_cast<const float4*>(ep.mult + co);
    k.u[4 * g] = u4.x; k.u[4 * g + 1] = u4.y; k.u[4 * g + 2] = u4.z; k.u[4 * g + 3] = u4.w;
    k.v[4 * g] = v4.x; k.v[4 * g + 1] = v4.y; k.v[4 * g + 2] = v4.z; k.v[4 * g + 3] = v4.w;
    k.m[4 * g] = m4.x; k.m[4 * g + 1] = m4.y; k.m[4 * g + 2] = m4.z; k.m[4 * g + 3] = m4.w;
  }
  return k;
}

// Same constants from the workgroup's LDS copy (stage_epik): broadcast reads
// instead of per-tile global loads in the epilogue.
QCN_DEV EpiK load_epik_lds(const float* ek, int cout, int co_base, int hi) {
  EpiK k;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int co = co_base + 8 * g + 4 * hi;
    const float4 u4 = *reinterpret_cast<const float4*>(ek + co);
    const float4 v4 = *reinterpret_cast<const float4*>(ek + cout + co);
    const float4 m4 = *reinterpret_cast<const float4*>(ek + 2 * cout + co);
    k.u[4 * g] = u4.x; k.u[4 * g + 1] = u4.y; k.u[4 * g + 2] = u4.z; k.u[4 * g + 3] = u4.w;
    k.v[4 * g] = v4.x; k.v[4 * g + 1] = v4.y; k.v[4 * g + 2] = v4.z; k.v[4 * g + 3] = v4.w;
    k.m[4 * g] = m4.x; k.m[4 * g + 1] = m4.y; k.m[4 * g + 2] = m4.z; k.m[4 * g + 3] = m4.w;
  }
  return k;
}

// Copy u | v | mult (COUT floats each) into LDS at ek; called in the prologue
// so the loads overlap the patch staging (visible after the main loop's barriers).
template <int COUT, int NT>
QCN_DEV void stage_epik(const ConvEpi& ep, float* ek, int tid) {
  asm volatile("" : "+v"(tid));   // a fresh copy: no tid-derived offset held across phases
  for (int e = tid; e < 3 * COUT / 4; e += NT) {
    const int arr = e / (COUT / 4), o = (e % (COUT / 4)) * 4;
    const float* src = arr == 0 ? ep.u : (arr == 1 ? ep.v : ep.mult);
    *reinterpret_cast<float4*>(ek + arr * COUT + o) = *reinterpret_cast<const float4*>(src + o);
  }
}

// EM (epilogue mode) 1 — FAST: zp_y == 0, lo == 0 and no QDQ hand-off (every
// post-ReLU layer of the static net).  Then clamp(rne(ab) + zp, lo, 255) == v_cvt_pk_u8_f32(ab), which
// rounds half-to-even and saturates to [0, 255] (probed exhaustively on gfx950,
// tools/micro/cvt_probe.hip), and the fma / mul run as packed fp32 pairs:
// 3 VALU per element instead of 7 (the epilogue is VALU-issue bound).
// EM 2: the QDQ hand-off in its one-fma form (qdq == 2): 6 VALU per element
// instead of 15.  EM 0: the general requant (+ qdq_next_f).
template <int NQ, bool XORIN, int EM, bool D32 = false, bool GWT = false>
QCN_DEV void epilogue_tile_k(const v16i* accs, const EpiK& K, const ConvEpi& ep, int co_base,
                             int hi, uint8_t* orow, const uint8_t* wbase = nullptr, uint32_t woff = 0) {
  // accumulators already include the zero-point correction (acc_init_corr)
  uint32_t w[4];
  const float zpf = (float)ep.zp_y, lof = (float)ep.lo;
  const float z1f = (float)ep.z1, z2f = (float)ep.z2;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    uint32_t wd = 0;
    int a[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int rg = 4 * g + e;
      a[e] = accs[0][rg];
      if constexpr (NQ == 4) a[e] = max(max(a[e], accs[1][rg]), max(accs[2][rg], accs[3][rg]));
      if constexpr (NQ == 2) {   // lane-pooled tiles: column pair in registers, row pair across lanes l ^ 16
        a[e] = max(a[e], accs[1][rg]);
        const auto r = __builtin_amdgcn_permlane16_swap(a[e], a[e], false, false);
        a[e] = max((int)r[0], (int)r[1]);
      }
    }
    if constexpr (EM != 0) {
      // scalar fma / mul (built with -fno-slp-vectorize so they stay scalar):
      // packed fp32 issues slower beside a partner wave's MFMAs
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rg = 4 * g + e;
        float f = __builtin_fmaf(K.u[rg], K.v[rg], (float)a[e]);
        f = f * K.m[rg];
        if constexpr (EM == 2) f = qdq_aff_f(f, ep);
        wd = __builtin_amdgcn_cvt_pk_u8_f32(f, e, wd);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rg = 4 * g + e;
        float q = requant_f(a[e], K.u[rg], K.v[rg], K.m[rg], zpf, lof);
        if (ep.qdq) q = qdq_next_f(q, ep.s1, z1f, ep.inv2, z2f);
        wd = __builtin_amdgcn_cvt_pk_u8_f32(q, e, wd);
      }
    }
    w[g] = wd;
  }
  if constexpr (D32) {
    // the lane's 4-channel groups 8g + 4hi straight to their dwords of the
    // destination row (v_permlane32_swap costs ~25 cycles each)
    uint32_t* od = reinterpret_cast<uint32_t*>(orow + co_base) + hi;
#pragma unroll
    for (int g = 0; g < 4; ++g) od[2 * g] = XORIN ? xor80(w[g]) : w[g];
    return;
  }
  // low lanes: c0-3 | c8-11 | c16-19 | c24-27 ; high lanes: c4-7 | c12-15 | ...
  auto s01 = __builtin_amdgcn_permlane32_swap(w[0], w[1], false, false);
  auto s23 = __builtin_amdgcn_permlane32_swap(w[2], w[3], false, false);
  w[0] = s01[0]; w[1] = s01[1]; w[2] = s23[0]; w[3] = s23[1];
  auto s02 = __builtin_amdgcn_permlane32_swap(w[0], w[2], false, false);
  auto s13 = __builtin_amdgcn_permlane32_swap(w[1], w[3], false, false);
  w[0] = s02[0]; w[2] = s02[1]; w[1] = s13[0]; w[3] = s13[1];
  // now low lanes hold couts co_base + 0..15, high lanes co_base + 16..31
  if constexpr (XORIN) {  // destination is a conv input patch: store q - 128
#pragma unroll
    for (int g = 0; g < 4; ++g) w[g] = xor80(w[g]);
  }
  if constexpr (GWT)   // orow unused: global destination wr + woff (write-through)
    store_wt16(wt_rsrc(wbase), woff + co_base + 16 * hi, make_uint4(w[0], w[1], w[2], w[3]));
  else
    *reinterpret_cast<uint4*>(orow + co_base + 16 * hi) = make_uint4(w[0], w[1], w[2], w[3]);
}

template <int NQ, bool XORIN = false, bool D32 = false, bool GWT = false>
QCN_DEV void epilogue_tile_kf(const v16i* accs, const EpiK& K, const ConvEpi& ep, int co_base,
                              int hi, uint8_t* orow, const uint8_t* wbase = nullptr, uint32_t woff = 0) {
  if (epi_fast(ep)) epilogue_tile_k<NQ, XORIN, 1, D32, GWT>(accs, K, ep, co_base, hi, orow, wbase, woff);
  else if (ep.qdq == 2) epilogue_tile_k<NQ, XORIN, 2, D32, GWT>(accs, K, ep, co_base, hi, orow, wbase, woff);
  else epilogue_tile_k<NQ, XORIN, 0, D32, GWT>(accs, K, ep, co_base, hi, orow, wbase, woff);
}

template <int NQ, bool XORIN = false>
QCN_DEV void epilogue_tile(const v16i* accs, const ConvEpi& ep, int co_base, int hi,
                           uint8_t* orow) {
  epilogue_tile_kf<NQ, XORIN>(accs, load_epik(ep, co_base, hi), ep, co_base, hi, orow);
}

// Accumulator tile initialised with the zero-point correction
// corr[co] = (128 - zp_x) * sum_k w[co][k] of its 16 output channels, so the
// MFMA sum is the exact sum_k (q_x - zp_x) * w directly.
QCN_DEV v16i acc_init_corr(const int* __restrict__ corr, int co_base, int hi) {
  v16i a;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int4 c4 = *reinterpret_cast<const int4*>(corr + co_base + 8 * g + 4 * hi);
    a[4 * g + 0] = c4.x;
    a[4 * g + 1] = c4.y;
    a[4 * g + 2] = c4.z;
    a[4 * g + 3] = c4.w;
  }
  return a;
}

// Copy the staged [opx][cout] u8 tile (row stride OS) to its contiguous NHWC
// destination with 16-B coalesced stores (full cache lines, no partial writes).
// WT: write-through (the next launch reads it); plain stores otherwise.
template <int COUT, int OS, int NT, bool WT = true>
QCN_DEV void store_staged(const uint8_t* lds_out, int opx, uint8_t* dst, long valid_px, int tid,
                          int rstride = COUT) {
  constexpr int CPR = COUT / 16;
  const int total = opx * CPR;
  const wt_rsrc_t wr = wt_rsrc(dst);
  for (int e = tid; e < total; e += NT) {
    const int row = e / CPR, ch = e % CPR;
    if (row < valid_px) {
      const uint4 v = *reinterpret_cast<const uint4*>(lds_out + row * OS + ch * 16);
      if constexpr (WT) store_wt16(wr, (uint32_t)(row * rstride + ch * 16), v);
      else *reinterpret_cast<uint4*>(dst + row * rstride + ch * 16) = v;
    }
  }
}

// Per-lane B-operand (pixel) addressing shared by both main loops: the patch
// address of tap (r, s) is the tap-(0,0) address plus a per-(tap, j) constant —
// with the parity-split column order (pooled layers only) the column step
// depends on the pixel column's parity, which is (j & 1) for pooled tiles — so
// a fully unrolled K loop reads with immediate offsets and no address math.
template <class C>
struct PatchAddr {
  static_assert(!C::kSplit || C::kPool, "parity-split columns need pooled tiles");
  int base[C::JT];
  // y0: (band tiles) the image row of the band's first row
  QCN_DEV PatchAddr(int wp, int l32, int hi, int y0 = 0) {
#pragma unroll
    for (int j = 0; j < C::JT; ++j) {
      int seg, prow, pcol;
      if constexpr (C::kBand) {
        // band row i sits in patch row i + 2 seg + 1 (seg: images crossed
        // before it, each adding a bottom and a top halo row); base = tap (0, 0)
        const int m = (wp * C::JT + j) * 32 + l32;
        const int i = m / C::W;
        seg = (y0 + i) / C::H;
        base[j] = (i + 2 * seg) * C::RS + (m % C::W) * C::PS + hi * 16;
        continue;
      }
      if constexpr (C::kLanePool) {
        const int q = l32 & 15, rp = l32 >> 4;   // pooled pixel (4 x 4), row parity
        seg = 0;
        prow = 2 * (q >> 2) + rp;
        pcol = 2 * (q & 3) + j;
      } else if constexpr (C::kPool) {
        constexpr int PW = C::W / 2, PR = C::R / 2;
        const int q = wp * 32 + l32;
        seg = q / (PR * PW);
        prow = 2 * ((q / PW) % PR) + (j >> 1);
        pcol = 2 * (q % PW) + (j & 1);
      } else {
        const int m = (wp * C::JT + j) * 32 + l32;
        seg = m / (C::R * C::W);
        prow = (m / C::W) % C::R;
        pcol = m % C::W;
      }
      base[j] = C::slot(seg, prow, pcol) + hi * 16;
    }
  }
  static constexpr int delta(int tap, int j) {
    const int r = tap / 3, s = tap % 3;
    int dc = s;
    if (C::kSplit) dc = s == 0 ? 0 : (s == 2 ? 1 : ((j & 1) ? 1 - C::HALF : C::HALF));
    return r * C::RS + dc * C::PS;
  }
};

// Main MFMA loop over the 9 taps x CIN/64 K-chunks for a patch already staged
// in LDS (q - 128 bytes, layout C::slot).  Weights stream through a 3-deep
// LDS-DMA ring at wring.  Entered with all waves' patch writes issued (the
// caller's loads may still be in flight); returns with the ring drained and all
// waves past a barrier.
//
// Software pipeline over (chunk, kk) steps, fully unrolled: the fragments of
// step s+1 are read from LDS one per MFMA of step s (a burst of 6 reads ahead
// of the MFMAs measured 30 % slower, interleaved 8 %: tools/micro/mfma_lds.hip).
// Chunk ch+1's weights are needed from step (ch, 1) on, so that step waits for
// its DMA and passes the workgroup barrier first; the same barrier proves every
// wave has consumed chunk ch-1 (read during step (ch-1,0), used by step
// (ch-1,1)), so the DMA of ch+2 into that buffer is issued during that step.
template <class C>
QCN_DEV void conv_mainloop(const uint8_t* patch, uint8_t* wring, const int8_t* __restrict__ wpk,
                           const int* __restrict__ corr, int wave, int lane,
                           v16i (&acc)[C::WI][C::JT], int band_y0 = 0) {
  constexpr int JT = C::JT;
  constexpr int CB = C::kCin / 64;
  constexpr int WI = C::WI, MPS = C::MPS;
  const int wc = wave % C::WCO, wp = wave / C::WCO;
  const int l32 = lane & 31, hi = lane >> 5;
  // weight ring: K-chunk ch (64 input channels of one tap, all COUT rows
  // of 64 B) -> buffer ch % 3 by LDS-DMA (global_load_lds, 16 B per lane),
  // two chunks in flight.  Row r's 16-B slot c is stored at slot c ^ ((r>>2)&3)
  // (swizzle applied on the SOURCE address, the LDS image stays lane-linear)
  // so the A-operand ds_read_b128 of 16 consecutive rows is conflict-free.
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  auto issue_g = [&](int ch, int g) {
    if constexpr (C::NPC % C::NWAVES != 0)   // (wave-uniform) fewer pieces than waves in this round
      if (g * C::NWAVES + wave_u >= C::NPC) return;
    uint8_t* buf = wring + (ch % 3) * C::WBUF;
    const int8_t* base = wpk + (long)ch * C::WBUF;
    const int o = (g * C::NWAVES + wave_u) * 1024 + lane * 16;
    const int r = o >> 6, sl = (o >> 4) & 3;
    glds16(base + r * 64 + ((sl ^ ((r >> 2) & 3)) << 4), buf + (g * C::NWAVES + wave_u) * 1024);
  };
  const PatchAddr<C> pa(wp, l32, hi, band_y0);
  // A operand: row wc*32*WI + 32i + l32, 16-B slot (2kk + hi) ^ swizzle
  const int arow = wc * 32 * WI + l32;
  const int aswz = (arow >> 2) & 3;  // same for arow + 32i
  // the zero-point correction is the first K-step's C operand (no copies
  // into the JT accumulator tiles)
  v16i c0[WI];
#pragma unroll
  for (int i = 0; i < WI; ++i) c0[i] = acc_init_corr(corr, wc * 32 * WI + i * 32, hi);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // patch + corr loads retired
#pragma unroll
  for (int g = 0; g < C::NG; ++g) issue_g(0, g);
  if constexpr (C::NCH > 1) {
#pragma unroll
    for (int g = 0; g < C::NG; ++g) issue_g(1, g);
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(C::NG) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  const uint8_t* abase = wring + arow * 64;
  auto rd_a = [&](int ch, int kk, int i) {
    return *reinterpret_cast<const v4i*>(abase + (ch % 3) * C::WBUF + i * 32 * 64 +
                                         (((2 * kk + hi) ^ aswz) << 4));
  };
  auto rd_b = [&](int ch, int kk, int j) {
    const int tap = ch / CB, cb = ch % CB;
    return *reinterpret_cast<const v4i*>(patch + pa.base[j] + PatchAddr<C>::delta(tap, j) + cb * 64 +
                                         kk * 32);
  };
  // one step: MPS MFMAs on (fa, fb); reads of step (rch, rkk) into (fan, fbn)
  // interleaved one per MFMA; DMA pieces of chunk dch spread over the MFMAs
  auto step = [&](v4i (&fan)[WI], v4i (&fbn)[JT], int rch, int rkk, bool rd,
                  const v4i (&fa)[WI], const v4i (&fb)[JT], bool dma, int dch, bool first) {
#pragma unroll
    for (int m = 0; m < MPS; ++m) {
      if (rd) {
        // the WI + JT fragment reads of the next step, spread over the MPS
        // MFMAs (read r in slot r * MPS / NR; two share a slot when NR > MPS,
        // e.g. the 32-cout x 128-pixel tiles: 5 reads over 4 MFMAs)
        constexpr int NR = WI + JT;
#pragma unroll
        for (int r = 0; r < NR; ++r)
          if (r * MPS / NR == m) {
            if (r < WI) fan[r] = rd_a(rch, rkk, r);
            else fbn[r - WI] = rd_b(rch, rkk, r - WI);
          }
      }
      __builtin_amdgcn_sched_barrier(0);
      acc[m / JT][m % JT] = __builtin_amdgcn_mfma_i32_32x32x32_i8(
          fa[m / JT], fb[m % JT], first ? c0[m / JT] : acc[m / JT][m % JT], 0, 0, 0);
#pragma unroll
      for (int g = 0; g < C::NG; ++g)
        if (dma && m == (2 * g + 1) * MPS / (2 * C::NG)) {
          __builtin_amdgcn_sched_barrier(0);
          issue_g(dch, g);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
    // pin the step's MFMAs here: they are side-effect free, and IR sinking
    // could otherwise move them past the next barrier towards the epilogue
    // (the fragment registers then stay live, and spill, across the loop)
    if constexpr (WI == 2) {   // (WI = 4 keeps its accumulators in AGPRs)
#pragma unroll
      for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int j = 0; j < JT; ++j) asm volatile("" : "+v"(acc[i][j]));
    }
  };
  v4i fa0[WI], fb0[JT], fa1[WI], fb1[JT];
#pragma unroll
  for (int i = 0; i < WI; ++i) fa0[i] = rd_a(0, 0, i);
#pragma unroll
  for (int j = 0; j < JT; ++j) fb0[j] = rd_b(0, 0, j);
  // Stagger (8-wave workgroups): the second half of the waves (4-7, the
  // SIMD partners of 0-3, working on the other pixel half) passes each ring
  // barrier one K-step EARLIER in its program — before step (ch, 0) instead
  // of (ch, 1) — and issues chunk ch+2's DMA in step (ch, 0), so it runs one
  // K-step behind its partner and the two no longer reach their reads,
  // barrier waits and epilogues together (MI355X_MICROARCH 'two waves per
  // SIMD', item 9).  Hazards as before: barrier c still certifies chunk c
  // landed (every wave waited for its own pieces) and every wave done with
  // chunk c-2's buffer (the lagging half consumed its last fragments of it
  // in the step before the barrier); both halves pass NCH + 1 barriers.
  // Same-box conv5+6 51.4 -> 47.9 us (profiles/r02_diag_stagger_step_ab.txt);
  // a whole-chunk stagger measured slower (r02_diag_stagger_chunk_ab.txt).
  const bool lag = C::NWAVES >= 8 && wave_u >= C::NWAVES / 2;
  // the leading half issues first (s_setprio 1 for the loop): same-box
  // conv5+6 48.0 -> 47.6 us; the lagging half at priority 1 measured 48.7
  // (profiles/r02_diag_stagger_priority_ab.txt)
  if (C::NWAVES >= 8 && !lag) __builtin_amdgcn_s_setprio(1);
  auto ring_barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
#pragma unroll
  for (int ch = 0; ch < C::NCH; ++ch) {
    if (lag && ch + 1 < C::NCH) ring_barrier();
    // step (ch, 0): read (ch, 1), multiply (ch, 0)
    step(fa1, fb1, ch, 1, true, fa0, fb0, lag && ch + 2 < C::NCH, ch + 2, ch == 0);
    if (ch + 1 < C::NCH) {
      // step (ch, 1): chunk ch+1 landed and visible -> read (ch+1, 0), multiply (ch, 1)
      if (!lag) ring_barrier();   // chunk ch-1's reads stay before the barrier
      step(fa0, fb0, ch + 1, 0, true, fa1, fb1, !lag && ch + 2 < C::NCH, ch + 2, false);
    } else {
      step(fa0, fb0, 0, 0, false, fa1, fb1, false, 0, false);
    }
  }
  // every wave's last reads are consumed; the caller reuses the LDS
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  if (C::NWAVES >= 8) __builtin_amdgcn_s_setprio(0);
}

// Requantize the accumulators, stage [pixel][cout] in LDS (offset 0) and write
// the workgroup's contiguous NHWC output span with 16-B stores.
// Workgroup barrier (the default synchronisation of the conv bodies).
struct WgBar {
  QCN_DEV void operator()() const { __syncthreads(); }
};

// ch0 / cstride: the workgroup's couts are channels ch0 .. ch0 + COUT - 1 of
// an output with cstride channels per pixel (the cout-split conv6).
template <class C, bool WT = true, class Bar = WgBar>
QCN_DEV void conv_epilogue(v16i (&acc)[C::WI][C::JT], const ConvEpi& ep, uint8_t* lds, int nimg,
                           int wave, int lane, int tid, uint8_t* __restrict__ y, int tile,
                           const float* ek_override = nullptr, Bar&& bar = Bar{}, int ch0 = 0,
                           int cstride = C::kCout) {
  const int wc = wave % C::WCO, wp = wave / C::WCO;
  const int l32 = lane & 31, hi = lane >> 5;
  constexpr bool POOL = C::kPool;
  constexpr int COUT = C::kCout;
  uint8_t* lout = lds;  // the patch / weight ring is dead after the last barrier
  const float* ek = ek_override ? ek_override : reinterpret_cast<const float*>(lds + C::EPI);
#pragma unroll
  for (int i = 0; i < C::WI; ++i) {
    const int co_base = wc * 32 * C::WI + i * 32;
    const EpiK K = load_epik_lds(ek, COUT, co_base, hi);
    if constexpr (C::kLanePool) {   // lanes l32 and l32 ^ 16 hold the same pooled pixel
      epilogue_tile_kf<2>(acc[i], K, ep, co_base, hi, lout + (l32 & 15) * C::OS);
    } else if constexpr (POOL) {
      const int opx = wp * 32 + l32;
      epilogue_tile_kf<4>(acc[i], K, ep, co_base, hi, lout + opx * C::OS);
    } else {
#pragma unroll
      for (int j = 0; j < C::JT; ++j) {
        const int opx = (wp * C::JT + j) * 32 + l32;
        epilogue_tile_kf<1>(&acc[i][j], K, ep, co_base, hi, lout + opx * C::OS);
      }
    }
  }
  bar();
  const long out0 = (long)tile * C::OPX;
  const long total_out = POOL ? (long)nimg * C::IMG / 4 : (long)nimg * C::IMG;
  if (ep.kmajor) {
    // chunk-major for the classifier GEMM: 32-byte chunk kc of image n at
    // y + (kc * nimg + n) * 32.  The workgroup holds whole images, so the
    // IMGS images of one chunk form one contiguous run (IMGS * 32 bytes).
    constexpr int OPI = POOL ? C::IMG / 4 : C::IMG;   // output pixels per image
    constexpr int IMGS = C::OPX / OPI;
    if constexpr (IMGS >= 1 && C::OPX % OPI == 0) {
      constexpr int CC = COUT / 32;
      const int CCT = cstride / 32, cc0 = ch0 / 32;   // chunks per pixel of the whole output
      const int n0 = (int)(out0 / OPI);
      const wt_rsrc_t wr = wt_rsrc(y + (long)n0 * 32);   // offsets < 2^31: nimg * 4096 checked at launch
      for (int e = tid; e < OPI * CC * IMGS * 2; e += C::NT) {
        const int half = e & 1, img = (e >> 1) % IMGS, pc = (e >> 1) / IMGS;
        const int p = pc / CC, cc = pc % CC;
        if (n0 + img < nimg)
          store_wt16(wr, (uint32_t)(((p * CCT + cc0 + cc) * nimg + img) * 32 + half * 16),
                     *reinterpret_cast<const uint4*>(lout + (img * OPI + p) * C::OS + cc * 32 + half * 16));
      }
    }
    return;
  }
  store_staged<COUT, C::OS, C::NT, WT>(lout, C::OPX, y + out0 * cstride + ch0, total_out - out0, tid,
                                       cstride);
}

// Stage the input patch of the workgroup's tile (images n0.., first output row
// y0) in LDS: q ^ 0x80 = q - 128 as s8, halo = zp ^ 0x80.  Loads are issued in
// unconditional batches (halo / tail lanes read a valid dummy address and are
// replaced afterwards) so a thread keeps BATCH 16-B loads in flight instead of
// one dependent HBM round trip per element.
template <class C>
QCN_DEV void stage_patch(const uint8_t* __restrict__ x, int nimg, int x_zp, int n0, int y0,
                         uint8_t* patch, int tid) {
  constexpr int CIN = C::kCin;
  const uint32_t padw = xor80(splat_u8(x_zp));
  constexpr int CH16 = CIN / 16;
  constexpr int NSLOT = C::SEGS * C::PROWS * C::PCOLS;
  constexpr int TOTAL = NSLOT * CH16;
  constexpr int NITER = (TOTAL + C::NT - 1) / C::NT;
  constexpr int BATCH = NITER < 8 ? NITER : 8;
  for (int b0 = 0; b0 < NITER; b0 += BATCH) {
    uint4 v[BATCH];
    int dst[BATCH];
    bool inside[BATCH];
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      const int it = tid + (b0 + k) * C::NT;
      const int itc = it < TOTAL ? it : 0;
      const int sl = itc / CH16, chunk = itc % CH16;
      const int seg = sl / (C::PROWS * C::PCOLS);
      const int rem = sl % (C::PROWS * C::PCOLS);
      const int pr = rem / C::PCOLS, pc = rem % C::PCOLS;
      const int n = n0 + seg, yy = y0 + pr - 1, xx = pc - 1;
      inside[k] = n < nimg && yy >= 0 && yy < C::H && xx >= 0 && xx < C::W;
      dst[k] = (it < TOTAL && b0 + k < NITER) ? C::slot(seg, pr, pc) + chunk * 16 : -1;
      const long src = inside[k] ? (((long)n * C::H + yy) * C::W + xx) * CIN + chunk * 16 : 0;
      v[k] = *reinterpret_cast<const uint4*>(x + src);
    }
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      const uint4 val = inside[k] ? make_uint4(xor80(v[k].x), xor80(v[k].y), xor80(v[k].z), xor80(v[k].w))
                                  : make_uint4(padw, padw, padw, padw);
      if (dst[k] >= 0) *reinterpret_cast<uint4*>(patch + dst[k]) = val;
    }
  }

}

// Band tiles: the patch of RB flattened rows starting at image n0, row y0.
// Patch row pr belongs to segment k (the k-th image the band touches) when
// pr - 2k - 1 is one of that segment's band rows or its halo: image n0 + k,
// image row (k == 0 ? y0 : 0) + (pr - 2k - first_k) - 1, zero point outside.
template <class C>
QCN_DEV void stage_band(const uint8_t* __restrict__ x, int nimg, int x_zp, int n0, int y0,
                        uint8_t* patch, int tid) {
  constexpr int CIN = C::kCin, CH16 = CIN / 16;
  constexpr int PR = C::R + 2 * C::SEGS;
  constexpr int TOTAL = PR * C::PCOLS * CH16;
  constexpr int NITER = (TOTAL + C::NT - 1) / C::NT;
  constexpr int BATCH = NITER < 8 ? NITER : 8;
  const uint32_t padw = xor80(splat_u8(x_zp));
  const int first1 = C::H - y0;   // band rows of segment 0 (>= 1)
  for (int b0 = 0; b0 < NITER; b0 += BATCH) {
    uint4 v[BATCH];
    int dst[BATCH];
    bool inside[BATCH];
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      const int it = tid + (b0 + k) * C::NT;
      const int itc = it < TOTAL ? it : 0;
      const int sl = itc / CH16, chunk = itc % CH16;
      const int pr = sl / C::PCOLS, pc = sl % C::PCOLS;
      // segment of patch row pr: segment 0 holds patch rows [0, first1 + 2),
      // segment k >= 1 rows [first1 + 2 + (k - 1)(H + 2), ... + H + 2)
      int seg = 0, yy = y0 - 1 + pr;
      if (pr >= first1 + 2) {
        const int q = pr - first1 - 2;
        seg = 1 + q / (C::H + 2);
        yy = q % (C::H + 2) - 1;
      }
      const int n = n0 + seg, xx = pc - 1;
      // rows of the last segment past the band end read as padding (never used)
      inside[k] = n < nimg && yy >= 0 && yy < C::H && xx >= 0 && xx < C::W;
      dst[k] = (it < TOTAL && b0 + k < NITER) ? pr * C::RS + pc * C::PS + chunk * 16 : -1;
      const long src = inside[k] ? (((long)n * C::H + yy) * C::W + xx) * CIN + chunk * 16 : 0;
      v[k] = *reinterpret_cast<const uint4*>(x + src);
    }
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      const uint4 val = inside[k] ? make_uint4(xor80(v[k].x), xor80(v[k].y), xor80(v[k].z), xor80(v[k].w))
                                  : make_uint4(padw, padw, padw, padw);
      if (dst[k] >= 0) *reinterpret_cast<uint4*>(patch + dst[k]) = val;
    }
  }
}

template <int CIN, int COUT, int HW, bool POOL, int WPX, int PSP, int RPAD, int SPAD, bool SPLIT,
          int JT, int RB>
// JT = 2 (seven-wave 64-pixel tiles): two workgroups per CU need four waves on
// some SIMDs, so at most 128 VGPRs
__global__ __launch_bounds__(COUT * WPX, JT == 2 ? 4 : 2)
void conv3x3_u8s8_kernel(const uint8_t* __restrict__ x, int nimg, int x_zp,
                         const int8_t* __restrict__ wpk, ConvEpi ep,
                         uint8_t* __restrict__ y) {
  using C = ConvCfg<CIN, COUT, HW, POOL, WPX, PSP, RPAD, SPAD, SPLIT, 2, JT, RB>;
  static_assert(C::NT == COUT * WPX, "64-cout wave tiles");
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t* patch = lds;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;

  const long p0 = (long)blockIdx.x * C::PXB;         // first output pixel (pre-pool)
  const int n0 = (int)(p0 / C::IMG);
  const int y0 = (int)((p0 % C::IMG) / C::W);

  stage_epik<COUT, C::NT>(ep, reinterpret_cast<float*>(lds + C::EPI), tid);
  if constexpr (C::kBand) stage_band<C>(x, nimg, x_zp, n0, y0, patch, tid);
  else stage_patch<C>(x, nimg, x_zp, n0, y0, patch, tid);

  v16i acc[C::WI][C::JT];
  conv_mainloop<C>(patch, lds + C::PATCH, wpk, ep.corr, wave, lane, acc, C::kBand ? y0 : 0);
  conv_epilogue<C>(acc, ep, lds, nimg, wave, lane, tid, y, (int)blockIdx.x);
}

// --------------------------------------------------------------------------
// Two convolutions of one SimpleConvNet block in one launch: A (no pool) then
// B (2x2 pool), e.g. conv3 -> conv4 and conv5 -> conv6.  The workgroup tile is
// whole images for both, so A's output for the tile is exactly B's input
// patch: A's epilogue requantizes straight into B's swizzled LDS patch (as
// q - 128, plus B's zero-point halo) and B runs without touching HBM.  Saves
// A's output store, B's patch load and one lockstep prologue per tile.
template <class CA, class CB>
struct PairCfg {
  static_assert(!CA::kPool && CA::kCout == CB::kCin, "A feeds B");
  // (the wave tiles of A and B may differ — e.g. the 8-wave one-image conv3+4
  // of small batches: A 64 couts x 64 pixels, B 32 couts x 128 pixels)
  static_assert(CA::NT == CB::NT && CA::PXB == CB::PXB && CA::SEGS == CB::SEGS && CA::R == CB::R &&
                CA::W == CB::W && !CA::kBand && !CB::kBand, "same whole-image tiling");
  static constexpr int MAIN_A = CA::PATCH + 3 * CA::WBUF;
  static constexpr int MAIN_B = CB::PATCH + 3 * CB::WBUF;
  static constexpr int MAIN = MAIN_A > MAIN_B ? MAIN_A : MAIN_B;
  static constexpr int OUT_B = CB::OPX * CB::OS;
  static_assert(OUT_B <= MAIN, "B's staging fits the dead patch");
  // A's constants are dead once A's epilogue has run: park them in B's weight
  // ring when they fit there (B's ring is only written once B's loop starts)
  static constexpr bool EA_IN_RING = MAIN_A + 12 * CA::kCout <= MAIN_B && MAIN_A >= CB::PATCH;
  static constexpr int OFF_EA = EA_IN_RING ? MAIN_A : MAIN;
  static constexpr int OFF_EB = EA_IN_RING ? MAIN : MAIN + 12 * CA::kCout;
  static constexpr int LDS = OFF_EB + 12 * CB::kCout;
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// A's epilogue into B's LDS patch (zero-point halo, then the requantized
// interior as q - 128).  Shared by both pair bodies.
template <class CA, class CB>
QCN_DEV void pair_handoff(v16i (&acc)[CA::WI][CA::JT], const ConvEpi& epa, const float* eka, int xb_zp,
                          uint8_t* lds, int wave, int lane, int tid) {
  const uint32_t padw = xor80(splat_u8(xb_zp));
  const uint4 pad4 = make_uint4(padw, padw, padw, padw);
  constexpr int CH16 = CB::kCin / 16;
  constexpr int HALO = CB::SEGS * (2 * CB::PCOLS + 2 * (CB::PROWS - 2));
  for (int e = tid; e < HALO * CH16; e += CB::NT) {
    const int hs = e / CH16, chunk = e % CH16;
    const int seg = hs / (2 * CB::PCOLS + 2 * (CB::PROWS - 2));
    int r = hs % (2 * CB::PCOLS + 2 * (CB::PROWS - 2)), pr, pc;
    if (r < CB::PCOLS) { pr = 0; pc = r; }
    else if (r < 2 * CB::PCOLS) { pr = CB::PROWS - 1; pc = r - CB::PCOLS; }
    else { r -= 2 * CB::PCOLS; pr = 1 + (r >> 1); pc = (r & 1) ? CB::PCOLS - 1 : 0; }
    *reinterpret_cast<uint4*>(lds + CB::slot(seg, pr, pc) + chunk * 16) = pad4;
  }
  const int wc = wave % CA::WCO, wp = wave / CA::WCO;
  const int l32 = lane & 31, hi = lane >> 5;
#pragma unroll
  for (int i = 0; i < CA::WI; ++i) {
    const int co_base = wc * 32 * CA::WI + i * 32;
    const EpiK K = load_epik_lds(eka, CA::kCout, co_base, hi);
#pragma unroll
    for (int j = 0; j < CA::JT; ++j) {
      const int m = (wp * CA::JT + j) * 32 + l32;
      const int seg = m / (CA::R * CA::W), row = (m / CA::W) % CA::R, col = m % CA::W;
      epilogue_tile_kf<1, true, true>(&acc[i][j], K, epa, co_base, hi,
                                      lds + CB::slot(seg, row + 1, col + 1));
    }
  }
}

template <class CA, class CB>
QCN_DEV void convpair_body(int tile, const uint8_t* __restrict__ x, int nimg, int x_zp,
                           const int8_t* __restrict__ wa, ConvEpi epa, int xb_zp,
                           const int8_t* __restrict__ wb, ConvEpi epb,
                           uint8_t* __restrict__ y) {
  using P = PairCfg<CA, CB>;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  // laundered: no thread-id-derived address is hoisted and held live across
  // the two main loops
  int tid_l = threadIdx.x;
  asm volatile("" : "+v"(tid_l));
  const int tid = tid_l, lane = tid & 63, wave = tid >> 6;
  const long p0 = (long)tile * CA::PXB;
  const int n0 = (int)(p0 / CA::IMG);
  const int y0 = (int)((p0 % CA::IMG) / CA::W);
  float* eka = reinterpret_cast<float*>(lds + P::OFF_EA);
  float* ekb = reinterpret_cast<float*>(lds + P::OFF_EB);
  stage_epik<CA::kCout, CA::NT>(epa, eka, tid);
  stage_epik<CB::kCout, CB::NT>(epb, ekb, tid);
  stage_patch<CA>(x, nimg, x_zp, n0, y0, lds, tid);

  v16i acc[CA::WI][CA::JT];
  conv_mainloop<CA>(lds, lds + CA::PATCH, wa, epa.corr, wave, lane, acc);

  // A's epilogue into B's patch (A's patch and ring are dead past the main
  // loop's final barrier)
  pair_handoff<CA, CB>(acc, epa, eka, xb_zp, lds, wave, lane, tid);
  __syncthreads();
  if constexpr (CA::WI == CB::WI && CA::JT == CB::JT) {
    conv_mainloop<CB>(lds, lds + CB::PATCH, wb, epb.corr, wave, lane, acc);
    conv_epilogue<CB>(acc, epb, lds, nimg, wave, lane, tid, y, tile, ekb);
  } else {
    v16i accb[CB::WI][CB::JT];
    conv_mainloop<CB>(lds, lds + CB::PATCH, wb, epb.corr, wave, lane, accb);
    conv_epilogue<CB>(accb, epb, lds, nimg, wave, lane, tid, y, tile, ekb);
  }
}

template <class CA, class CB>
__global__ __launch_bounds__(CA::NT, CA::WI == 4 ? 1 : 2)
void convpair_kernel(const uint8_t* __restrict__ x, int nimg, int x_zp,
                     const int8_t* __restrict__ wa, ConvEpi epa, int xb_zp,
                     const int8_t* __restrict__ wb, ConvEpi epb, uint8_t* __restrict__ y) {
  convpair_body<CA, CB>((int)blockIdx.x, x, nimg, x_zp, wa, epa, xb_zp, wb, epb, y);
}

// --------------------------------------------------------------------------
// Weights straight from global memory (L2) into registers.  When a workgroup
// has one wave along the pixels (WPX = 1), every weight fragment is used by
// exactly ONE of its waves: an LDS ring would stage bytes that are read once,
// and its per-chunk barriers would hold the waves in lockstep.  Here each wave
// loads its own A fragments D K-steps ahead (buffer loads, the step's offset in
// the scalar operand) and the K loop has no barrier at all, so the LDS holds
// only the patch and two independent 4-wave workgroups fit on a CU: one
// workgroup's staging and epilogues run beside the other's MFMAs.
template <class C, int D>
struct GaFrag {
  v4i fa[D + 1][C::WI];
};

// Issue the A-fragment loads of K-step s (chunk s / 2, half kk = s % 2) into
// slot s % (D + 1).  wr: buffer resource of the packed weights; voff: this
// lane's row offset ((wc*32*WI + l32) * 64 + hi * 16).
// CST: bytes between consecutive K chunks of the packed weights (C::WBUF, or
// the whole layer's cout x 64 for a workgroup that owns a slice of the couts).
template <class C, int D, int CST = C::WBUF>
QCN_DEV void ga_issue(GaFrag<C, D>& g, wt_rsrc_t wr, int voff, int s) {
  const int ch = s >> 1, kk = s & 1;
#pragma unroll
  for (int i = 0; i < C::WI; ++i) {
    const auto t = __builtin_amdgcn_raw_buffer_load_b128(wr, voff, ch * CST + i * 32 * 64 + kk * 32, 0);
    g.fa[s % (D + 1)][i] = (v4i){(int)t[0], (int)t[1], (int)t[2], (int)t[3]};
  }
}

template <class C>
QCN_DEV int ga_voff(int wave, int lane) {
  return ((wave % C::WCO) * 32 * C::WI + (lane & 31)) * 64 + (lane >> 5) * 16;
}

// The first D K-steps' loads (issued early so their latency overlaps the
// patch staging or the previous conv's epilogue).
template <class C, int D, int CST = C::WBUF>
QCN_DEV void ga_prefetch(GaFrag<C, D>& g, const int8_t* __restrict__ wpk, int wave, int lane, int co0 = 0) {
  const wt_rsrc_t wr = wt_rsrc(wpk);
  const int voff = ga_voff<C>(wave, lane) + co0 * 64;
#pragma unroll
  for (int s = 0; s < D; ++s) ga_issue<C, D, CST>(g, wr, voff, s);
}

// K loop over the patch staged in LDS (layout C::slot, all waves' writes
// visible), A fragments from g (steps 0..D-1 already issued).  Returns after a
// workgroup barrier: every wave's patch reads are done and the caller may
// reuse the LDS.
template <class C, int D, int CST = C::WBUF, class Bar = WgBar>
QCN_DEV void conv_mainloop_ga(const uint8_t* patch, const int8_t* __restrict__ wpk,
                              const int* __restrict__ corr, int wave, int lane,
                              v16i (&acc)[C::WI][C::JT], GaFrag<C, D>& g, Bar&& bar = Bar{}, int co0 = 0) {
  constexpr int CB = C::kCin / 64;
  constexpr int WI = C::WI, JT = C::JT, MPS = C::MPS, S = 2 * C::NCH;
  static_assert(D >= 1 && D < S, "prefetch depth");
  const int wc = wave % C::WCO, wp = wave / C::WCO;
  const int l32 = lane & 31, hi = lane >> 5;
  const PatchAddr<C> pa(wp, l32, hi);
  const wt_rsrc_t wr = wt_rsrc(wpk);
  const int voff = ga_voff<C>(wave, lane) + co0 * 64;
  v16i c0[WI];   // the first K-step's C operand
#pragma unroll
  for (int i = 0; i < WI; ++i) c0[i] = acc_init_corr(corr, wc * 32 * WI + i * 32, hi);
  auto rd_b = [&](int s, int j) {
    const int ch = s >> 1, kk = s & 1;
    const int tap = ch / CB, cb = ch % CB;
    return *reinterpret_cast<const v4i*>(patch + pa.base[j] + PatchAddr<C>::delta(tap, j) + cb * 64 +
                                         kk * 32);
  };
  v4i fb[2][JT];
#pragma unroll
  for (int j = 0; j < JT; ++j) fb[0][j] = rd_b(0, j);
#pragma unroll
  for (int s = 0; s < S; ++s) {
#pragma unroll
    for (int m = 0; m < MPS; ++m) {
      // next step's JT B fragments spread over the step's MFMAs (every
      // other one when there are 2 JT), the A loads of step s + D mid-step
      constexpr int BSP = MPS / JT;
      if (s + 1 < S && m % BSP == 0) fb[(s + 1) & 1][m / BSP] = rd_b(s + 1, m / BSP);
      __builtin_amdgcn_sched_barrier(0);
      acc[m / JT][m % JT] = __builtin_amdgcn_mfma_i32_32x32x32_i8(
          g.fa[s % (D + 1)][m / JT], fb[s & 1][m % JT], s == 0 ? c0[m / JT] : acc[m / JT][m % JT], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (s + D < S && m == MPS / 2 - 1) {
        // slot (s + D) % (D + 1) == (s - 1) % (D + 1): consumed by step s - 1
        ga_issue<C, D, CST>(g, wr, voff, s + D);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (WI <= 2) {
#pragma unroll
      for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int j = 0; j < JT; ++j) asm volatile("" : "+v"(acc[i][j]));
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  bar();
}

// LDS plan of the direct-weight pair: A's patch and then B's patch at offset
// 0 (A's is dead once every wave is past A's loop), both convs' epilogue
// constants behind the larger patch; B's output staging reuses the patch.
template <class CA, class CB>
struct PairGaCfg {
  static_assert(!CA::kPool && CA::kCout == CB::kCin, "A feeds B");
  static_assert(CA::JT == CB::JT, "one wave-tile width for both convs (128 or 64 pixels)");
  // (B may own a slice of the couts with a narrower wave tile: the patch
  // layout depends only on B's input side)
  static_assert(CA::NT == CB::NT && CA::PXB == CB::PXB && CA::SEGS == CB::SEGS && CA::R == CB::R &&
                CA::W == CB::W, "same whole-image tiling");
  static constexpr int PATCH = CA::PATCH > CB::PATCH ? CA::PATCH : CB::PATCH;
  static_assert(CB::OPX * CB::OS <= PATCH, "B's staging fits the dead patch");
  static constexpr int OFF_EA = PATCH;
  static constexpr int OFF_EB = OFF_EA + 12 * CA::kCout;
  static constexpr int LDS = OFF_EB + 12 * CB::kCout;
  static_assert(LDS <= (CA::NT >= 512 ? 160 : 80) * 1024, "two 4-wave or one 8-wave workgroup per CU");
};

// One tile (CA::PXB pixels of whole images) through A then B, weights from
// L2.  lb: this tile's LDS patch region (PairGaCfg<CA, CB>::PATCH bytes; B's
// output staging reuses it); eka / ekb: both convs' epilogue constants in
// LDS; tid: thread index within the CA::NT threads that run the tile; bar:
// their barrier.
template <class CA, class CB, int D, class Bar>
QCN_DEV void convpair_ga_tile(int tile, const uint8_t* __restrict__ x, int nimg, int x_zp,
                              const int8_t* __restrict__ wa, const ConvEpi& epa, int xb_zp,
                              const int8_t* __restrict__ wb, const ConvEpi& epb,
                              uint8_t* __restrict__ y, uint8_t* lb, const float* eka,
                              const float* ekb, int tid, Bar& bar) {
  const int lane = tid & 63, wave = tid >> 6;
  const long p0 = (long)tile * CA::PXB;
  const int n0 = (int)(p0 / CA::IMG);
  const int y0 = (int)((p0 % CA::IMG) / CA::W);
  GaFrag<CA, D> ga;
  ga_prefetch<CA, D>(ga, wa, wave, lane);
  stage_patch<CA>(x, nimg, x_zp, n0, y0, lb, tid);
  bar();
  v16i acc[CA::WI][CA::JT];
  conv_mainloop_ga<CA, D>(lb, wa, epa.corr, wave, lane, acc, ga, bar);
  GaFrag<CB, D> gb;
  ga_prefetch<CB, D>(gb, wb, wave, lane);   // B's first loads ride under A's epilogue
  pair_handoff<CA, CB>(acc, epa, eka, xb_zp, lb, wave, lane, tid);
  bar();
  conv_mainloop_ga<CB, D>(lb, wb, epb.corr, wave, lane, acc, gb, bar);
  conv_epilogue<CB, true>(acc, epb, lb, nimg, wave, lane, tid, y, tile, ekb, bar);
}

template <class CA, class CB, int D>
QCN_DEV void convpair_ga_body(int tile, const uint8_t* __restrict__ x, int nimg, int x_zp,
                              const int8_t* __restrict__ wa, ConvEpi epa, int xb_zp,
                              const int8_t* __restrict__ wb, ConvEpi epb, uint8_t* __restrict__ y) {
  using P = PairGaCfg<CA, CB>;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  // laundered: no thread-id-derived address is hoisted and held live across
  // the two main loops
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  float* eka = reinterpret_cast<float*>(lds + P::OFF_EA);
  float* ekb = reinterpret_cast<float*>(lds + P::OFF_EB);
  stage_epik<CA::kCout, CA::NT>(epa, eka, tid);
  stage_epik<CB::kCout, CB::NT>(epb, ekb, tid);
  WgBar bar;
  convpair_ga_tile<CA, CB, D>(tile, x, nimg, x_zp, wa, epa, xb_zp, wb, epb, y, lds, eka, ekb, tid, bar);
}

template <class CA, class CB, int D>
__global__ __launch_bounds__(CA::NT, CA::NT >= 512 ? 1 : 2)
void convpair_ga_kernel(const uint8_t* __restrict__ x, int nimg, int x_zp,
                        const int8_t* __restrict__ wa, ConvEpi epa, int xb_zp,
                        const int8_t* __restrict__ wb, ConvEpi epb, uint8_t* __restrict__ y) {
  convpair_ga_body<CA, CB, D>((int)blockIdx.x, x, nimg, x_zp, wa, epa, xb_zp, wb, epb, y);
}

// --------------------------------------------------------------------------
// Small batches (config 2, batch 256: 128 two-image workgroups on 256 CUs):
// workgroup 2t + h owns images 2t, 2t+1 and conv B's output channels
// [h * CB::kCout, (h + 1) * CB::kCout) of a COUTB-channel layer.  Each of the
// two computes conv A in full (B's input patch needs all of A's channels), so
// the pair costs 4/3 of the MFMAs in twice the workgroups.  B's wave tile is
// narrower (CB::WI) so four waves still cover the slice.
template <class CA, class CB, int D, int COUTB>
QCN_DEV void convpair_ga_split_body(int blk, const uint8_t* __restrict__ x, int nimg, int x_zp,
                                    const int8_t* __restrict__ wa, ConvEpi epa, int xb_zp,
                                    const int8_t* __restrict__ wb, ConvEpi epb, uint8_t* __restrict__ y) {
  using P = PairGaCfg<CA, CB>;
  static_assert(COUTB % CB::kCout == 0 && CA::NWAVES == CB::NWAVES, "cout slices");
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NS = COUTB / CB::kCout;
  const int tile = blk / NS, co0 = (blk % NS) * CB::kCout;
  ConvEpi eph = epb;   // this slice's constants
  eph.u += co0; eph.v += co0; eph.mult += co0; eph.corr += co0;
  float* eka = reinterpret_cast<float*>(lds + P::OFF_EA);
  float* ekb = reinterpret_cast<float*>(lds + P::OFF_EB);
  stage_epik<CA::kCout, CA::NT>(epa, eka, tid);
  stage_epik<CB::kCout, CB::NT>(eph, ekb, tid);
  const long p0 = (long)tile * CA::PXB;
  const int n0 = (int)(p0 / CA::IMG);
  const int y0 = (int)((p0 % CA::IMG) / CA::W);
  GaFrag<CA, D> ga;
  ga_prefetch<CA, D>(ga, wa, wave, lane);
  stage_patch<CA>(x, nimg, x_zp, n0, y0, lds, tid);
  __syncthreads();
  v16i acc[CA::WI][4];
  conv_mainloop_ga<CA, D>(lds, wa, epa.corr, wave, lane, acc, ga);
  constexpr int CSTB = COUTB * 64;
  GaFrag<CB, D> gb;
  ga_prefetch<CB, D, CSTB>(gb, wb, wave, lane, co0);
  pair_handoff<CA, CB>(acc, epa, eka, xb_zp, lds, wave, lane, tid);
  __syncthreads();
  v16i accb[CB::WI][4];
  conv_mainloop_ga<CB, D, CSTB>(lds, wb, eph.corr, wave, lane, accb, gb, WgBar{}, co0);
  conv_epilogue<CB, true>(accb, eph, lds, nimg, wave, lane, tid, y, tile, ekb, WgBar{}, co0, COUTB);
}

template <class CA, class CB, int D, int COUTB>
__global__ __launch_bounds__(CA::NT, 2)
void convpair_ga_split_kernel(const uint8_t* __restrict__ x, int nimg, int x_zp,
                              const int8_t* __restrict__ wa, ConvEpi epa, int xb_zp,
                              const int8_t* __restrict__ wb, ConvEpi epb, uint8_t* __restrict__ y) {
  convpair_ga_split_body<CA, CB, D, COUTB>((int)blockIdx.x, x, nimg, x_zp, wa, epa, xb_zp, wb, epb, y);
}

// One conv of the pipeline over a staged patch: 2 * C::NCH K-steps of 8
// MFMAs (64 couts x 128 pixels per wave), A fragments from registers (ga,
// steps 0..D-1 already in flight), B fragments from the patch; fill(k) runs
// after MFMA k.  Loads for the next job's first D steps come from wrn.
template <class C, int D, bool PIN = false, class Fill>
QCN_DEV void pipe_job(const uint8_t* patch, const int* corr, wt_rsrc_t wr, wt_rsrc_t wrn, int voff, int wc,
                      int wp, int l32, int hi, v16i (&acc)[2][4], v4i (&ga)[D + 1][2], Fill&& fill) {
  constexpr int CBK = C::kCin / 64, S = 2 * C::NCH;
  const PatchAddr<C> pa(wp, l32, hi);
  v16i c0[2];   // the first K-step's C operand: the zero-point correction
#pragma unroll
  for (int i = 0; i < 2; ++i) c0[i] = acc_init_corr(corr, wc * 64 + i * 32, hi);
  auto rd_b = [&](int s, int j) {
    const int ch = s >> 1, kk = s & 1;
    const int tap = ch / CBK, cb = ch % CBK;
    return *reinterpret_cast<const v4i*>(patch + pa.base[j] + PatchAddr<C>::delta(tap, j) + cb * 64 + kk * 32);
  };
  auto issue = [&](wt_rsrc_t r, int t, int slot) {
    const int ch = t >> 1, kk = t & 1;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, ch * C::WBUF + i * 32 * 64 + kk * 32, 0);
      ga[slot][i] = (v4i){(int)v[0], (int)v[1], (int)v[2], (int)v[3]};
    }
  };
  v4i fb[2][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) fb[0][j] = rd_b(0, j);
  static_for<S>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    static_for<8>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      if constexpr (s + 1 < S && (m & 1) == 0) fb[(s + 1) & 1][m >> 1] = rd_b(s + 1, m >> 1);
      __builtin_amdgcn_sched_barrier(0);
      acc[m >> 2][m & 3] = __builtin_amdgcn_mfma_i32_32x32x32_i8(ga[s % (D + 1)][m >> 2], fb[s & 1][m & 3],
                                                                 s == 0 ? c0[m >> 2] : acc[m >> 2][m & 3], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (m == 3) {
        // slot (s + D) % (D + 1) == (s - 1) % (D + 1): consumed by step s - 1
        constexpr int t = s + D;
        if constexpr (t < S) issue(wr, t, t % (D + 1));
        else issue(wrn, t - S, t % (D + 1));
        __builtin_amdgcn_sched_barrier(0);
      }
      fill(std::integral_constant<int, s * 8 + m>{});
      __builtin_amdgcn_sched_barrier(0);
    });
    // pin the step's MFMAs here (as conv_mainloop): side-effect free, they
    // could otherwise be sunk towards their uses and the fragment registers
    // held live (spilled) across the loop.  Only for accumulators that live
    // in VGPRs (two waves per SIMD): the pin would copy AGPR accumulators.
    if constexpr (PIN) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(acc[i][j]));
    }
  });
}

#ifdef QCN_PIPE34_STAMP
// Diagnostic builds only (tools/build_variant.sh): per-workgroup s_memtime
// stamps of wave 0 around every pipeline barrier, [wg][stamp]; plain vector
// stores into a buffer nothing else reads.
__device__ unsigned long long g_p34_stamp[2][1024][64];   // [conv3+4, conv5+6]
QCN_DEV void p34_stamp(int kind, int& idx, unsigned long long t) {
  const unsigned lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if (threadIdx.x < 64 && lane == 0 && blockIdx.x < 1024 && idx < 64) {
    volatile unsigned long long* d = &g_p34_stamp[kind][blockIdx.x][idx];
    *d = t + lane;
  }
  ++idx;
}
#define P34_STAMP() p34_stamp(stamp_kind, stamp_i, __builtin_amdgcn_s_memtime())
#else
#define P34_STAMP()
#endif

// --------------------------------------------------------------------------
// Two convolutions of a block with wave-specialised roles (persistent; the
// headline's conv3+conv4 and conv5+conv6 at batch 1024).  One 8-wave
// workgroup per CU: waves 0-3 run conv A, waves 4-7 conv B, so every SIMD
// holds one wave of each role (a workgroup's waves go to the SIMDs
// cyclically).  The workgroup takes tiles b, b + G, ... (a tile = CA::PXB
// pixels of whole images: one 16x16 image for conv3+4, two 8x8 images for
// conv5+6).  In period p (one workgroup barrier per period):
//
//   A waves:  conv A(p) -> acc, then A's epilogue of tile p into B's patch
//             buffer p & 1, and tile p + 1's input staged (loads issued
//             before the epilogue);
//   B waves:  B's pooled epilogue of tile p - 2 (acc), then conv B(p - 1) ->
//             acc from B's patch buffer (p - 1) & 1.
//
// Each role's VALU epilogue runs beside the other role's MFMAs on the same
// SIMD, at a fixed phase (B's at the period start, A's at its end), instead
// of wherever two independent workgroups happen to drift.  Weights stream
// from L2 into registers D K-steps ahead; the last D steps of a job prefetch
// the next period's first D.  LDS: B's patch double-buffered, A's patch
// double-buffered when it fits (conv3+4), else single with the staged input
// held in registers and written after the period barrier behind a second
// barrier (conv5+6); halos written once per launch; epilogue constants and
// corr tables.
template <class CA, class CB, int D>
struct PairWs {
  static_assert(CA::NWAVES == 4 && CB::NWAVES == 4 && CA::WCO == CB::WCO && CA::WI == 2 && CB::WI == 2 &&
                CA::JT == 4 && CB::JT == 4, "four waves of 64-cout x 128-pixel tiles per role");
  static_assert(!CA::kPool && CB::kPool && CA::kCout == CB::kCin, "A feeds B");
  static_assert(CA::PXB == CB::PXB && CA::SEGS == CB::SEGS && CA::R == CA::H && CA::W == CB::W &&
                !CA::kBand && !CB::kBand, "whole images per tile");
  static_assert(!CA::kSplit && CA::WBUF % 2048 == 0 && CB::WBUF % 2048 == 0, "weight layouts");
  static constexpr int SEGS = CA::SEGS, IMG = CA::IMG;
  static constexpr int IN_BYTES = SEGS * IMG * CA::kCin;   // a tile's input
  static_assert(IN_BYTES == 4 * 256 * 16, "four 16-B staging pieces per A-role thread");
  static constexpr int SA = 2 * CA::NCH, SB = 2 * CB::NCH;   // K-steps per job
  static_assert(SA % (D + 1) == 0 && SB % (D + 1) == 0, "every job starts at register slot 0");
  static constexpr int PA = (CA::PATCH + 15) / 16 * 16, PB = (CB::PATCH + 15) / 16 * 16;
  static constexpr int TAB = 16 * (CA::kCout + CB::kCout);   // u | v | mult | corr of both
  static constexpr bool DOUBLE_A = 2 * PA + 2 * PB + TAB <= 160 * 1024;
  static constexpr int OFF_PB = 0;
  static constexpr int OFF_PA = 2 * PB;
  static constexpr int OFF_EA = OFF_PA + (DOUBLE_A ? 2 : 1) * PA;   // u | v | mult, fp32 x cout each
  static constexpr int OFF_EB = OFF_EA + 12 * CA::kCout;
  static constexpr int OFF_CA = OFF_EB + 12 * CB::kCout;            // corr, int32 x cout
  static constexpr int OFF_CB = OFF_CA + 4 * CA::kCout;
  static constexpr int LDS = OFF_CB + 4 * CB::kCout;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static constexpr int OPI = CB::OPX / SEGS;   // pooled output pixels per image
};

// Workgroup b of G: its tiles are k = 0 .. T-1.  Image of segment s of tile k:
// (b + k G) SEGS + s (ILV = false: tile b + k G of the batch), or
// b + (k SEGS + s) G (ILV = true: the images b, b + G, b + 2G, ... that the
// earlier phases of the one-launch kernel gave this workgroup, paired up).
template <class CA, class CB, int D, int FA, int FB, bool KMAJOR, bool ILV = false>
QCN_DEV void convpair_ws_body(int b, int G, const uint8_t* __restrict__ x, int nimg, int x_zp,
                              const int8_t* __restrict__ wa, const ConvEpi& epa, int xb_zp,
                              const int8_t* __restrict__ wb, const ConvEpi& epb, uint8_t* __restrict__ y) {
  using P = PairWs<CA, CB, D>;
  constexpr int SEGS = P::SEGS, IMG = CA::IMG, W = CA::W, WCO = CA::WCO;
  constexpr int CH16 = CA::kCin / 16;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x;
  const int role = __builtin_amdgcn_readfirstlane(tid >> 8);   // 0: conv A, 1: conv B
  const int rt = tid & 255, lane = tid & 63, wave = rt >> 6;   // thread / wave within the role
  const int wc = wave % WCO, wp = wave / WCO;
  int T;
  if constexpr (ILV) {
    const int mine = b < nimg ? (nimg - 1 - b) / G + 1 : 0;   // images b, b + G, ...
    T = (mine + SEGS - 1) / SEGS;
  } else {
    const int ntile = (nimg + SEGS - 1) / SEGS;
    T = b < ntile ? (ntile - 1 - b) / G + 1 : 0;   // this workgroup's tiles b, b + G, ...
  }
  auto img_of = [&](int k, int sg) { return ILV ? b + (k * SEGS + sg) * G : (b + k * G) * SEGS + sg; };
#ifdef QCN_PIPE34_STAMP
  int stamp_i = 0;
  constexpr int stamp_kind = CA::kCin == 64 ? 0 : 1;
  if (threadIdx.x < 64) p34_stamp(stamp_kind, stamp_i, __builtin_amdgcn_s_memrealtime());
#endif
  P34_STAMP();
  // tile k's input piece q of this A-role thread (a phantom segment of a
  // ragged last tile reads the tile's first image, which this workgroup owns:
  // its outputs are never stored, and no other workgroup's bytes are read)
  auto in_src = [&](int k, int q) {
    const int p = rt + 256 * q;
    int n = img_of(k, p / (IMG * CH16));
    n = n < nimg ? n : img_of(k, 0);
    return x + ((long)n * IMG + (p / CH16) % IMG) * CA::kCin + (p % CH16) * 16;
  };
  auto in_dst = [&](int q) {
    const int p = rt + 256 * q;
    const int pix = (p / CH16) % IMG;
    return CA::slot(p / (IMG * CH16), pix / W + 1, pix % W + 1) + (p % CH16) * 16;
  };
  // tile b's input (A waves): loads first, their latency under the set-up below
  uint4 sv[4];
  if (role == 0 && T > 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) sv[q] = *reinterpret_cast<const uint4*>(in_src(0, q));
  }
  float* eka = reinterpret_cast<float*>(lds + P::OFF_EA);
  float* ekb = reinterpret_cast<float*>(lds + P::OFF_EB);
  int* cra = reinterpret_cast<int*>(lds + P::OFF_CA);
  int* crb = reinterpret_cast<int*>(lds + P::OFF_CB);
  // the epilogue tables (u | v | mult of both convs, both corr) in 16-B
  // pieces over the B-role threads, loaded now and written after the halos
  constexpr int NA = 3 * CA::kCout / 4, NB = 3 * CB::kCout / 4;       // float4 pieces
  constexpr int NCA = CA::kCout / 4, NCB = CB::kCout / 4;
  constexpr int NTAB = NA + NB + NCA + NCB, TPT = (NTAB + 255) / 256;
  float4 tval[TPT];
  auto tab = [&](int e, bool dst) -> float4* {
    if (e < NA) {
      const int a = e / (CA::kCout / 4), o = e % (CA::kCout / 4);
      const float* s = a == 0 ? epa.u : (a == 1 ? epa.v : epa.mult);
      return dst ? reinterpret_cast<float4*>(eka) + e : const_cast<float4*>(reinterpret_cast<const float4*>(s) + o);
    }
    e -= NA;
    if (e < NB) {
      const int a = e / (CB::kCout / 4), o = e % (CB::kCout / 4);
      const float* s = a == 0 ? epb.u : (a == 1 ? epb.v : epb.mult);
      return dst ? reinterpret_cast<float4*>(ekb) + e : const_cast<float4*>(reinterpret_cast<const float4*>(s) + o);
    }
    e -= NB;
    if (e < NCA)
      return dst ? reinterpret_cast<float4*>(cra) + e
                 : const_cast<float4*>(reinterpret_cast<const float4*>(epa.corr) + e);
    e -= NCA;
    return dst ? reinterpret_cast<float4*>(crb) + e
               : const_cast<float4*>(reinterpret_cast<const float4*>(epb.corr) + e);
  };
  if (role == 1) {
#pragma unroll
    for (int k = 0; k < TPT; ++k)
      if (rt + 256 * k < NTAB) tval[k] = *tab(rt + 256 * k, false);
  }
  {  // zero-point halos of every buffer of both patches (never overwritten)
    const uint32_t pa4 = xor80(splat_u8(x_zp)), pb4 = xor80(splat_u8(xb_zp));
    auto halo = [&](auto cfg, uint8_t* base, int nbuf, int pbytes, uint32_t pad) {
      using C = decltype(cfg);
      constexpr int HS = 2 * C::PCOLS + 2 * (C::PROWS - 2), CH = C::kCin / 16;
      const int total = nbuf * C::SEGS * HS * CH;
      for (int e = tid; e < total; e += 512) {
        const int c = e % CH, hs = (e / CH) % HS, sg = (e / (CH * HS)) % C::SEGS, bf = e / (CH * HS * C::SEGS);
        int pr, pc;
        if (hs < C::PCOLS) { pr = 0; pc = hs; }
        else if (hs < 2 * C::PCOLS) { pr = C::PROWS - 1; pc = hs - C::PCOLS; }
        else { const int r = hs - 2 * C::PCOLS; pr = 1 + (r >> 1); pc = (r & 1) ? C::PCOLS - 1 : 0; }
        *reinterpret_cast<uint4*>(base + bf * pbytes + C::slot(sg, pr, pc) + c * 16) = make_uint4(pad, pad, pad, pad);
      }
    };
    halo(CA{}, lds + P::OFF_PA, P::DOUBLE_A ? 2 : 1, P::PA, pa4);
    halo(CB{}, lds + P::OFF_PB, 2, P::PB, pb4);
  }
  if (role == 1) {
#pragma unroll
    for (int k = 0; k < TPT; ++k)
      if (rt + 256 * k < NTAB) *tab(rt + 256 * k, true) = tval[k];
  }
  if (T == 0) return;   // (uniform; the launcher never makes such a workgroup)

  const int l32 = lane & 31, hi = lane >> 5;
  const wt_rsrc_t wra = wt_rsrc(wa), wrb = wt_rsrc(wb);
  const int voff = (wc * 64 + l32) * 64 + hi * 16;
  auto pa_buf = [&](int j) { return lds + P::OFF_PA + (P::DOUBLE_A ? (j & 1) * P::PA : 0); };
  auto pb_buf = [&](int j) { return lds + P::OFF_PB + (j & 1) * P::PB; };
  auto write_in = [&](uint8_t* pa) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<uint4*>(pa + in_dst(q)) =
          make_uint4(xor80(sv[q].x), xor80(sv[q].y), xor80(sv[q].z), xor80(sv[q].w));
  };

  v16i acc[2][4];
  v4i ga[D + 1][2];
  {
    const wt_rsrc_t w0 = role == 0 ? wra : wrb;
    constexpr int CST = CA::WBUF;
    static_assert(CA::WBUF == CB::WBUF || true, "");
#pragma unroll
    for (int t = 0; t < D; ++t) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int cst = role == 0 ? CA::WBUF : CB::WBUF;
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(w0, voff, (t >> 1) * cst + i * 2048 + (t & 1) * 32, 0);
        ga[t][i] = (v4i){(int)v[0], (int)v[1], (int)v[2], (int)v[3]};
      }
    }
    (void)CST;
  }
  if (role == 0) write_in(pa_buf(0));
  P34_STAMP();
  lds_barrier();
  P34_STAMP();

  // lane-derived epilogue addressing from a laundered lane id (not hoisted
  // out of the period loop and held live across the MFMA jobs)
  struct Lane {
    int l32, hi, ek;
    int hb[4];          // B-patch offset of A's output pixel (wp * 4 + jj) * 32 + l32
    int q;              // pooled output pixel of B within the tile
    const int *ca, *cb;
  };
  auto lanes = [&]() {
    int lz = lane;
    asm volatile("" : "+v"(lz));
    Lane L;
    L.l32 = lz & 31;
    L.hi = lz >> 5;
    L.ek = wc * 64 + 4 * L.hi;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int m = (wp * 4 + jj) * 32 + L.l32;
      const int pix = m % IMG;
      L.hb[jj] = CB::slot(m / IMG, pix / W + 1, pix % W + 1) + wc * 64 + 4 * L.hi;
    }
    L.q = wp * 32 + L.l32;
    L.ca = cra + (lz >> 6);   // (lz >> 6 == 0: an address the compiler cannot hoist)
    L.cb = crb + (lz >> 6);
    return L;
  };
  // A's epilogue of acc into B's patch pb (epilogue_tile_k's numerics).  The
  // constants of a 32-channel tile row (4 groups of 4 channels) are read from
  // LDS together: one LDS round trip per tile row.
  auto epi_a = [&](const Lane& L, uint8_t* pb) {
    static_for<2>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      EpiG K[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) K[g] = load_epig(eka, CA::kCout, L.ek + i * 32 + 8 * g);
      static_for<16>([&](auto qc) {   // (tile jj, group g): one dword of 4 channels
        constexpr int jj = decltype(qc)::value >> 2, g = decltype(qc)::value & 3;
        uint32_t wd = 0;
#pragma unroll
        for (int ee = 0; ee < 4; ++ee) wd = rq_elem<FA>(acc[i][jj][4 * g + ee], K[g], ee, epa, wd);
        *reinterpret_cast<uint32_t*>(pb + L.hb[jj] + i * 32 + 8 * g) = xor80(wd);
      });
    });
  };
  // B's pooled epilogue of acc for tile t (max over the four quadrant tiles,
  // requant, two permlane32 swap rounds, one 16-B store per tile row and lane)
  auto epi_b = [&](const Lane& L, int k) {
    const int n = img_of(k, L.q / P::OPI), pix = L.q % P::OPI;
    static_for<2>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      EpiG K[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) K[g] = load_epig(ekb, CB::kCout, L.ek + i * 32 + 8 * g);
      uint32_t wq[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint32_t wd = 0;
#pragma unroll
        for (int ee = 0; ee < 4; ++ee) {
          const int r = 4 * g + ee;
          const int a = max(max(acc[i][0][r], acc[i][1][r]), max(acc[i][2][r], acc[i][3][r]));
          wd = rq_elem<FB>(a, K[g], ee, epb, wd);
        }
        wq[g] = wd;
      }
      auto s01 = __builtin_amdgcn_permlane32_swap(wq[0], wq[1], false, false);
      auto s23 = __builtin_amdgcn_permlane32_swap(wq[2], wq[3], false, false);
      uint32_t w0 = s01[0], w1 = s01[1], w2 = s23[0], w3 = s23[1];
      auto s02 = __builtin_amdgcn_permlane32_swap(w0, w2, false, false);
      auto s13 = __builtin_amdgcn_permlane32_swap(w1, w3, false, false);
      const uint4 v = make_uint4(s02[0], s13[0], s02[1], s13[1]);
      const int co = wc * 64 + i * 32;   // + 16 hi: this lane's 16 channels
      if (n < nimg) {
        if constexpr (KMAJOR) {   // [f / 32][image][32], f = pix * cout + channel (NHWC flatten)
          const int kc = (pix * CB::kCout + co) / 32;
          store_wt16(wt_rsrc(y), (uint32_t)(((long)kc * nimg + n) * 32 + 16 * L.hi), v);
        } else {
          store_wt16(wt_rsrc(y + (long)n * P::OPI * CB::kCout), (uint32_t)(pix * CB::kCout + co + 16 * L.hi), v);
        }
      }
    });
  };
  auto nofill = [](auto) {};

  // Each role runs its own period loop (T + 1 periods, one barrier each, or
  // two with a single A patch, so both roles pass the same barriers).
  if (role == 0) {
#pragma unroll 1
    for (int p = 0; p <= T; ++p) {
      if constexpr (!P::DOUBLE_A) {   // tile p's input, held since period p - 1
        if (p >= 1 && p < T) write_in(pa_buf(p));
        lds_barrier();
      }
      if (p < T) {
        const Lane L = lanes();
        pipe_job<CA, D, true>(pa_buf(p), L.ca, wra, wra, voff, wc, wp, L.l32, L.hi, acc, ga, nofill);
        // tile p + 1 (a valid dummy past the last): loads now, written after the
        // epilogue (double A patch) or after the next period barrier
        const int kn = p + 1 < T ? p + 1 : p;
#pragma unroll
        for (int q = 0; q < 4; ++q) sv[q] = *reinterpret_cast<const uint4*>(in_src(kn, q));
        epi_a(L, pb_buf(p));
        if constexpr (P::DOUBLE_A) write_in(pa_buf(p + 1));
      }
      P34_STAMP();
      lds_barrier();
      P34_STAMP();
    }
  } else {
#pragma unroll 1
    for (int p = 0; p <= T; ++p) {
      if constexpr (!P::DOUBLE_A) lds_barrier();
      if (p >= 1) {
        const Lane L = lanes();
        if (p >= 2) epi_b(L, p - 2);
        pipe_job<CB, D, true>(pb_buf(p - 1), L.cb, wrb, wrb, voff, wc, wp, L.l32, L.hi, acc, ga, nofill);
      }
      P34_STAMP();
      lds_barrier();
      P34_STAMP();
    }
    const Lane L = lanes();
    epi_b(L, T - 1);
  }
  P34_STAMP();
#ifdef QCN_PIPE34_STAMP
  if (threadIdx.x < 64) p34_stamp(stamp_kind, stamp_i, __builtin_amdgcn_s_memrealtime());
#endif
}

template <class CA, class CB, int D, int FA, int FB, bool KMAJOR>
__global__ __launch_bounds__(512, 1)
void convpair_ws_kernel(const uint8_t* __restrict__ x, int nimg, int x_zp, const int8_t* __restrict__ wa,
                        ConvEpi epa, int xb_zp, const int8_t* __restrict__ wb, ConvEpi epb,
                        uint8_t* __restrict__ y) {
  convpair_ws_body<CA, CB, D, FA, FB, KMAJOR>((int)blockIdx.x, (int)gridDim.x, x, nimg, x_zp, wa, epa, xb_zp,
                                              wb, epb, y);
}

// --------------------------------------------------------------------------
// The wave-specialised pair on v_mfma_i32_16x16x64_i8 (r05).
//
// The 16x16x64 shape does the same MACs per cycle as 32x32x32, but under a
// random-data int8 load the chip holds a higher clock with it: +11-18 % int8
// TOP/s at equal operand bytes per MAC (tools/micro/mfma_shape2.hip,
// profiles/r05_diag_mfma_shape.txt; r01's "2x slower" reading was a loop the
// compiler had filled with accumulator moves).  The convs here are power
// bound (DESIGN §5 "What bounds the convs"), so the shape is energy per image.
//
// Wave tile: 64 couts x 128 pixels as 4 x 8 blocks of 16 x 16; one K-step is
// one 64-byte chunk (a tap's 64 input channels).  Lane l = (p = l % 16,
// g = l / 16): A (weights, from L2) row 16 i + p, B (pixels, from the LDS
// patch) pixel p of block j, both K bytes 16 g .. 16 g + 15 of the chunk; the
// accumulator holds couts 16 i + 4 g + r (r = 0..3) of pixel p.  Pixel blocks:
// rows of 16 output pixels (conv A), or for a pooled conv B block j = 4 gq + jq
// is quadrant jq of pooled pixels 16 gq .. 16 gq + 15, so the 2x2 max is over
// four blocks in registers.  The patch layouts are re-searched for these
// reads (tools/lds_banks.py: every ds_read_b128 conflict-free needs a pixel
// stride of 16 B x 2 mod 4, i.e. Cin + 32).

// Diagnostic builds only (tools/clock: -DQCN_CONVNET_STAMP): s_memtime of lane
// 0 of wave 0 (conv A role) and wave 4 (conv B role) in every period of the
// 16x16 pair phases: [wg][phase: conv3+4, conv5+6][role][period][k], k = 0 the
// period's start (after its barrier), 1 the role's first piece done (A: the
// conv job; B: the previous tile's pooled epilogue), 2 its second (A: the
// epilogue and input hand-off; B: the conv job).  Plain vector stores into a
// buffer nothing else reads; the product library compiles none of it.
#ifdef QCN_CONVNET_STAMP
__device__ unsigned long long g_ws16_stamp[4096][2][2][8][3];
QCN_DEV void ws16_stamp(int ph, int p, int k) {
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  const unsigned lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int w = threadIdx.x >> 6;
  if ((w == 0 || w == 4) && lane == 0 && blockIdx.x < 4096 && p < 8) {
    volatile unsigned long long* d = &g_ws16_stamp[blockIdx.x][ph][w >> 2][p][k];
    *d = t + lane;
  }
}
#define WS16_STAMP(p, k) ws16_stamp(CA::kCin == 64 ? 0 : 1, (p), (k))
#else
#define WS16_STAMP(p, k)
#endif

// Patch slot of (wave wp, block j, lane pixel p) of conv C (output pixel
// coordinates, the 3x3 taps add PatchAddr<C>::delta).  Every layout used is
// affine: slot(wp, j, p) = slot(wp, 0, p) + jofs(j), checked at compile time,
// so a lane holds one base address and the K loop reads at immediate offsets.
template <class C>
struct Pix16 {
  static constexpr int slot(int seg, int prow, int pcol) {
    const int cpos = C::kSplit ? ((pcol & 1) * C::HALF + (pcol >> 1)) : pcol;
    return seg * C::SS + prow * C::RS + cpos * C::PS;
  }
  static constexpr int at(int wp, int j, int p) {
    if (C::kPool) {
      const int PW = C::W / 2, PR = C::R / 2;
      const int q = wp * 32 + (j >> 2) * 16 + p, jq = j & 3;
      return slot(q / (PR * PW), 2 * ((q / PW) % PR) + (jq >> 1), 2 * (q % PW) + (jq & 1));
    }
    const int m = (wp * 8 + j) * 16 + p;
    return slot(m / (C::R * C::W), (m / C::W) % C::R, m % C::W);
  }
  // conv A's output pixel as an interior slot of the NEXT conv's patch (layout N)
  template <class N>
  static constexpr int out_at(int wp, int j, int p) {
    const int m = (wp * 8 + j) * 16 + p;
    return Pix16<N>::slot(m / (C::R * C::W), (m / C::W) % C::R + 1, m % C::W + 1);
  }
  static constexpr int jofs(int j) { return at(0, j, 0) - at(0, 0, 0); }
  template <class N>
  static constexpr int out_jofs(int j) { return out_at<N>(0, j, 0) - out_at<N>(0, 0, 0); }
  static constexpr bool affine() {
    for (int wp = 0; wp < C::kWpx; ++wp)
      for (int j = 0; j < 8; ++j)
        for (int p = 0; p < 16; ++p)
          if (at(wp, j, p) != at(wp, 0, p) + jofs(j)) return false;
    return true;
  }
  template <class N>
  static constexpr bool out_affine() {
    for (int wp = 0; wp < C::kWpx; ++wp)
      for (int j = 0; j < 8; ++j)
        for (int p = 0; p < 16; ++p)
          if (out_at<N>(wp, j, p) != out_at<N>(wp, 0, p) + out_jofs<N>(j)) return false;
    return true;
  }
};

// One conv of the 16x16 pipeline over a staged patch: C::NCH K-steps of 32
// MFMAs.  ga[s & 1] holds step s's four A fragments (step 0's issued by the
// caller or by the previous job); step s + 1's are issued into the other slot
// early in step s; after the last step the NEXT job's first chunk is issued
// from wrn into slot 0 (its latency hides under the epilogue that follows).
// B fragments are single-buffered: block j's fragment of step s + 1 is read
// right after its fourth MFMA of step s.  lb: this lane's patch byte offset
// (Pix16<C>::at(wp, 0, p) + 16 g); voff: ((wc 64 + p) 64 + 16 g).
template <class C>
QCN_DEV void pipe_job16(const uint8_t* patch, const int* corr, wt_rsrc_t wr, wt_rsrc_t wrn, int voff, int wc,
                        int lb, int g, v4i (&acc)[4][8], v4i (&ga)[2][4]) {
  constexpr int CBK = C::kCin / 64, S = C::NCH;
  using X = Pix16<C>;
  static_assert(X::affine(), "pixel blocks at constant offsets");
  v4i c0[4];   // the first K-step's C operand: the zero-point correction
#pragma unroll
  for (int i = 0; i < 4; ++i) c0[i] = *reinterpret_cast<const v4i*>(corr + wc * 64 + 16 * i + 4 * g);
  auto rd_b = [&](int s, int j) {
    const int tap = s / CBK, cb = s % CBK;
    return *reinterpret_cast<const v4i*>(patch + lb + X::jofs(j) + PatchAddr<C>::delta(tap, j) + cb * 64);
  };
  auto issue = [&](wt_rsrc_t r, int s, int slot) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, s * C::WBUF + i * 1024, 0);
      ga[slot][i] = (v4i){(int)v[0], (int)v[1], (int)v[2], (int)v[3]};
    }
  };
  v4i fb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) fb[j] = rd_b(0, j);
  static_for<S>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    static_for<32>([&](auto mc) {
      constexpr int m = decltype(mc)::value, j = m >> 2, i = m & 3;
      __builtin_amdgcn_sched_barrier(0);
      acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ga[s & 1][i], fb[j], s == 0 ? c0[i] : acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (m == 1 && s + 1 < S) {
        // slot (s + 1) & 1 was step s - 1's: all its MFMAs have issued
        issue(wr, s + 1, (s + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (i == 3 && s + 1 < S) {
        fb[j] = rd_b(s + 1, j);
        __builtin_amdgcn_sched_barrier(0);
      }
    });
    // pin the step's MFMAs here (as pipe_job): side-effect free, they could
    // otherwise be sunk towards their uses with the fragments held live
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(acc[i][j]));
  });
  issue(wrn, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
}

template <class CA, class CB>
struct PairWs16 {
  static_assert(CA::NWAVES == 4 && CB::NWAVES == 4 && CA::WCO == CB::WCO && CA::WI == 2 && CB::WI == 2,
                "four waves of 64-cout x 128-pixel tiles per role");
  static_assert(!CA::kPool && CB::kPool && CA::kCout == CB::kCin, "A feeds B");
  static_assert(CA::PXB == CB::PXB && CA::SEGS == CB::SEGS && CA::R == CA::H && CA::W == CB::W &&
                !CA::kBand && !CB::kBand && !CA::kSplit, "whole images per tile");
  static_assert(Pix16<CA>::affine() && Pix16<CB>::affine() && Pix16<CA>::template out_affine<CB>(),
                "pixel blocks at constant offsets");
  static constexpr int SEGS = CA::SEGS, IMG = CA::IMG;
  static constexpr int IN_BYTES = SEGS * IMG * CA::kCin;   // a tile's input
  static_assert(IN_BYTES == 4 * 256 * 16, "four 16-B staging pieces per A-role thread");
  static constexpr int PA = (CA::PATCH + 15) / 16 * 16, PB = (CB::PATCH + 15) / 16 * 16;
  static constexpr int TAB = 16 * (CA::kCout + CB::kCout);   // u | v | mult | corr of both
  static constexpr bool DOUBLE_A = 2 * PA + 2 * PB + TAB <= 160 * 1024;
  static constexpr int OFF_PB = 0;
  static constexpr int OFF_PA = 2 * PB;
  static constexpr int OFF_EA = OFF_PA + (DOUBLE_A ? 2 : 1) * PA;   // u | v | mult, fp32 x cout each
  static constexpr int OFF_EB = OFF_EA + 12 * CA::kCout;
  static constexpr int OFF_CA = OFF_EB + 12 * CB::kCout;            // corr, int32 x cout
  static constexpr int OFF_CB = OFF_CA + 4 * CA::kCout;
  static constexpr int LDS = OFF_CB + 4 * CB::kCout;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static constexpr int OPI = CB::OPX / SEGS;   // pooled output pixels per image
};

// convpair_ws_body's schedule (roles, periods, LDS plan, tile -> image map
// b, b + G, ... with ILV as there) on the 16x16 pipeline above.
template <class CA, class CB, int FA, int FB, bool KMAJOR, bool ILV = false>
QCN_DEV void convpair_ws16_body(int b, int G, const uint8_t* __restrict__ x, int nimg, int x_zp,
                                const int8_t* __restrict__ wa, const ConvEpi& epa, int xb_zp,
                                const int8_t* __restrict__ wb, const ConvEpi& epb, uint8_t* __restrict__ y) {
  using P = PairWs16<CA, CB>;
  using XA = Pix16<CA>;
  using XB = Pix16<CB>;
  constexpr int SEGS = P::SEGS, IMG = CA::IMG, W = CA::W, WCO = CA::WCO;
  constexpr int CH16 = CA::kCin / 16;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x;
  const int role = __builtin_amdgcn_readfirstlane(tid >> 8);   // 0: conv A, 1: conv B
  const int rt = tid & 255, lane = tid & 63, wave = rt >> 6;   // thread / wave within the role
  const int wc = wave % WCO, wp = wave / WCO;
  int T;
  if constexpr (ILV) {
    const int mine = b < nimg ? (nimg - 1 - b) / G + 1 : 0;   // images b, b + G, ...
    T = (mine + SEGS - 1) / SEGS;
  } else {
    const int ntile = (nimg + SEGS - 1) / SEGS;
    T = b < ntile ? (ntile - 1 - b) / G + 1 : 0;   // this workgroup's tiles b, b + G, ...
  }
  // image of segment sg of tile k; a phantom segment of a ragged last tile
  // (images past this workgroup's) maps to the tile's first image, which this
  // workgroup owns: its outputs are never stored and no other workgroup's
  // data is read
  auto img_of = [&](int k, int sg) {
    const int n = ILV ? b + (k * SEGS + sg) * G : (b + k * G) * SEGS + sg;
    return n < nimg ? n : (ILV ? b + k * SEGS * G : (b + k * G) * SEGS);
  };
  auto in_src = [&](int k, int q) {
    const int p = rt + 256 * q;
    const int n = img_of(k, p / (IMG * CH16));
    return x + ((long)n * IMG + (p / CH16) % IMG) * CA::kCin + (p % CH16) * 16;
  };
  auto in_dst = [&](int q) {
    const int p = rt + 256 * q;
    const int pix = (p / CH16) % IMG;
    return CA::slot(p / (IMG * CH16), pix / W + 1, pix % W + 1) + (p % CH16) * 16;
  };
  // tile 0's input (A waves), loaded first so the latency hides under the
  // set-up; this copy dies at the first write: the A-role loop keeps its own
  // (a value live across the other role's branch would be spilled around it)
  uint4 sv0[4];
  if (role == 0 && T > 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) sv0[q] = *reinterpret_cast<const uint4*>(in_src(0, q));
  }
  float* eka = reinterpret_cast<float*>(lds + P::OFF_EA);
  float* ekb = reinterpret_cast<float*>(lds + P::OFF_EB);
  int* cra = reinterpret_cast<int*>(lds + P::OFF_CA);
  int* crb = reinterpret_cast<int*>(lds + P::OFF_CB);
  constexpr int NA = 3 * CA::kCout / 4, NB = 3 * CB::kCout / 4;       // float4 pieces
  constexpr int NCA = CA::kCout / 4, NCB = CB::kCout / 4;
  constexpr int NTAB = NA + NB + NCA + NCB, TPT = (NTAB + 255) / 256;
  float4 tval[TPT];
  auto tab = [&](int e, bool dst) -> float4* {
    if (e < NA) {
      const int a = e / (CA::kCout / 4), o = e % (CA::kCout / 4);
      const float* s = a == 0 ? epa.u : (a == 1 ? epa.v : epa.mult);
      return dst ? reinterpret_cast<float4*>(eka) + e : const_cast<float4*>(reinterpret_cast<const float4*>(s) + o);
    }
    e -= NA;
    if (e < NB) {
      const int a = e / (CB::kCout / 4), o = e % (CB::kCout / 4);
      const float* s = a == 0 ? epb.u : (a == 1 ? epb.v : epb.mult);
      return dst ? reinterpret_cast<float4*>(ekb) + e : const_cast<float4*>(reinterpret_cast<const float4*>(s) + o);
    }
    e -= NB;
    if (e < NCA)
      return dst ? reinterpret_cast<float4*>(cra) + e
                 : const_cast<float4*>(reinterpret_cast<const float4*>(epa.corr) + e);
    e -= NCA;
    return dst ? reinterpret_cast<float4*>(crb) + e
               : const_cast<float4*>(reinterpret_cast<const float4*>(epb.corr) + e);
  };
  {  // zero-point halos of every buffer of both patches (never overwritten)
    const uint32_t pa4 = xor80(splat_u8(x_zp)), pb4 = xor80(splat_u8(xb_zp));
    auto halo = [&](auto cfg, uint8_t* base, int nbuf, int pbytes, uint32_t pad) {
      using C = decltype(cfg);
      constexpr int HS = 2 * C::PCOLS + 2 * (C::PROWS - 2), CH = C::kCin / 16;
      const int total = nbuf * C::SEGS * HS * CH;
      for (int e = tid; e < total; e += 512) {
        const int c = e % CH, hs = (e / CH) % HS, sg = (e / (CH * HS)) % C::SEGS, bf = e / (CH * HS * C::SEGS);
        int pr, pc;
        if (hs < C::PCOLS) { pr = 0; pc = hs; }
        else if (hs < 2 * C::PCOLS) { pr = C::PROWS - 1; pc = hs - C::PCOLS; }
        else { const int r = hs - 2 * C::PCOLS; pr = 1 + (r >> 1); pc = (r & 1) ? C::PCOLS - 1 : 0; }
        *reinterpret_cast<uint4*>(base + bf * pbytes + C::slot(sg, pr, pc) + c * 16) = make_uint4(pad, pad, pad, pad);
      }
    };
    halo(CA{}, lds + P::OFF_PA, P::DOUBLE_A ? 2 : 1, P::PA, pa4);
    halo(CB{}, lds + P::OFF_PB, 2, P::PB, pb4);
  }
  // the epilogue tables (u | v | mult of both convs, both corr) in 16-B
  // pieces over the B-role threads, after the halos (values held across the
  // halo loop were spilled)
  if (role == 1) {
#pragma unroll
    for (int k = 0; k < TPT; ++k)
      if (rt + 256 * k < NTAB) tval[k] = *tab(rt + 256 * k, false);
#pragma unroll
    for (int k = 0; k < TPT; ++k)
      if (rt + 256 * k < NTAB) *tab(rt + 256 * k, true) = tval[k];
  }
  if (T == 0) return;   // (uniform; the launcher never makes such a workgroup)

  const int p16 = lane & 15, g = lane >> 4;
  const wt_rsrc_t wra = wt_rsrc(wa), wrb = wt_rsrc(wb);
  const int voff = (wc * 64 + p16) * 64 + g * 16;
  auto pa_buf = [&](int j) { return lds + P::OFF_PA + (P::DOUBLE_A ? (j & 1) * P::PA : 0); };
  auto pb_buf = [&](int j) { return lds + P::OFF_PB + (j & 1) * P::PB; };
  auto write_in = [&](uint8_t* pa, const uint4 (&sv)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<uint4*>(pa + in_dst(q)) =
          make_uint4(xor80(sv[q].x), xor80(sv[q].y), xor80(sv[q].z), xor80(sv[q].w));
  };
  // each role's first weight chunk, issued inside its own branch (the B
  // waves' first job starts a period later, the A waves' at once)
  auto first_chunk = [&](wt_rsrc_t w0, v4i (&ga)[2][4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(w0, voff, i * 1024, 0);
      ga[0][i] = (v4i){(int)v[0], (int)v[1], (int)v[2], (int)v[3]};
    }
  };

  v4i acc[4][8];
  if (role == 0) write_in(pa_buf(0), sv0);
  lds_barrier();

  // lane-derived addressing from a laundered lane id (not hoisted out of the
  // period loop and held live across the MFMA jobs)
  struct Lane {
    int p16, g, ek;
    int la, lb;   // patch offsets of block 0: conv A's and conv B's B-fragment reads
    int hb;       // conv B patch slot of conv A's output pixel (block 0) + this lane's channels
    int q;        // pooled output pixel of conv B within the tile (block group 0)
    const int *ca, *cb;
  };
  auto lanes = [&]() {
    int lz = lane;
    asm volatile("" : "+v"(lz));
    Lane L;
    L.p16 = lz & 15;
    L.g = lz >> 4;
    L.ek = wc * 64 + 4 * L.g;
    L.la = XA::at(wp, 0, L.p16) + 16 * L.g;
    L.lb = XB::at(wp, 0, L.p16) + 16 * L.g;
    L.hb = XA::template out_at<CB>(wp, 0, L.p16) + wc * 64 + 4 * L.g;
    L.q = wp * 32 + L.p16;
    L.ca = cra + (lz >> 6);   // (lz >> 6 == 0: an address the compiler cannot hoist)
    L.cb = crb + (lz >> 6);
    return L;
  };
  // A's epilogue into B's patch pb: one dword (4 channels) per block and row
  // of 16 channels, at the block's constant offset
  auto epi_a = [&](const Lane& L, uint8_t* pb) {
    static_for<4>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      const EpiG K = load_epig(eka, CA::kCout, L.ek + 16 * i);
      static_for<8>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        uint32_t wd = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) wd = rq_elem<FA>(acc[i][j][r], K, r, epa, wd);
        *reinterpret_cast<uint32_t*>(pb + L.hb + XA::template out_jofs<CB>(j) + 16 * i) = xor80(wd);
      });
    });
  };
  // B's pooled epilogue of tile k: per group of 16 pooled pixels, the max over
  // the four quadrant blocks, requant, a 4 x 4 dword transpose across the lane
  // groups (two permlane32 + two permlane16 swaps) and one 16-B store per lane
  auto epi_b = [&](const Lane& L, int k) {
    static_for<2>([&](auto gc) {
      constexpr int gq = decltype(gc)::value;
      uint32_t d[4];
      static_for<4>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const EpiG K = load_epig(ekb, CB::kCout, L.ek + 16 * i);
        uint32_t wd = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int a = max(max(acc[i][4 * gq][r], acc[i][4 * gq + 1][r]),
                            max(acc[i][4 * gq + 2][r], acc[i][4 * gq + 3][r]));
          wd = rq_elem<FB>(a, K, r, epb, wd);
        }
        d[i] = wd;
      });
      const auto s02 = __builtin_amdgcn_permlane32_swap(d[0], d[2], false, false);
      const auto s13 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);
      const auto t01 = __builtin_amdgcn_permlane16_swap(s02[0], s13[0], false, false);
      const auto t23 = __builtin_amdgcn_permlane16_swap(s02[1], s13[1], false, false);
      const uint4 v = make_uint4(t01[0], t01[1], t23[0], t23[1]);   // channels co .. co + 15
      const int q = L.q + 16 * gq;
      const int n = img_of(k, q / P::OPI), pix = q % P::OPI;
      const int co = wc * 64 + 16 * L.g;
      const bool real = ILV ? b + (k * SEGS + q / P::OPI) * G < nimg : (b + k * G) * SEGS + q / P::OPI < nimg;
      if (real) {
        if constexpr (KMAJOR) {   // [f / 32][image][32], f = pix * cout + channel (NHWC flatten)
          const int kc = (pix * CB::kCout + co) / 32;
          store_wt16(wt_rsrc(y), (uint32_t)(((long)kc * nimg + n) * 32 + 16 * (L.g & 1)), v);
        } else {
          store_wt16(wt_rsrc(y + (long)n * P::OPI * CB::kCout), (uint32_t)(pix * CB::kCout + co), v);
        }
      }
    });
  };

  if (role == 0) {
    v4i ga[2][4];
    first_chunk(wra, ga);
    uint4 sv[4] = {};   // tile p + 1's input, loaded during period p
#pragma unroll 1
    for (int p = 0; p <= T; ++p) {
      if constexpr (!P::DOUBLE_A) {   // tile p's input, held since period p - 1
        if (p >= 1 && p < T) write_in(pa_buf(p), sv);
        lds_barrier();
      }
      WS16_STAMP(p, 0);
      if (p < T) {
        const Lane L = lanes();
        pipe_job16<CA>(pa_buf(p), L.ca, wra, wra, voff, wc, L.la, L.g, acc, ga);
        WS16_STAMP(p, 1);
        const int kn = p + 1 < T ? p + 1 : p;
#pragma unroll
        for (int q = 0; q < 4; ++q) sv[q] = *reinterpret_cast<const uint4*>(in_src(kn, q));
        epi_a(L, pb_buf(p));
        if constexpr (P::DOUBLE_A) write_in(pa_buf(p + 1), sv);
        WS16_STAMP(p, 2);
      }
      lds_barrier();
    }
  } else {
    v4i ga[2][4];
    first_chunk(wrb, ga);
#pragma unroll 1
    for (int p = 0; p <= T; ++p) {
      if constexpr (!P::DOUBLE_A) lds_barrier();
      WS16_STAMP(p, 0);
      if (p >= 1) {
        const Lane L = lanes();
        if (p >= 2) epi_b(L, p - 2);
        WS16_STAMP(p, 1);
        pipe_job16<CB>(pb_buf(p - 1), L.cb, wrb, wrb, voff, wc, L.lb, L.g, acc, ga);
        WS16_STAMP(p, 2);
      }
      lds_barrier();
    }
    const Lane L = lanes();
    epi_b(L, T - 1);
#ifdef QCN_CONVNET_STAMP
    if (T + 1 < 8) { WS16_STAMP(T + 1, 0); }   // the last pooled epilogue ends here
#endif
  }
}

template <class CA, class CB, int FA, int FB, bool KMAJOR>
__global__ __launch_bounds__(512, 1)
void convpair_ws16_kernel(const uint8_t* __restrict__ x, int nimg, int x_zp, const int8_t* __restrict__ wa,
                          ConvEpi epa, int xb_zp, const int8_t* __restrict__ wb, ConvEpi epb,
                          uint8_t* __restrict__ y) {
  convpair_ws16_body<CA, CB, FA, FB, KMAJOR>((int)blockIdx.x, (int)gridDim.x, x, nimg, x_zp, wa, epa, xb_zp,
                                             wb, epb, y);
}

// The headline's patch layouts for the 16x16 reads (tools/lds_banks.py)
using W16A3 = ConvCfg<64, 128, 16, false, 2, 32, 0, 0, false>;
// (conv4 on its r04 layout — 2-way conflicted 16x16 B reads — would leave
// room for a double conv3 patch; measured 0.6 % slower,
// profiles/r05_diag_w16b4_double_a_ab.txt)
using W16B4 = ConvCfg<128, 128, 16, true, 2, 32, 64, 0, true>;
using W16A5 = ConvCfg<128, 256, 8, false, 1, 32, 192, 0, false>;
using W16B6 = ConvCfg<256, 256, 8, true, 1, 32, 0, 0, true>;

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
__global__ __launch_bounds__(256, 3)
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
      acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b, acc_init_corr(ep.corr, i * 32, hi),
                                                        0, 0, 0);
  }
  __syncthreads();  // im2col / patch are dead: the LDS becomes the output image
  uint8_t* lout = lds;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      epilogue_tile<1>(&acc[i][j], ep, i * 32, hi, lout + ((wave * 4 + j) * 32 + l32) * 80);
  __syncthreads();
  const long total = (long)nimg * H * W;
  store_staged<64, 80, 256>(lout, 512, y + p0 * 64, total - p0, tid);
}

using Conv2Cfg = ConvCfg<64, 64, 32, true, 4, 16, 96, 0, true>;

// --------------------------------------------------------------------------
// conv1 + conv2 fused, persistent and wave-specialised (the production path).
// One 512-thread workgroup per CU loops over half-image tiles.  Waves 4-7
// (producer) build conv2's input patch for tile j — fp32 window -> quantize ->
// conv1 on MFMA -> requant into the patch — while waves 0-3 (consumer) run
// conv2 on tile j-1 from the other patch buffer and store its pooled output.
// conv2's weights (36 KB) stay resident in LDS, so the consumer loop has no
// barriers and no weight traffic; the only synchronisation is one workgroup
// barrier per tile.  The producer's VALU-heavy conv1 and the consumer's MFMA
// work share the SIMDs instead of alternating.  The fp32 window of tile j+1 is
// loaded into registers at the start of the producer's phase, so its latency
// hides behind the conv1 work.
struct Conv12P {
  using C = Conv2Cfg;
  static constexpr int PATCH = C::PATCH;
  static constexpr int WRES = 9 * C::WBUF;                 // all conv2 weights
  // quantized fp32 input window: rows y0-2..y0+17, cols -2..33, one dword per
  // pixel (c0, c1, c2, 0) so conv1's im2col operand is plain aligned dwords
  static constexpr int IN_R = 20, IN_C = 40;   // cols -4 .. 35: interior 16-B aligned
  static constexpr int IN8 = IN_R * IN_C * 4;
  static constexpr int OFF_W = 2 * PATCH;
  static constexpr int OFF_IN = OFF_W + WRES;              // 2 x quantized input window
  static constexpr int OFF_EPI1 = OFF_IN + 2 * IN8;
  static constexpr int OFF_EPI2 = OFF_EPI1 + 12 * 64;
  static constexpr int OFF_CORR2 = OFF_EPI2 + 12 * 64;      // conv2 corr (int32 x 64)
  // conv1's MFMA A operand, per lane, in the dword-per-tap K order
  // ([i][lane] v4i), and conv1's corr: built once, read per tile
  static constexpr int OFF_A1 = OFF_CORR2 + 4 * 64;
  static constexpr int OFF_CORR1 = OFF_A1 + 2 * 64 * 16;
  static constexpr int LDS = OFF_CORR1 + 4 * 64;
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// conv_mainloop for weights resident in LDS (same swizzled chunk layout as the
// ring, chunk ch at wres + ch * WBUF): a barrier-free, fully unrolled pipeline.
template <class C>
QCN_DEV void conv_mainloop_res(const uint8_t* patch, const uint8_t* wres,
                               const int* __restrict__ corr, int wave, int lane,
                               v16i (&acc)[2][4]) {
  constexpr int CB = C::kCin / 64;
  const int wc = wave % C::WCO, wp = wave / C::WCO;
  const int l32 = lane & 31, hi = lane >> 5;
  const PatchAddr<C> pa(wp, l32, hi);
  const int arow = wc * 64 + l32;
  const int aswz = (arow >> 2) & 3;
  v16i c0[2];   // the first K-step's C operand
#pragma unroll
  for (int i = 0; i < 2; ++i) c0[i] = acc_init_corr(corr, wc * 64 + i * 32, hi);
  const uint8_t* abase = wres + arow * 64;
  auto rd_a = [&](int ch, int kk, int i) {
    return *reinterpret_cast<const v4i*>(abase + ch * C::WBUF + i * 32 * 64 +
                                         (((2 * kk + hi) ^ aswz) << 4));
  };
  auto rd_b = [&](int ch, int kk, int j) {
    const int tap = ch / CB, cb = ch % CB;
    return *reinterpret_cast<const v4i*>(patch + pa.base[j] + PatchAddr<C>::delta(tap, j) + cb * 64 +
                                         kk * 32);
  };
  auto step = [&](v4i (&fan)[2], v4i (&fbn)[4], int rch, int rkk, bool rd,
                  const v4i (&fa)[2], const v4i (&fb)[4], bool first) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      if (rd) {
        if (m < 2) fan[m] = rd_a(rch, rkk, m);
        else if (m < 6) fbn[m - 2] = rd_b(rch, rkk, m - 2);
      }
      __builtin_amdgcn_sched_barrier(0);
      acc[m >> 2][m & 3] = __builtin_amdgcn_mfma_i32_32x32x32_i8(
          fa[m >> 2], fb[m & 3], first ? c0[m >> 2] : acc[m >> 2][m & 3], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  v4i fa0[2], fb0[4], fa1[2], fb1[4];
  fa0[0] = rd_a(0, 0, 0);
  fa0[1] = rd_a(0, 0, 1);
#pragma unroll
  for (int j = 0; j < 4; ++j) fb0[j] = rd_b(0, 0, j);
#pragma unroll
  for (int ch = 0; ch < C::NCH; ++ch) {
    step(fa1, fb1, ch, 1, true, fa0, fb0, ch == 0);
    step(fa0, fb0, ch + 1, 0, ch + 1 < C::NCH, fa1, fb1, false);
  }
}

// Diagnostic builds only (tools/clock: -DQCN_C12_STAMP): s_memtime of lane 0
// of waves 0 (consumer), 4 and 5 (producer) at the top of every tile
// iteration, before its barrier and after conv2's main loop, plain vector
// stores.  Not in the product.
#ifdef QCN_C12_STAMP
__device__ unsigned long long g_c12_stamp[4096][3][12][3];
QCN_DEV void c12_stamp(int j, int k) {
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  const unsigned lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int w = threadIdx.x >> 6;
  const int s = w == 0 ? 0 : (w == 4 ? 1 : (w == 5 ? 2 : -1));
  if (s >= 0 && lane == 0 && blockIdx.x < 4096 && j < 12) {
    volatile unsigned long long* d = &g_c12_stamp[blockIdx.x][s][j][k];
    *d = t + lane;
  }
}
#define C12_STAMP(j, k) c12_stamp(j, k)
#else
#define C12_STAMP(j, k)
#endif

// Images t0, t0 + ts, ... (T / 2 of them, each as its top then its bottom
// half-image tile) through the producer/consumer pipeline.  512 threads, LDS
// layout Conv12P.
QCN_DEV void conv12p_body(int t0, int ts, int T, const float* __restrict__ x, int nimg,
                          float in_inv, int in_zp, const int8_t* __restrict__ w1, ConvEpi ep1,
                          int x2_zp, const int8_t* __restrict__ w2, ConvEpi ep2,
                          uint8_t* __restrict__ y) {
  using C = Conv2Cfg;
  using L = Conv12P;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool producer = wave >= 4;
  // window-staging thread id: producer waves 5-7 (0..191, 180 used).  Wave 4
  // computes the most conv1 rows of a top half (5 of 17), so it stages none
  const int ptid = tid - 320;
  // tile j of this workgroup: image t0 + (j / 2) * ts, top half then bottom
  // half (so every odd j reuses two conv1 rows from tile j - 1)
  auto tile_of = [&](int j) { return (t0 + (j >> 1) * ts) * 2 + (j & 1); };
  uint8_t* patch0 = lds;
  uint8_t* patch1 = lds + L::PATCH;
  uint8_t* in8_0 = lds + L::OFF_IN;
  uint8_t* in8_1 = lds + L::OFF_IN + L::IN8;

  float4 xraw[3];
  const uint32_t padw = xor80(splat_u8(x2_zp));
  const uint4 pad4 = make_uint4(padw, padw, padw, padw);
  for (int e = tid; e < 2 * C::PROWS * 8; e += 512) {
    const int buf = e / (C::PROWS * 8), r = e % (C::PROWS * 8);
    const int pr = r / 8, pc = ((r / 4) & 1) ? C::PCOLS - 1 : 0, chunk = r & 3;
    *reinterpret_cast<uint4*>(lds + buf * L::PATCH + C::slot(0, pr, pc) + chunk * 16) = pad4;
  }

  // tables the tile loop reads (issued after the producer's first window
  // loads, so the two latencies overlap); run by the consumer waves
  auto setup = [&]() {
    // ---- once per workgroup: resident conv2 weights (ring layout), epilogue
    // constants of both layers, conv1's operand tables.  The weights go by
    // LDS-DMA (9 x 1 KB per consumer wave); the producer waves only load
    // their first input window meanwhile
    if (!producer) {
      const int wave_u = __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
      for (int i = 0; i < L::WRES / 4096; ++i) {
        const int p = i * 4 + wave_u;
        const int o = p * 1024 + lane * 16;
        const int ch = o / C::WBUF, oc = o % C::WBUF;
        const int r = oc >> 6, sl = (oc >> 4) & 3;
        glds16(w2 + (long)ch * C::WBUF + r * 64 + ((sl ^ ((r >> 2) & 3)) << 4), lds + L::OFF_W + p * 1024);
      }
    }

    // the input windows' constant zero-point border (both buffers)
    const uint32_t in_pad = xor80(splat_u8(in_zp)) & 0x00ffffffu;
    for (int e = tid; e < 2 * L::IN_R * L::IN_C; e += 512) {
      const int b = e / (L::IN_R * L::IN_C), rc = e % (L::IN_R * L::IN_C);
      const int rr = rc / L::IN_C, cc = rc % L::IN_C;
      const bool pad_row = b == 0 ? rr < 2 : rr >= 18;
      if (pad_row || cc < 4 || cc >= 36)
        reinterpret_cast<uint32_t*>(lds + L::OFF_IN + b * L::IN8)[rc] = in_pad;
    }
    if (!producer) stage_epik<64, 256>(ep1, reinterpret_cast<float*>(lds + L::OFF_EPI1), tid);
    if (!producer) stage_epik<64, 256>(ep2, reinterpret_cast<float*>(lds + L::OFF_EPI2), tid);
    {
      int t = tid;
      asm volatile("" : "+v"(t));   // a fresh copy: no tid-derived offset held across phases
      if (t < 16)
        reinterpret_cast<int4*>(lds + L::OFF_CORR2)[t] = reinterpret_cast<const int4*>(ep2.corr)[t];
      if (t >= 64 && t < 80)
        reinterpret_cast<int4*>(lds + L::OFF_CORR1)[t - 64] = reinterpret_cast<const int4*>(ep1.corr)[t - 64];
    }
    if (wave == 3) {
      // conv1 A operand in the dword-per-tap K order (k' = 4 tap + c, taps
      // 0..7) from the [64][32] (k = 3 tap + c) packing
      const int l32 = lane & 31, hi = lane >> 5;
      v4i* a1t = reinterpret_cast<v4i*>(lds + L::OFF_A1);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint4 r0 = *reinterpret_cast<const uint4*>(w1 + (i * 32 + l32) * 32);
        const uint4 r1 = *reinterpret_cast<const uint4*>(w1 + (i * 32 + l32) * 32 + 16);
        const uint32_t wd[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
        auto byte = [&](int k) -> uint32_t { return (wd[k >> 2] >> (8 * (k & 3))) & 0xff; };
        auto tapw = [&](int t) -> int {   // (w[3t], w[3t+1], w[3t+2], 0)
          return (int)(byte(3 * t) | (byte(3 * t + 1) << 8) | (byte(3 * t + 2) << 16));
        };
        // tap 8's three channels ride in the pad byte (byte 3) of taps 0, 1, 2,
        // so the whole 27-long K fits one K=32 MFMA step
        const v4i lo4 = (v4i){tapw(0) | (int)(byte(24) << 24), tapw(1) | (int)(byte(25) << 24),
                              tapw(2) | (int)(byte(26) << 24), tapw(3)};
        const v4i hi4 = (v4i){tapw(4), tapw(5), tapw(6), tapw(7)};
        a1t[i * 64 + lane] = hi ? hi4 : lo4;
      }
    }
  };
  // Window staging: the fp32 NCHW input rows of tile t, quantized (aten
  // quantize_per_tensor) to one s8 dword (c0, c1, c2, 0) per pixel.  Window
  // row rr is input row y0 - 2 + rr, window column cc is input column cc - 4.
  // Only the image interior changes from tile to tile: the two rows outside
  // the image (rows 0-1 of a top half, 18-19 of a bottom half — each half has
  // its own buffer) and the side columns are zero points written once.
  // Producer thread pt < 144 (waves 5-7) owns window row rr0 + pt / 8 and
  // input columns 4g .. 4g + 3 (g = pt % 8): three aligned 16-B loads, 12
  // values at 4 VALU each (mul, rndne, + zp, saturating v_cvt_pk_u8_f32), one
  // ds_write_b128.  stage_load only issues the loads (their latency hides
  // behind conv1_tile); stage_store quantizes and writes.
  // The window index math depends only on the thread id; laundering it
  // through an empty asm per use keeps LICM from hoisting loop-invariant
  // values out of the tile loop (they were spilled: the consumer's MFMA state
  // shares the register budget).
  auto fresh_ptid = [&]() {
    int v = ptid;
    asm volatile("" : "+v"(v));
    return v;
  };
  auto stage_load = [&](int t) {
    if (ptid < 0) return;   // wave 4 (whole wave): no window share
    const int n = t >> 1, y0 = (t & 1) * 16;
    const int pt = fresh_ptid();
    const int r = pt < 144 ? pt >> 3 : 0, g = pt & 7;
    const int iy = y0 + (y0 == 0 ? 0 : -2) + r;   // rows 0..17 of the top half, 14..31 of the bottom
    const int nc = n < nimg ? n : nimg - 1;
#pragma unroll
    for (int c = 0; c < 3; ++c)
      xraw[c] = *reinterpret_cast<const float4*>(x + (((long)nc * 3 + c) * 32 + iy) * 32 + 4 * g);
  };
  auto stage_store = [&](uint8_t* in8, int half) {
    const int pt = fresh_ptid();
    if (pt >= 0 && pt < 144) {
      const int rr = (half ? 0 : 2) + (pt >> 3), g = pt & 7;
      const float zpf = (float)in_zp;
      uint32_t wd[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        uint32_t d = 0;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float xv = e == 0 ? xraw[c].x : e == 1 ? xraw[c].y : e == 2 ? xraw[c].z : xraw[c].w;
          // zp + rint(x / s), saturated to [0, 255]; rint(...) + zp is exact
          // below 2^24 and saturates the same way above
          d = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_rintf(xv * in_inv) + zpf, c, d);
        }
        wd[e] = d ^ 0x00808080u;
      }
      *reinterpret_cast<uint4*>(in8 + (rr * L::IN_C + 4 + 4 * g) * 4) = make_uint4(wd[0], wd[1], wd[2], wd[3]);
    }
  };
  auto fresh = [](int v) {  // see fresh_ptid
    asm volatile("" : "+v"(v));
    return v;
  };
  bool vuni = false, muni = false;
  const bool fast1 = epi_fast(ep1);
  // conv2's patch for tile t: its 18 rows are conv1 rows y0 - 1 .. y0 + 16.
  // The row outside the image (row 0 of a top half, row 17 of a bottom half)
  // is conv2's zero-point padding, written without computing it.  A bottom
  // half right after its top half (prev != nullptr) copies rows 0 and 1
  // from rows 16 and 17 of the top half's patch (conv1 rows 15 and 16) instead
  // of recomputing them.  The remaining rows are computed as r0 + w,
  // r0 + w + step, ... (wave w of `step` waves).
  auto conv1_tile = [&](int t, const uint8_t* in8, uint8_t* pb, const uint8_t* prev, int w,
                        int step) {
    // producer waves issue first: their VALU-bound conv1 is the longer phase,
    // the consumer's MFMAs fill the gaps (measured 53.6 vs 59.2 us)
    __builtin_amdgcn_s_setprio(kProdPrio);
    const int h = t & 1, y0 = h * 16;
    const int r0 = h == 0 ? 1 : (prev ? 2 : 0), r1 = h == 0 ? 18 : 17;
    const int ln = fresh(lane), l32 = ln & 31, hi = ln >> 5;
    if (w == step - 1) {   // the wave with the fewest rows: the padding row
      uint8_t* prow_ptr = pb + C::slot(0, h == 0 ? 0 : 17, l32 + 1);
      *reinterpret_cast<uint4*>(prow_ptr + hi * 32) = pad4;
      *reinterpret_cast<uint4*>(prow_ptr + hi * 32 + 16) = pad4;
    }
    if (prev) {   // rows 16, 17 of the top half -> rows 0, 1 (whole rows, halos included)
      for (int e = w * 64 + ln; e < 2 * C::RS / 16; e += step * 64)
        *reinterpret_cast<uint4*>(pb + C::slot(0, 0, 0) + e * 16) =
            *reinterpret_cast<const uint4*>(prev + C::slot(0, 16, 0) + e * 16);
    }
    const float* ek1 = reinterpret_cast<const float*>(lds + L::OFF_EPI1);
    // conv1 A operand and corrected accumulator init from the LDS tables
    // (built once in the prologue; LDS latency instead of a dependent L2
    // round trip at every tile start; re-read per tile so they are not live
    // across the consumer's MFMA region)
    v4i a1[2];
    v16i c1[2];
    {
      const v4i* a1t = reinterpret_cast<const v4i*>(lds + L::OFF_A1);
      const int* corr1 = reinterpret_cast<const int*>(lds + L::OFF_CORR1);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a1[i] = a1t[i * 64 + ln];
        c1[i] = acc_init_corr(corr1, i * 32, hi);
      }
    }
    const int* in32 = reinterpret_cast<const int*>(in8);
    // B operand of one conv1 row: window dwords (c0, c1, c2, 0) per pixel;
    // low lanes carry taps (0,0) (0,1) (0,2) (1,0) with tap (2,2)'s channel c
    // in the pad byte of tap (0,c) (v_perm), high lanes (1,1) (1,2) (2,0) (2,1)
    auto bop = [&](int tr, v4i& b0) {
      const int* r0 = in32 + (tr + 0) * L::IN_C + l32 + 3;   // input cols l32-1 .. l32+1
      const int* r1 = r0 + L::IN_C;
      const int* r2 = r1 + L::IN_C;
      if (hi == 0) {
        const uint32_t t8 = (uint32_t)r2[2];
        b0 = (v4i){(int)__builtin_amdgcn_perm((uint32_t)r0[0], t8, 0x00060504u),
                   (int)__builtin_amdgcn_perm((uint32_t)r0[1], t8, 0x01060504u),
                   (int)__builtin_amdgcn_perm((uint32_t)r0[2], t8, 0x02060504u), r1[0]};
      } else {
        b0 = (v4i){r1[1], r1[2], r2[0], r2[1]};
      }
    };
    auto rows = [&](auto mode) {
      // 0 general, 1 v+mult uniform, 2 v uniform; 3 / 4: 1 / 2 with the
      // one-fma QDQ hand-off (ep1.qdq == 2)
      constexpr int MODE = decltype(mode)::value > 2 ? decltype(mode)::value - 2 : decltype(mode)::value;
      constexpr bool AFF = decltype(mode)::value > 2;
      // lean epilogue constants: u (and mult unless uniform) of this lane's
      // 16 channels per half; v (and mult) as scalars.  EpiK (96 VGPRs) for
      // the general path only.
      float u[2][16], m[2][16];
      const float sv = ek1[64], sm = ek1[128];
      if constexpr (MODE != 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int co = i * 32 + 8 * g + 4 * hi;
            const float4 u4 = *reinterpret_cast<const float4*>(ek1 + co);
            u[i][4 * g] = u4.x; u[i][4 * g + 1] = u4.y; u[i][4 * g + 2] = u4.z; u[i][4 * g + 3] = u4.w;
            if constexpr (MODE == 2) {
              const float4 m4 = *reinterpret_cast<const float4*>(ek1 + 128 + co);
              m[i][4 * g] = m4.x; m[i][4 * g + 1] = m4.y; m[i][4 * g + 2] = m4.z; m[i][4 * g + 3] = m4.w;
            }
          }
      }
      if constexpr (MODE == 0) {
        for (int tr = r0 + w; tr < r1; tr += step) {
          const int iy = y0 - 1 + tr;
          uint8_t* prow_ptr = pb + C::slot(0, tr, l32 + 1);
          if (iy < 0 || iy >= 32) {  // wave-uniform: conv2's zero-point padding row
            *reinterpret_cast<uint4*>(prow_ptr + hi * 32) = pad4;
            *reinterpret_cast<uint4*>(prow_ptr + hi * 32 + 16) = pad4;
            continue;
          }
          v4i b0;
          bop(tr, b0);
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            v16i acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1[i], b0, c1[i], 0, 0, 0);
            epilogue_tile_kf<1, true>(&acc, load_epik_lds(ek1, 64, i * 32, hi), ep1, i * 32, hi,
                                      prow_ptr);
          }
        }
      } else {
        // rows w, w+4, ... of this producer wave, software-pipelined: the next
        // row's im2col reads and MFMAs are issued before this row's requant,
        // so the VALU never waits on an MFMA result (that cost ~40 s_nop per
        // row).  Halo rows are computed like the others and then overwritten.
        const int wr = r0 + w;   // first row of this wave
        const int nr = (r1 - wr + step - 1) / step;
        auto mfma_row = [&](int tr, v16i (&acc)[2]) {
          v4i b0;
          bop(tr, b0);
#pragma unroll
          for (int i = 0; i < 2; ++i)
            acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1[i], b0, c1[i], 0, 0, 0);
        };
        // requantize one conv1 row (both 32-channel halves) straight into its
        // conv2 patch row
        auto requant_row = [&](const v16i (&acc)[2], int tr) {
          v2f t[2][8];
          // scalar fma / mul (-fno-slp-vectorize keeps them scalar): packed fp32
          // beside another wave's MFMAs costs more issue than two scalar ops
          // (MI355X_MICROARCH 'price of one filler'); 53.5 -> 45.4 us here
          // (tools/micro/flag_ab.sh)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              float f = (float)acc[i][e];
              f = __builtin_fmaf(u[i][e], sv, f);
              f = f * (MODE == 1 ? sm : m[i][e]);
              if constexpr (AFF) f = qdq_aff_f(f, ep1);
              t[i][e >> 1][e & 1] = f;
            }
          uint8_t* prow_ptr = pb + C::slot(0, tr, l32 + 1);
          // the lane's 4-channel groups 8g + 4hi go straight to their dwords in
          // the patch row (v_permlane32_swap costs ~25 cycles each,
          // tools/micro/valu_rate.hip; four ds_write_b32 are cheaper)
          uint32_t* pdw = reinterpret_cast<uint32_t*>(prow_ptr) + hi;
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              uint32_t wd = __builtin_amdgcn_cvt_pk_u8_f32(t[i][2 * g].x, 0, 0u);
              wd = __builtin_amdgcn_cvt_pk_u8_f32(t[i][2 * g].y, 1, wd);
              wd = __builtin_amdgcn_cvt_pk_u8_f32(t[i][2 * g + 1].x, 2, wd);
              wd = __builtin_amdgcn_cvt_pk_u8_f32(t[i][2 * g + 1].y, 3, wd);
              pdw[i * 8 + 2 * g] = xor80(wd);   // channels i*32 + 8g + 4hi .. +3
            }
          const int iy = y0 - 1 + tr;
          if (iy < 0 || iy >= 32) {  // wave-uniform: conv2's zero-point padding row
            *reinterpret_cast<uint4*>(prow_ptr + hi * 32) = pad4;
            *reinterpret_cast<uint4*>(prow_ptr + hi * 32 + 16) = pad4;
          }
        };
        // two named accumulator sets in ping-pong (a copy per row cost 16
        // v_mov_b64): row kr+1's im2col reads and MFMAs go out before row kr's
        // requant, so the VALU never waits on an MFMA result
        v16i acc_x[2], acc_y[2];
        if (nr > 0) mfma_row(wr, acc_x);
#pragma unroll
        for (int kr = 0; kr < 5; kr += 2) {
          if (kr >= nr) break;
          if (kr + 1 < nr) mfma_row(wr + step * (kr + 1), acc_y);
          requant_row(acc_x, wr + step * kr);
          if (kr + 1 < nr) {
            if (kr + 2 < nr) mfma_row(wr + step * (kr + 2), acc_x);
            requant_row(acc_y, wr + step * (kr + 1));
          }
        }
      }
    };
    if (fast1 && vuni) {
      if (muni) rows(std::integral_constant<int, 1>{});
      else rows(std::integral_constant<int, 2>{});
    } else if (ep1.qdq == 2 && vuni) {
      if (muni) rows(std::integral_constant<int, 3>{});
      else rows(std::integral_constant<int, 4>{});
    } else {
      rows(std::integral_constant<int, 0>{});
    }
  };
  auto conv2_tile = [&](int t, const uint8_t* pb) {
    const int ln = fresh(lane), l32 = ln & 31, hi = ln >> 5;
    v16i acc[2][4];
    conv_mainloop_res<C>(pb, lds + L::OFF_W, reinterpret_cast<const int*>(lds + L::OFF_CORR2),
                         wave, ln, acc);
    C12_STAMP(((t >> 1) - t0) / ts * 2 + (t & 1) + 1, 2);
    const int n = t >> 1, h = t & 1;
    const float* ek2 = reinterpret_cast<const float*>(lds + L::OFF_EPI2);
    uint8_t* dst = y + ((long)n * 256 + h * 128 + wave * 32 + l32) * 64;
    const uint8_t* wbase = y + ((long)n * 256 + h * 128) * 64;   // write-through destination
    const uint32_t woff = (uint32_t)((wave * 32 + l32) * 64);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      epilogue_tile_kf<4, false, false, true>(acc[i], load_epik_lds(ek2, 64, i * 32, hi), ep2, i * 32, hi,
                                              dst, wbase, woff);
  };

  if (producer && T > 0) stage_load(tile_of(0));
  setup();
  if (producer && T > 0) stage_store(in8_0, 0);
  if (!producer) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // own weight DMA landed
  __syncthreads();
  // conv1 requant specialisation: v (and mult) identical across channels —
  // per-tensor weights give v = 1/aws, mult = aws/s_y; per-channel v = 1
  {
    const float* ek1 = reinterpret_cast<const float*>(lds + L::OFF_EPI1);
    const int l = lane;
    vuni = __builtin_amdgcn_ballot_w64(ek1[64 + l] != ek1[64]) == 0;
    muni = __builtin_amdgcn_ballot_w64(ek1[128 + l] != ek1[128]) == 0;
  }
  constexpr bool SPLIT0 = true;
  for (int j = 0; j <= T; ++j) {
    C12_STAMP(j, 0);
    if (producer) {
      if (j + 1 < T) stage_load(tile_of(j + 1));
      if (j < T) {
        // the first tile's conv1 is split with the (otherwise idle) consumer waves
        const bool split = SPLIT0 && j == 0;
        conv1_tile(tile_of(j), (j & 1) ? in8_1 : in8_0, (j & 1) ? patch1 : patch0,
                   (j & 1) ? patch0 : nullptr, split ? wave : wave - 4, split ? 8 : 4);
      }
      if (j + 1 < T) stage_store(((j + 1) & 1) ? in8_1 : in8_0, (j + 1) & 1);
    } else if (j >= 1) {
      conv2_tile(tile_of(j - 1), ((j - 1) & 1) ? patch1 : patch0);
    } else if (SPLIT0 && T > 0) {
      conv1_tile(tile_of(0), in8_0, patch0, nullptr, wave, 8);
      __builtin_amdgcn_s_setprio(0);
    }
    C12_STAMP(j, 1);
    __syncthreads();
  }
}

__global__ __launch_bounds__(512, 1)
void conv12p_kernel(const float* __restrict__ x, int nimg, float in_inv, int in_zp,
                    const int8_t* __restrict__ w1, ConvEpi ep1, int x2_zp,
                    const int8_t* __restrict__ w2, ConvEpi ep2, uint8_t* __restrict__ y) {
  const int T = (int)blockIdx.x < nimg ? 2 * ((nimg - 1 - (int)blockIdx.x) / (int)gridDim.x + 1) : 0;
  conv12p_body((int)blockIdx.x, (int)gridDim.x, T, x, nimg, in_inv, in_zp, w1, ep1, x2_zp, w2, ep2, y);
}

// --------------------------------------------------------------------------
// conv1 .. conv6 in ONE persistent launch (r04).  Every conv of the net reads
// only its own image, and the three persistent kernels of the forward give
// workgroup b of G the same images b, b + G, b + 2G, ... (conv12p: whole
// images, top half then bottom half; the conv3+4 pair: one image per tile;
// the conv5+6 pair: two images per tile, paired as b + 2kG, b + (2k+1)G
// here).  So the workgroup runs the three phases back to back over its own
// images with no cross-workgroup dependency: the two dependent-launch
// boundaries (a kernel's drain, the next one's dispatch ramp and prologue)
// go away.  a2 / a4 pass through memory as before (write-through stores,
// drained before the phase barrier; this CU never read those addresses
// before in this launch, so its L1 holds no stale copy).  Same LDS, same
// numerics, same code as the three launches (phase bodies shared).
// the six layers as separate by-value kernel arguments (a struct of arrays
// passed whole made the compiler copy it to scratch to take references into it)
#define QCN_C16_PARAMS                                                                                   \
  const int8_t* __restrict__ w0, ConvEpi e0, int z0, const int8_t* __restrict__ w1, ConvEpi e1, int z1, \
      const int8_t* __restrict__ w2, ConvEpi e2, int z2, const int8_t* __restrict__ w3, ConvEpi e3,      \
      int z3, const int8_t* __restrict__ w4, ConvEpi e4, int z4, const int8_t* __restrict__ w5,          \
      ConvEpi e5, int z5
#define QCN_C16_ARGS(L)                                                                                  \
  (L).w[0], (L).ep[0], (L).x_zp[0], (L).w[1], (L).ep[1], (L).x_zp[1], (L).w[2], (L).ep[2], (L).x_zp[2],   \
      (L).w[3], (L).ep[3], (L).x_zp[3], (L).w[4], (L).ep[4], (L).x_zp[4], (L).w[5], (L).ep[5], (L).x_zp[5]

struct ConvnetLayers {
  const int8_t* w[6];
  ConvEpi ep[6];
  int x_zp[6];   // input zero point of conv i (x_zp[0]: the QuantStub's)
};

// one image per workgroup (<= 1 image per CU): the 8-wave forms of the pairs
using SmA3 = ConvCfg<64, 128, 16, false, 4, 16, 96, 0, false, 2, 2>;
using SmB4 = ConvCfg<128, 128, 16, true, 2, 16, 32, 0, true, 1, 4>;
using SmA5 = ConvCfg<128, 256, 8, false, 1, 16, 224, 0, false, 1, 2>;
using SmB6 = ConvCfg<256, 256, 8, true, 1, 16, 32, 64, true, 1, 2>;

using WsA3 = ConvCfg<64, 128, 16, false, 2, 16, 96, 0, false>;
using WsB4 = ConvCfg<128, 128, 16, true, 2, 16, 32, 0, true>;
using WsA5 = ConvCfg<128, 256, 8, false, 1, 16, 224, 0, false>;
using WsB6 = ConvCfg<256, 256, 8, true, 1, 16, 32, 64, true>;

constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int kConvnet16Lds = cmax(Conv12P::LDS, cmax(PairWs16<W16A3, W16B4>::LDS, PairWs16<W16A5, W16B6>::LDS));
constexpr int kConvnetSmLds = cmax(Conv12P::LDS, cmax(PairCfg<SmA3, SmB4>::LDS, PairGaCfg<SmA5, SmB6>::LDS));

// Diagnostic builds only (tools/clock: -DQCN_CONVNET_STAMP): s_memtime /
// s_memrealtime of wave 0 at the start, after each phase and at the end of
// every workgroup, stored by one lane with plain vector stores.  The product
// library compiles none of it.
#ifdef QCN_CONVNET_STAMP
__device__ unsigned long long g_c16_stamp[4096][8];
QCN_DEV void c16_stamp(int i) {
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  const unsigned long long r = __builtin_amdgcn_s_memrealtime();
  const unsigned lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if ((threadIdx.x >> 6) == 0 && lane == 0 && blockIdx.x < 4096) {
    volatile unsigned long long* d = g_c16_stamp[blockIdx.x];
    d[i] = t + lane;
    d[4 + i] = r + lane;
  }
}
#define C16_STAMP(i) c16_stamp(i)
#else
#define C16_STAMP(i)
#endif

QCN_DEV void phase_boundary() {
  // every wave's stores of the phase complete, all LDS use done, default priority
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_setprio(0);
  __syncthreads();
}

// The same launch with the pair phases on the 16x16x64 pipeline (r05).  The
// conv12 phase is unchanged.  Each pair phase reads only a2 / a4 images its
// own workgroup wrote (conv3+4 tiles b, b + G, ... of one image each —
// static_assert below — and conv5+6 the interleaved pairs).
template <int EM, bool KMAJOR>
__global__ __launch_bounds__(512, 1)
void convnet_convs16_kernel(const float* __restrict__ x, int nimg, float in_inv, QCN_C16_PARAMS,
                            uint8_t* __restrict__ a2, uint8_t* __restrict__ a4, uint8_t* __restrict__ a6) {
  static_assert(PairWs16<W16A3, W16B4>::SEGS == 1, "conv3+4 tile k of workgroup b is image b + kG");
  const int b = (int)blockIdx.x, G = (int)gridDim.x;
  const int T = b < nimg ? 2 * ((nimg - 1 - b) / G + 1) : 0;
  C16_STAMP(0);
  conv12p_body(b, G, T, x, nimg, in_inv, z0, w0, e0, z1, w1, e1, a2);
  phase_boundary();
  C16_STAMP(1);
  convpair_ws16_body<W16A3, W16B4, EM, EM, false>(b, G, a2, nimg, z2, w2, e2, z3, w3, e3, a4);
  phase_boundary();
  C16_STAMP(2);
  convpair_ws16_body<W16A5, W16B6, EM, EM, KMAJOR, true>(b, G, a4, nimg, z4, w4, e4, z5, w5, e5, a6);
#ifdef QCN_CONVNET_STAMP
  __syncthreads();
#endif
  C16_STAMP(3);
}

// The same at one image per workgroup (batch <= CUs, e.g. configs[1]'s 256):
// conv12p over the workgroup's image, then the 8-wave conv3+4 and conv5+6
// pair bodies of the small-batch launches on that image.  Epilogue forms and
// conv6's layout (ep.kmajor) are runtime here.
__global__ __launch_bounds__(512, 1)
void convnet_convs_sm_kernel(const float* __restrict__ x, int nimg, float in_inv, QCN_C16_PARAMS,
                             uint8_t* __restrict__ a2, uint8_t* __restrict__ a4, uint8_t* __restrict__ a6) {
  const int b = (int)blockIdx.x;
  C16_STAMP(0);
  conv12p_body(b, (int)gridDim.x, 2, x, nimg, in_inv, z0, w0, e0, z1, w1, e1, a2);
  phase_boundary();
  C16_STAMP(1);
  convpair_body<SmA3, SmB4>(b, a2, nimg, z2, w2, e2, z3, w3, e3, a4);
  phase_boundary();
  C16_STAMP(2);
  convpair_ga_body<SmA5, SmB6, kSm56D>(b, a4, nimg, z4, w4, e4, z5, w5, e5, a6);
#ifdef QCN_CONVNET_STAMP
  __syncthreads();
#endif
  C16_STAMP(3);
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

// ---- host: the QDQ hand-off in one fma (ConvEpi::qdq == 2)
//
// After the requant the hand-off is a function of one integer only: with
// r = rint(ab), the layer's u8 output is q1 = clamp(r + zp_y, lo, 255) and the
// next stub's input g(q1) = clamp(rint(relu((q1 - z1) s1) inv2) + z2, 0, 255)
// (qdq_next_f's fp32 op order).  g is nondecreasing, so on the 256 values of q1
// it can be an exact affine map followed by a clamp: find fp32 (qa, qb) with
// rne(fma(r, qa, qb)) == g(clamp(r + zp_y, lo, 255)) for every r with q1 in
// [lo, 255] (glo = g(lo), ghi = g(255) clamp the rest: fma is monotone in r
// for qa > 0), and check every one of those r in the device's fp32
// arithmetic.  Layers for which no candidate passes keep the general path.
namespace {

float qdq_ref_host(float q1, const ConvEpi& ep) {
  float x = (q1 - (float)ep.z1) * ep.s1;
  x = x > 0.0f ? x : 0.0f;
  const float t = std::fmin(x * ep.inv2, 1.0e9f);
  const float r = std::nearbyint(t) + (float)ep.z2;
  return std::fmin(std::fmax(r, 0.0f), 255.0f);
}

float rne_sat_u8(float x) {   // v_cvt_pk_u8_f32: round half to even, saturate
  const float r = std::nearbyint(x);
  return std::fmin(std::fmax(r, 0.0f), 255.0f);
}

bool qdq_affine_solve(ConvEpi& ep) {
  const int zp = ep.zp_y, lo = ep.lo;
  const int r0 = lo - zp, r1 = 255 - zp;
  if (r0 > r1) return false;
  auto g = [&](int r) {
    const float q1 = std::fmin(std::fmax((float)r + (float)zp, (float)lo), 255.0f);
    return qdq_ref_host(q1, ep);
  };
  const float glo = g(r0), ghi = g(r1);
  const double c = (double)ep.s1 * (double)ep.inv2;
  if (!(c > 0.0) || !std::isfinite(c)) return false;
  for (int k = 0; k < 81; ++k) {   // qa = c (1 + d), d = 0, -1e-7, +1e-7, -2e-7, ...
    const double d = ((k + 1) / 2) * 1.0e-7 * ((k & 1) ? -1.0 : 1.0);
    const float qa = (float)(c * (1.0 + d));
    if (!(qa > 0.0f)) continue;
    double lb = -1.0e30, ub = 1.0e30;
    for (int r = r0; r <= r1; ++r) {
      const double gr = g(r), ar = (double)qa * r;
      if (gr > glo) lb = std::max(lb, gr - 0.5 - ar);
      if (gr < ghi) ub = std::min(ub, gr + 0.5 - ar);
    }
    double mid;
    if (lb > -1.0e29 && ub < 1.0e29) mid = 0.5 * (lb + ub);
    else if (lb > -1.0e29) mid = lb + 0.25;
    else if (ub < 1.0e29) mid = ub - 0.25;
    else mid = (double)glo;
    if (!(lb < ub)) continue;
    const float qb = (float)mid;
    bool ok = true;
    for (int r = r0; r <= r1 && ok; ++r) {
      const float v = std::fmin(std::fmax(std::fma((float)r, qa, qb), glo), ghi);
      ok = rne_sat_u8(v) == g(r);
    }
    if (ok) {
      ep.qa = qa; ep.qb = qb; ep.glo = glo; ep.ghi = ghi;
      return true;
    }
  }
  return false;
}

}  // namespace

// The QDQ hand-off of qcn_qdq_t q into ep (ep.zp_y / ep.lo already set):
// qdq = 2 with the one-fma constants when an exact form exists, else 1.
// Solved once per distinct (layer qparams, next stub) and cached.
void set_qdq(ConvEpi& ep, const qcn_qdq_t* q) {
  ep.qdq = 1;
  ep.s1 = q->s1; ep.z1 = q->z1; ep.inv2 = q->inv2; ep.z2 = q->z2;
  struct Entry { float s1, inv2; int z1, z2, zp, lo; bool ok; float qa, qb, glo, ghi; };
  static thread_local Entry cache[16];
  static thread_local int ncache = 0, next = 0;
  for (int i = 0; i < ncache; ++i) {
    const Entry& e = cache[i];
    if (e.s1 == ep.s1 && e.inv2 == ep.inv2 && e.z1 == ep.z1 && e.z2 == ep.z2 && e.zp == ep.zp_y &&
        e.lo == ep.lo) {
      if (e.ok) { ep.qdq = 2; ep.qa = e.qa; ep.qb = e.qb; ep.glo = e.glo; ep.ghi = e.ghi; }
      return;
    }
  }
  const bool ok = qdq_affine_solve(ep);
  if (ok) ep.qdq = 2;
  cache[next] = Entry{ep.s1, ep.inv2, ep.z1, ep.z2, ep.zp_y, ep.lo, ok, ep.qa, ep.qb, ep.glo, ep.ghi};
  next = (next + 1) % 16;
  if (ncache < 16) ++ncache;
}

}  // namespace qcn

#ifndef QCN_NO_ABI   // (defined only by single-kernel diagnostic translation units)
// ==========================================================================
// C-ABI dispatch
// ==========================================================================
#include "qconvnet_abi.hpp"

namespace {
using namespace qcn;

template <int CIN, int COUT, int HW, bool POOL, int WPX, int PSP = 16, int RPAD = 0,
          int SPAD = 0, bool SPLIT = false, int JT = 4, int RB = 0>
int launch_conv(const uint8_t* x, int nimg, int x_zp, const int8_t* wpk, const ConvEpi& ep,
                uint8_t* y, hipStream_t st) {
  using C = ConvCfg<CIN, COUT, HW, POOL, WPX, PSP, RPAD, SPAD, SPLIT, 2, JT, RB>;
  const long pix = (long)nimg * C::IMG;
  const int grid = (int)((pix + C::PXB - 1) / C::PXB);
  auto k = conv3x3_u8s8_kernel<CIN, COUT, HW, POOL, WPX, PSP, RPAD, SPAD, SPLIT, JT, RB>;
  static bool attr_done[QCN_MAX_DEV] = {};
  if (!qcn_set_lds_once((const void*)k, C::LDS, attr_done)) return QCN_ERR_HIP;
  hipLaunchKernelGGL(k, dim3(grid), dim3(C::NT), C::LDS, st, x, nimg, x_zp, wpk, ep, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

template <class CA, class CB>
int launch_pair(const uint8_t* x, int nimg, int x_zp, const int8_t* wa, const ConvEpi& epa,
                int xb_zp, const int8_t* wb, const ConvEpi& epb, uint8_t* y, hipStream_t st) {
  using P = PairCfg<CA, CB>;
  const long pix = (long)nimg * CA::IMG;
  const int grid = (int)((pix + CA::PXB - 1) / CA::PXB);
  auto k = convpair_kernel<CA, CB>;
  static bool attr_done[QCN_MAX_DEV] = {};
  if (!qcn_set_lds_once((const void*)k, P::LDS, attr_done)) return QCN_ERR_HIP;
  hipLaunchKernelGGL(k, dim3(grid), dim3(CA::NT), P::LDS, st, x, nimg, x_zp, wa, epa, xb_zp, wb, epb, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

template <class CA, class CB, int D>
int launch_pair_ga(const uint8_t* x, int nimg, int x_zp, const int8_t* wa, const ConvEpi& epa,
                   int xb_zp, const int8_t* wb, const ConvEpi& epb, uint8_t* y, hipStream_t st) {
  using P = PairGaCfg<CA, CB>;
  const long pix = (long)nimg * CA::IMG;
  const int grid = (int)((pix + CA::PXB - 1) / CA::PXB);
  auto k = convpair_ga_kernel<CA, CB, D>;
  static bool attr_done[QCN_MAX_DEV] = {};
  if (!qcn_set_lds_once((const void*)k, P::LDS, attr_done)) return QCN_ERR_HIP;
  hipLaunchKernelGGL(k, dim3(grid), dim3(CA::NT), P::LDS, st, x, nimg, x_zp, wa, epa, xb_zp, wb, epb, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

template <class CA, class CB, int D, int FA, int FB, bool KM>
int launch_pair_ws_k(const uint8_t* x, int nimg, int x_zp, const int8_t* wa, const ConvEpi& epa, int xb_zp,
                     const int8_t* wb, const ConvEpi& epb, uint8_t* y, hipStream_t st, int ncu) {
  using P = PairWs<CA, CB, D>;
  auto k = convpair_ws_kernel<CA, CB, D, FA, FB, KM>;
  static bool attr_done[QCN_MAX_DEV] = {};
  if (!qcn_set_lds_once((const void*)k, P::LDS, attr_done)) return QCN_ERR_HIP;
  const int ntile = (nimg + P::SEGS - 1) / P::SEGS;
  const int grid = ntile < ncu ? ntile : ncu;   // persistent: one workgroup per CU
  hipLaunchKernelGGL(k, dim3(grid), dim3(512), P::LDS, st, x, nimg, x_zp, wa, epa, xb_zp, wb, epb, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

template <class CA, class CB, int FA, int FB, bool KM>
int launch_pair_ws16_k(const uint8_t* x, int nimg, int x_zp, const int8_t* wa, const ConvEpi& epa, int xb_zp,
                       const int8_t* wb, const ConvEpi& epb, uint8_t* y, hipStream_t st, int ncu) {
  using P = PairWs16<CA, CB>;
  auto k = convpair_ws16_kernel<CA, CB, FA, FB, KM>;
  static bool attr_done[QCN_MAX_DEV] = {};
  if (!qcn_set_lds_once((const void*)k, P::LDS, attr_done)) return QCN_ERR_HIP;
  const int ntile = (nimg + P::SEGS - 1) / P::SEGS;
  const int grid = ntile < ncu ? ntile : ncu;   // persistent: one workgroup per CU
  hipLaunchKernelGGL(k, dim3(grid), dim3(512), P::LDS, st, x, nimg, x_zp, wa, epa, xb_zp, wb, epb, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

template <class CA, class CB, int D, class CA16 = void, class CB16 = void>
int launch_pair_ws(const uint8_t* x, int nimg, int x_zp, const int8_t* wa, const ConvEpi& epa, int xb_zp,
                   const int8_t* wb, const ConvEpi& epb, bool kmajor, uint8_t* y, hipStream_t st, int ncu) {
  // epilogue modes, known on the host: 1 the FBGEMM fast path (zp_y == 0, no
  // floor, no QDQ hand-off), 2 the one-fma QDQ form (both convs: the QDQ
  // net), 0 general
  int fa = epi_mode(epa), fb = epi_mode(epb);
  if ((fa == 2) != (fb == 2)) { fa = fa == 2 ? 0 : fa; fb = fb == 2 ? 0 : fb; }
  // the 16x16 forms for the two epilogue pairs the nets use (both convs on
  // the FBGEMM fast path, or both on the one-fma QDQ form); mixed forms stay
  // on the 32x32 kernel (results are identical: exact integer arithmetic)
  if constexpr (!std::is_void_v<CA16>) {
#define QCN_WS16(FA_, FB_, KM_)                                                                      \
  if (fa == FA_ && fb == FB_ && kmajor == KM_)                                                       \
    return launch_pair_ws16_k<CA16, CB16, FA_, FB_, KM_>(x, nimg, x_zp, wa, epa, xb_zp, wb, epb, y, st, ncu);
    QCN_WS16(1, 1, false) QCN_WS16(2, 2, false) QCN_WS16(1, 1, true) QCN_WS16(2, 2, true)
#undef QCN_WS16
  }
#define QCN_WS(FA_, FB_, KM_) \
  if (fa == FA_ && fb == FB_ && kmajor == KM_)                                                            \
    return launch_pair_ws_k<CA, CB, D, FA_, FB_, KM_>(x, nimg, x_zp, wa, epa, xb_zp, wb, epb, y, st, ncu);
  QCN_WS(1, 1, false) QCN_WS(1, 0, false) QCN_WS(0, 1, false) QCN_WS(0, 0, false) QCN_WS(2, 2, false)
  QCN_WS(1, 1, true) QCN_WS(1, 0, true) QCN_WS(0, 1, true) QCN_WS(0, 0, true) QCN_WS(2, 2, true)
#undef QCN_WS
  return QCN_ERR_UNSUPPORTED;
}

template <class CA, class CB, int D, int COUTB>
int launch_pair_ga_split(const uint8_t* x, int nimg, int x_zp, const int8_t* wa, const ConvEpi& epa,
                         int xb_zp, const int8_t* wb, const ConvEpi& epb, uint8_t* y, hipStream_t st) {
  using P = PairGaCfg<CA, CB>;
  const long pix = (long)nimg * CA::IMG;
  const int grid = (int)((pix + CA::PXB - 1) / CA::PXB) * (COUTB / CB::kCout);
  auto k = convpair_ga_split_kernel<CA, CB, D, COUTB>;
  static bool attr_done[QCN_MAX_DEV] = {};
  if (!qcn_set_lds_once((const void*)k, P::LDS, attr_done)) return QCN_ERR_HIP;
  hipLaunchKernelGGL(k, dim3(grid), dim3(CA::NT), P::LDS, st, x, nimg, x_zp, wa, epa, xb_zp, wb, epb, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

// Tuned instantiations: the SimpleConvNet layers and the
// small shapes the parity fixtures use.
int dispatch_conv(int cin, int cout, int hw, int pool, const uint8_t* x, int nimg, int x_zp,
                  const int8_t* wpk, const ConvEpi& ep, uint8_t* y, hipStream_t st) {
#define QCN_CONV_CASE(CI, CO, HWV, PL, WPXV, ...)                                      \
  if (cin == CI && cout == CO && hw == HWV && pool == PL)                              \
    return launch_conv<CI, CO, HWV, PL, WPXV, ##__VA_ARGS__>(x, nimg, x_zp, wpk, ep, y, st);
  //            cin  cout hw pool wpx | PSP RPAD SPAD SPLIT (bank-conflict-free layouts)
  QCN_CONV_CASE(64, 64, 32, 1, 4, 16, 96, 0, true)
  // ResNet-50 layer1 3x3 (56x56, 64 -> 64): bands of 8 rows (448 pixels, 7
  // waves of 64 couts x 64 pixels); RPAD 96 keeps the row-wrapping B reads
  // conflict-free (row stride 296 x 16 B == 0 mod 16 slots past 56 pixels)
  QCN_CONV_CASE(64, 64, 56, 0, 7, 16, 96, 0, false, 2)
  // ResNet-50 layer2 3x3 (28x28, 128 -> 128): bands of 16 flattened rows
  // (448 pixels, 14 waves), each image part with its own halo rows; RPAD 224
  // keeps row wraps conflict-free (a wrap across images costs one 2-way read)
  QCN_CONV_CASE(128, 128, 28, 0, 7, 16, 224, 0, false, 2, 16)
  QCN_CONV_CASE(64, 64, 32, 0, 4, 16, 0, 0, false)
  QCN_CONV_CASE(64, 128, 16, 0, 2, 16, 96, 0, false)
  QCN_CONV_CASE(128, 128, 16, 1, 2, 16, 32, 0, true)
  QCN_CONV_CASE(128, 128, 16, 0, 2, 16, 32, 0, false)
  QCN_CONV_CASE(128, 256, 8, 0, 2, 16, 224, 0, false)
  QCN_CONV_CASE(256, 256, 8, 1, 2, 16, 32, 64, true)
  QCN_CONV_CASE(256, 256, 8, 0, 2, 16, 32, 64, false)
  QCN_CONV_CASE(64, 64, 16, 0, 2, 16, 96, 0, false)
  QCN_CONV_CASE(64, 64, 16, 1, 2, 16, 96, 0, true)
  QCN_CONV_CASE(64, 64, 8, 0, 1, 16, 96, 0, false)
  QCN_CONV_CASE(64, 64, 8, 1, 2, 16, 96, 0, true)
  QCN_CONV_CASE(64, 128, 8, 0, 1, 16, 96, 0, false)
  QCN_CONV_CASE(128, 256, 4, 0, 2, 16, 32, 64, false)
  QCN_CONV_CASE(256, 256, 4, 0, 1, 16, 32, 64, false)
  QCN_CONV_CASE(256, 256, 4, 1, 1, 16, 0, 0, false)
#undef QCN_CONV_CASE
  return QCN_ERR_UNSUPPORTED;
}
}  // namespace

extern "C" {

#ifdef QCN_PIPE34_STAMP
int qcn_diag_p34_stamps(int kind, unsigned long long* host, int nwg) {
  if (!host || nwg <= 0 || nwg > 1024 || kind < 0 || kind > 1) return QCN_ERR_ARG;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(qcn::g_p34_stamp), (size_t)nwg * 64 * 8,
                             (size_t)kind * 1024 * 64 * 8, hipMemcpyDeviceToHost) == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}
#endif

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

int qcn_qdq_affine(const qcn_qdq_t* q, int y_zp, int lo, float* out) {
  if (!q || !out || y_zp < 0 || y_zp > 255 || lo < 0 || lo > 255) return QCN_ERR_ARG;
  qcn::ConvEpi ep{};
  ep.zp_y = y_zp;
  ep.lo = lo;
  qcn::set_qdq(ep, q);
  if (ep.qdq != 2) return 0;
  out[0] = ep.qa; out[1] = ep.qb; out[2] = ep.glo; out[3] = ep.ghi;
  return 1;
}

int qcn_conv3x3_pair_u8s8(const uint8_t* x, int nimg, int hw, int cin, int x_zp,
                          const int8_t* wa_packed, int cmid, const float* ua, const float* va,
                          const float* multa, const int32_t* corra, int zmid, int relua,
                          const qcn_qdq_t* qdqa, const int8_t* wb_packed, int cout, const float* ub,
                          const float* vb, const float* multb, const int32_t* corrb, int y_zp,
                          int relub, const qcn_qdq_t* qdqb, int kmajor, uint8_t* y, void* stream) {
  if (!x || !wa_packed || !ua || !va || !multa || !corra || !wb_packed || !ub || !vb || !multb ||
      !corrb || !y)
    return QCN_ERR_ARG;
  if (nimg <= 0 || hw <= 0 || x_zp < 0 || x_zp > 255 || zmid < 0 || zmid > 255 || y_zp < 0 ||
      y_zp > 255)
    return QCN_ERR_ARG;
  ConvEpi epa{ua, va, multa, corra, zmid, relua ? zmid : 0, 0, 0.f, 0, 0.f, 0, 0};
  int xb_zp = zmid;
  if (qdqa) {
    qcn::set_qdq(epa, qdqa);
    xb_zp = qdqa->z2;
  }
  if (kmajor && (long)nimg * 4096 > 0x7fffffffL) return QCN_ERR_UNSUPPORTED;   // 32-bit store offsets
  ConvEpi epb{ub, vb, multb, corrb, y_zp, relub ? y_zp : 0, 0, 0.f, 0, 0.f, 0, kmajor ? 1 : 0};
  if (qdqb) qcn::set_qdq(epb, qdqb);
  hipStream_t st = (hipStream_t)stream;
  using namespace qcn;
  // wave tile: 64 couts x 128 pixels, two waves per SIMD (two workgroups per
  // CU for conv3+conv4).  ConvCfg's WI = 4 (128 x 128 tiles, one wave per
  // SIMD, a third fewer LDS bytes per MFMA) measured slower with no partner
  // wave to cover the epilogues (63 vs 53 us, 56 vs 51 us) and is not built.
  const int ncu = qcn_cu_count();
  if (ncu <= 0) return QCN_ERR_HIP;
  if (hw == 16 && cin == 64 && cmid == 128 && cout == 128) {
    // one image per CU or fewer (config 2): eight waves per image — conv3 as
    // 64-cout x 64-pixel wave tiles, conv4 as 32-cout x 128-pixel tiles — so
    // each SIMD holds two waves of the image's work instead of one
    if (nimg <= ncu)
      return launch_pair<SmA3, SmB4>(
          x, nimg, x_zp, wa_packed, epa, xb_zp, wb_packed, epb, y, st);
    using A3 = WsA3;
    using B4 = WsB4;
    // two or more images per CU: the persistent wave-specialised kernel
    if (nimg >= 2 * ncu)
      return launch_pair_ws<A3, B4, kPipeD, W16A3, W16B4>(x, nimg, x_zp, wa_packed, epa, xb_zp,
                                                          wb_packed, epb, kmajor != 0, y, st, ncu);
    return launch_pair<A3, B4>(x, nimg, x_zp, wa_packed, epa, xb_zp, wb_packed, epb, y, st);
  }
  if (hw == 8 && cin == 128 && cmid == 256 && cout == 256) {
    // two images per 4-wave workgroup, two workgroups per CU, weights from L2
    // into registers 4 K-steps ahead (convpair_ga_kernel)
    using A1 = WsA5;
    using B1 = WsB6;
    // default: conv6's couts split over two 4-wave workgroups per image pair,
    // each computing all of conv5 (4/3 of the MFMAs, half the weight bytes per
    // image)
    if (nimg <= ncu)
      return launch_pair_ga_split<A1, ConvCfg<256, 128, 8, true, 1, 16, 32, 64, true, 1>, 4, 256>(
          x, nimg, x_zp, wa_packed, epa, xb_zp, wb_packed, epb, y, st);
    // two or more image pairs per CU: the persistent wave-specialised kernel
    if (nimg >= 4 * ncu)
      return launch_pair_ws<A1, B1, kPipeD, W16A5, W16B6>(x, nimg, x_zp, wa_packed, epa, xb_zp,
                                                          wb_packed, epb, kmajor != 0, y, st, ncu);
    return launch_pair_ga<A1, B1, 4>(x, nimg, x_zp, wa_packed, epa, xb_zp, wb_packed, epb, y, st);
  }
  return QCN_ERR_UNSUPPORTED;
}

int qcn_conv3x3_u8s8_kmajor(const uint8_t* x, int nimg, int h, int w, int cin, int x_zp,
                            const int8_t* w_packed, int cout, const float* u, const float* v,
                            const float* mult, const int32_t* corr, int y_zp, int relu, int pool,
                            uint8_t* y, void* stream) {
  if (!x || !w_packed || !u || !v || !mult || !corr || !y) return QCN_ERR_ARG;
  if (nimg <= 0 || h <= 0 || w <= 0 || cin <= 0 || cout <= 0) return QCN_ERR_ARG;
  if (x_zp < 0 || x_zp > 255 || y_zp < 0 || y_zp > 255) return QCN_ERR_ARG;
  if (pool && ((h & 1) || (w & 1))) return QCN_ERR_ARG;
  // whole images per workgroup: the 8x8 -> 4x4 and 8x8 layers of the net
  if (!(h == 8 && w == 8 && cin % 64 == 0 && cout == 256)) return QCN_ERR_UNSUPPORTED;
  if ((long)nimg * 4096 > 0x7fffffffL) return QCN_ERR_UNSUPPORTED;   // 32-bit store offsets
  ConvEpi ep{u, v, mult, corr, y_zp, relu ? y_zp : 0, 0, 0.f, 0, 0.f, 0, 1};
  return dispatch_conv(cin, cout, h, pool, x, nimg, x_zp, w_packed, ep, y, (hipStream_t)stream);
}

int qcn_conv3x3_u8s8_nhwc(const uint8_t* x, int nimg, int h, int w, int cin, int x_zp,
                          const int8_t* w_packed, int cout, const float* u, const float* v,
                          const float* mult, const int32_t* corr, int y_zp, int relu, int pool,
                          const qcn_qdq_t* qdq, uint8_t* y, void* stream) {
  if (!x || !w_packed || !u || !v || !mult || !corr || !y) return QCN_ERR_ARG;
  if (nimg <= 0 || h <= 0 || w <= 0 || cin <= 0 || cout <= 0) return QCN_ERR_ARG;
  if (x_zp < 0 || x_zp > 255 || y_zp < 0 || y_zp > 255) return QCN_ERR_ARG;
  if (pool && ((h & 1) || (w & 1))) return QCN_ERR_ARG;
  ConvEpi ep{u, v, mult, corr, y_zp, relu ? y_zp : 0, 0, 0.f, 0, 0.f, 0, 0};
  if (qdq) qcn::set_qdq(ep, qdq);
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

int qcn_conv12_fused_f32_nchw(const float* x, int nimg, float in_scale, int in_zp,
                              const int8_t* w1_packed, const float* u1, const float* v1,
                              const float* mult1, const int32_t* corr1, int z1, int relu1,
                              const qcn_qdq_t* qdq1, int x2_zp, const int8_t* w2_packed,
                              const float* u2, const float* v2, const float* mult2,
                              const int32_t* corr2, int y_zp, int relu2, const qcn_qdq_t* qdq2,
                              uint8_t* y, void* stream) {
  if (!x || !w1_packed || !u1 || !v1 || !mult1 || !corr1 || !w2_packed || !u2 || !v2 || !mult2 ||
      !corr2 || !y)
    return QCN_ERR_ARG;
  if (nimg <= 0 || in_zp < 0 || in_zp > 255 || !(in_scale > 0.f) || x2_zp < 0 || x2_zp > 255 ||
      y_zp < 0 || y_zp > 255 || z1 < 0 || z1 > 255)
    return QCN_ERR_ARG;
  ConvEpi ep1{u1, v1, mult1, corr1, z1, relu1 ? z1 : 0, 0, 0.f, 0, 0.f, 0, 0};
  if (qdq1) qcn::set_qdq(ep1, qdq1);
  ConvEpi ep2{u2, v2, mult2, corr2, y_zp, relu2 ? y_zp : 0, 0, 0.f, 0, 0.f, 0, 0};
  if (qdq2) qcn::set_qdq(ep2, qdq2);
  static bool attr_done[QCN_MAX_DEV] = {};
  static int ncu_dev[QCN_MAX_DEV] = {};
  if (!qcn_set_lds_once((const void*)qcn::conv12p_kernel, qcn::Conv12P::LDS, attr_done))
    return QCN_ERR_HIP;
  const int dev = qcn_current_device();
  int& ncu = ncu_dev[dev];
  if (!ncu && (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
               ncu <= 0)) {
    ncu = 0;
    return QCN_ERR_HIP;
  }
  const int grid = nimg < ncu ? nimg : ncu;   // persistent: one workgroup per CU
  hipLaunchKernelGGL(qcn::conv12p_kernel, dim3(grid), dim3(512), qcn::Conv12P::LDS,
                     (hipStream_t)stream, x, nimg, 1.0f / in_scale, in_zp, w1_packed, ep1, x2_zp,
                     w2_packed, ep2, y);
  return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
}

}  // extern "C"

namespace {
// The form qcn_convnet_convs_f32_nchw takes (shared with the host query
// qcn_convnet_convs_form): fills L and the epilogue mode em and returns 1 (one
// image per workgroup), 2 (persistent) or the error the launch returns.
int convnet_convs_plan(int nimg, float in_scale, int in_zp, const qcn_conv_layer_t* layers, int kmajor,
                       qcn::ConvnetLayers& L, int& em, int& ncu) {
  if (!layers) return QCN_ERR_ARG;
  if (nimg <= 0 || in_zp < 0 || in_zp > 255 || !(in_scale > 0.f)) return QCN_ERR_ARG;
  L = qcn::ConvnetLayers{};
  for (int i = 0; i < 6; ++i) {
    const qcn_conv_layer_t& l = layers[i];
    if (!l.w || !l.u || !l.v || !l.mult || !l.corr) return QCN_ERR_ARG;
    if (l.x_zp < 0 || l.x_zp > 255 || l.y_zp < 0 || l.y_zp > 255) return QCN_ERR_ARG;
    // conv i reads conv i-1's output: its input zero point is that layer's
    // output zero point, or the z2 of that layer's QDQ hand-off
    if (i > 0 && l.x_zp != (layers[i - 1].qdq ? layers[i - 1].qdq->z2 : layers[i - 1].y_zp)) return QCN_ERR_ARG;
    L.w[i] = l.w;
    L.ep[i] = qcn::ConvEpi{l.u, l.v, l.mult, l.corr, l.y_zp, l.relu ? l.y_zp : 0, 0, 0.f, 0, 0.f, 0, 0};
    if (l.qdq) qcn::set_qdq(L.ep[i], l.qdq);
    L.x_zp[i] = l.x_zp;
  }
  if (L.x_zp[0] != in_zp) return QCN_ERR_ARG;
  L.ep[5].kmajor = kmajor ? 1 : 0;
  if ((long)nimg * 4096 > 0x7fffffffL) return QCN_ERR_UNSUPPORTED;   // 32-bit store offsets
  ncu = qcn_cu_count();
  if (ncu <= 0) return QCN_ERR_HIP;
  if (nimg <= ncu) return 1;   // one image per workgroup
  // the two pair phases are the wave-specialised kernels of >= 4 images per CU;
  // conv3..conv6 all on the FBGEMM fast epilogue or all on the one-fma QDQ form
  if (nimg < 4 * ncu) return QCN_ERR_UNSUPPORTED;
  bool all1 = true, all2 = true;
  for (int i = 2; i < 6; ++i) {
    all1 = all1 && qcn::epi_mode(L.ep[i]) == 1;
    all2 = all2 && qcn::epi_mode(L.ep[i]) == 2;
  }
  if (all1) em = 1;
  else if (all2) em = 2;
  else return QCN_ERR_UNSUPPORTED;
  return 2;
}
}  // namespace

extern "C" {

int qcn_convnet_convs_form(int nimg, float in_scale, int in_zp, const qcn_conv_layer_t* layers, int kmajor) {
  qcn::ConvnetLayers L;
  int em = 0, ncu = 0;
  return convnet_convs_plan(nimg, in_scale, in_zp, layers, kmajor, L, em, ncu);
}

int qcn_convnet_convs_f32_nchw(const float* x, int nimg, float in_scale, int in_zp,
                               const qcn_conv_layer_t* layers, uint8_t* a2, uint8_t* a4, uint8_t* a6,
                               int kmajor, void* stream) {
  if (!x || !layers || !a2 || !a4 || !a6) return QCN_ERR_ARG;
  qcn::ConvnetLayers L;
  int em = 0, ncu = 0;
  const int form = convnet_convs_plan(nimg, in_scale, in_zp, layers, kmajor, L, em, ncu);
  if (form < 0) return form;
  const float inv = 1.0f / in_scale;
  if (form == 1) {   // one image per workgroup
    static bool sm_done[QCN_MAX_DEV] = {};
    if (!qcn_set_lds_once((const void*)qcn::convnet_convs_sm_kernel, qcn::kConvnetSmLds, sm_done))
      return QCN_ERR_HIP;
    hipLaunchKernelGGL(qcn::convnet_convs_sm_kernel, dim3(nimg), dim3(512), qcn::kConvnetSmLds,
                       (hipStream_t)stream, x, nimg, inv, QCN_C16_ARGS(L), a2, a4, a6);
    return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;
  }
  static bool attr_done[4][QCN_MAX_DEV] = {};
#define QCN_C16_KERNEL qcn::convnet_convs16_kernel
#define QCN_C16_LDS qcn::kConvnet16Lds
#define QCN_C16(EM_, KM_)                                                                          \
  if (em == EM_ && (kmajor != 0) == KM_) {                                                         \
    auto k = QCN_C16_KERNEL<EM_, KM_>;                                                             \
    if (!qcn_set_lds_once((const void*)k, QCN_C16_LDS, attr_done[(EM_ - 1) * 2 + KM_]))            \
      return QCN_ERR_HIP;                                                                          \
    hipLaunchKernelGGL(k, dim3(ncu), dim3(512), QCN_C16_LDS, (hipStream_t)stream, x, nimg, inv,    \
                       QCN_C16_ARGS(L), a2, a4, a6);                                               \
    return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;                                 \
  }
  QCN_C16(1, true) QCN_C16(1, false) QCN_C16(2, true) QCN_C16(2, false)
#undef QCN_C16
#undef QCN_C16_KERNEL
#undef QCN_C16_LDS
  return QCN_ERR_UNSUPPORTED;
}

int qcn_conv1_f32_nchw(const float* x, int nimg, int hw, float in_scale, int in_zp,
                       const int8_t* w1_packed, const float* u, const float* v, const float* mult,
                       const int32_t* corr, int y_zp, int relu, const qcn_qdq_t* qdq, uint8_t* y,
                       uint8_t* q_in, void* stream) {
  if (!x || !w1_packed || !u || !v || !mult || !corr || !y) return QCN_ERR_ARG;
  if (nimg <= 0 || in_zp < 0 || in_zp > 255 || !(in_scale > 0.f)) return QCN_ERR_ARG;
  ConvEpi ep{u, v, mult, corr, y_zp, relu ? y_zp : 0, 0, 0.f, 0, 0.f, 0, 0};
  if (qdq) qcn::set_qdq(ep, qdq);
  const float inv = 1.0f / in_scale;
  hipStream_t st = (hipStream_t)stream;
  const long pix = (long)nimg * hw * hw;
  const int grid = (int)((pix + 511) / 512);
#define QCN_C1(HWV)                                                                       \
  if (hw == HWV) {                                                                        \
    constexpr int R = (HWV * HWV >= 512) ? 512 / HWV : HWV;                              \
    constexpr int SEGS = (HWV * HWV >= 512) ? 1 : 512 / (HWV * HWV);                     \
    constexpr int LDS0 = ((SEGS * 3 * (R + 2) * (HWV + 2) + 15) / 16 * 16) + 512 * 48;    \
    constexpr int LDS = LDS0 > 512 * 80 ? LDS0 : 512 * 80;                                \
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
#endif  // QCN_NO_ABI
