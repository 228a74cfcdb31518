// conv3 .. conv6 of SimpleConvNet in ONE persistent launch with one wave per
// SIMD (r06): 256-thread workgroups, so each wave has the 512-register budget
// and computes a 64-cout x 256-pixel tile (the 256 int32 accumulators in
// AGPRs).  Every weight byte a wave streams from L2 then serves 256 pixels
// instead of 128: half the L2 -> VGPR bytes per MAC of the two-waves-per-SIMD
// pair kernels (convpair_ws16_body, conv3x3.hip), whose weight stream cost
// 13-16 % of their cycles (profiles/r05_diag_pair_weight_stream_probe.txt); the
// bare main loop of this shape held a 7 % higher clock under load
// (profiles/r05_diag_wave_tile_probe.txt).
//
// Reference semantics: the conv3..conv6 blocks of SimpleConvNet
// (/root/reference/models/baseline_model.py:20-33, forward :64-75) as
// torch.ao's fbgemm QuantizedConvReLU2d + MaxPool2d run them (SURVEY §8(a)
// rows A5, A6, A10); numerics exactly those of conv3x3.hip (conv_epi.hpp).
//
// Schedule.  Workgroup b of G (one per CU) owns images b, b + G, b + 2G, ...
// (the images conv12p wrote for it).  Phase 1 (conv3 + conv4) takes them two
// at a time, phase 2 (conv5 + conv6) four at a time; per tile:
//   stage the tile's input (halos + interior, from registers) into patch A,
//   barrier; conv A over patch A -> acc; barrier; A's requant into patch B
//   (conv B's input, which aliases patch A), barrier; conv B -> acc; barrier;
//   B's pooled requant -> global (a4, or a6 chunk-major for the classifier).
// The next tile's input loads are issued before conv A and held in registers.
// a4 passes from phase 1 to phase 2 through memory inside the workgroup
// (write-through stores drained before the phase barrier; this CU never read
// those addresses before, so its L1 holds no stale copy).
//
// Wave tile.  Wave w: cout block wc = w % WCO (64 couts), pixel slot
// wp = w / WCO (256 pixels = 16 blocks of 16).  One K-step is one 64-byte
// chunk (a tap's 64 input channels): 4 A fragments (weights, 1 KiB each, from
// L2 into registers, issued one K-step ahead) and 16 B fragments (the patch,
// ds_read_b128, each read right after its block's last MFMA of the previous
// step), 64 v_mfma_i32_16x16x64_i8.  Lane l = (p = l % 16, g = l / 16): A row
// 16 i + p, B pixel p of block j, K bytes 16 g .. 16 g + 15; acc[i][j][r] is
// cout 16 i + 4 g + r of pixel p of block j.  Pooled conv B: block
// j = 4 gq + jq is quadrant jq of pooled pixels 16 gq .. 16 gq + 15.  Patch
// layouts are the 16x16 conflict-free ones of the pair kernels
// (tools/lds_banks.py): a block's 16 pixels sit in the same relative
// positions here.
#include "common.hpp"
#include "conv_epi.hpp"
#include <type_traits>

namespace qcn {

// Input patch of one conv for a W4 tile: SEGS images of HW x HW, each padded
// to (HW + 2)^2 pixels of PS = CIN + PSP bytes, RPAD bytes per row; SPLIT
// stores even patch columns before odd ones (pooled convs read stride 2).
template <int CIN, int COUT, int HW, bool POOL, int SEGS_, int PSP, int RPAD, bool SPLIT>
struct W4Cfg {
  static constexpr int kCin = CIN, kCout = COUT, H = HW, W = HW, SEGS = SEGS_;
  static constexpr bool kPool = POOL, kSplit = SPLIT;
  static constexpr int IMG = H * W;
  static constexpr int WCO = COUT / 64;          // waves along cout
  static constexpr int WPX = 4 / WCO;            // waves along the pixels
  static_assert(WCO * WPX == 4 && SEGS * IMG == WPX * 256, "four waves of 64 couts x 256 pixels");
  static constexpr int PS = CIN + PSP, PCOLS = W + 2, PROWS = H + 2, HALF = (PCOLS + 1) / 2;
  static constexpr int RS = PCOLS * PS + RPAD, SS = PROWS * RS;
  static constexpr int PATCH = SEGS * SS;
  static constexpr int WBUF = COUT * 64;         // one K-chunk of packed weights
  static constexpr int NCH = 9 * CIN / 64;       // K-steps
  static constexpr int OPX = POOL ? SEGS * IMG / 4 : SEGS * IMG;   // output pixels per tile
  static_assert(CIN % 64 == 0 && PSP % 16 == 0 && RPAD % 16 == 0, "16-B aligned layout");
  static_assert(!SPLIT || POOL, "parity-split columns need pooled tiles");
  static constexpr int slot(int seg, int prow, int pcol) {
    const int cpos = SPLIT ? ((pcol & 1) * HALF + (pcol >> 1)) : pcol;
    return seg * SS + prow * RS + cpos * PS;
  }
  // tap (0, 0) patch slot of lane pixel p of block j of pixel slot wp
  static constexpr int at(int wp, int j, int p) {
    if (POOL) {
      constexpr int PW = W / 2, PH = H / 2;
      const int q = wp * 64 + (j >> 2) * 16 + p, jq = j & 3;
      return slot(q / (PH * PW), 2 * ((q / PW) % PH) + (jq >> 1), 2 * (q % PW) + (jq & 1));
    }
    const int m = (wp * 16 + j) * 16 + p;
    return slot(m / IMG, (m / W) % H, m % W);
  }
  // (conv A) output pixel of block j as an interior slot of the next conv's patch N
  template <class N>
  static constexpr int out_at(int wp, int j, int p) {
    const int m = (wp * 16 + j) * 16 + p;
    return N::slot(m / IMG, (m / W) % H + 1, m % W + 1);
  }
  static constexpr int jofs(int j) { return at(0, j, 0) - at(0, 0, 0); }
  template <class N>
  static constexpr int out_jofs(int j) { return out_at<N>(0, j, 0) - out_at<N>(0, 0, 0); }
  static constexpr bool affine() {
    for (int wp = 0; wp < WPX; ++wp)
      for (int j = 0; j < 16; ++j)
        for (int p = 0; p < 16; ++p)
          if (at(wp, j, p) != at(wp, 0, p) + jofs(j)) return false;
    return true;
  }
  template <class N>
  static constexpr bool out_affine() {
    for (int wp = 0; wp < WPX; ++wp)
      for (int j = 0; j < 16; ++j)
        for (int p = 0; p < 16; ++p)
          if (out_at<N>(wp, j, p) != out_at<N>(wp, 0, p) + out_jofs<N>(j)) return false;
    return true;
  }
  // patch offset of tap (r, s) relative to tap (0, 0); with parity-split
  // columns the column step depends on the pixel column's parity (j & 1)
  static constexpr int delta(int tap, int j) {
    const int r = tap / 3, s = tap % 3;
    int dc = s;
    if (SPLIT) dc = s == 0 ? 0 : (s == 2 ? 1 : ((j & 1) ? 1 - HALF : HALF));
    return r * RS + dc * PS;
  }
};

// the pair phases' layouts (the pair kernels' W16A3 / W16B4 / W16A5 / W16B6)
using W4A3 = W4Cfg<64, 128, 16, false, 2, 32, 0, false>;
using W4B4 = W4Cfg<128, 128, 16, true, 2, 32, 64, true>;
using W4A5 = W4Cfg<128, 256, 8, false, 4, 32, 192, false>;
using W4B6 = W4Cfg<256, 256, 8, true, 4, 32, 0, true>;

template <class CA, class CB>
struct W4Pair {
  static_assert(!CA::kPool && CB::kPool && CA::kCout == CB::kCin && CA::kCout == CB::kCout, "A feeds B");
  static_assert(CA::SEGS == CB::SEGS && CA::H == CB::H && CA::WCO == CB::WCO, "same tiles");
  static_assert(CA::affine() && CB::affine() && CA::template out_affine<CB>(), "blocks at constant offsets");
  static constexpr int SEGS = CA::SEGS, IMG = CA::IMG, COUT = CA::kCout;
  static constexpr int CH16 = CA::kCin / 16;                 // 16-B pieces per input pixel
  static_assert(SEGS * IMG * CA::kCin == 8 * 256 * 16, "eight 16-B staging pieces per thread");
  // LDS: the epilogue tables, patch B after them, patch A at the END of the
  // workgroup's 160 KiB.  The two patches overlap where they do not both fit:
  // A is dead once every wave's conv A loop has passed a barrier, B once conv
  // B's has.  Conv A's requant writes its pixel blocks straight into patch B
  // except the blocks whose bytes fall in the overlap (HOLD), which stay in
  // registers until that barrier; both patches' halos are rewritten per tile.
  static constexpr int OFF_EA = 0;                           // u | v | mult of conv A, fp32 x COUT each
  static constexpr int OFF_EB = OFF_EA + 12 * COUT;
  static constexpr int OFF_CA = OFF_EB + 12 * COUT;          // corr, int32 x COUT
  static constexpr int OFF_CB = OFF_CA + 4 * COUT;
  static constexpr int OFF_PB = OFF_CB + 4 * COUT;
  static constexpr int LDS = 160 * 1024;
  static constexpr int OFF_PA = (LDS - CA::PATCH) / 16 * 16;
  static_assert(OFF_PB + CB::PATCH <= LDS && OFF_PA >= OFF_PB, "LDS budget");
  // does any byte conv A's requant writes for pixel block j (any wave, lane,
  // cout block) fall inside patch A?
  static constexpr bool held(int j) {
    for (int wp = 0; wp < CA::WPX; ++wp)
      for (int p = 0; p < 16; ++p)
        for (int c = 0; c < COUT; c += 4) {
          const int o = OFF_PB + CA::template out_at<CB>(wp, j, p) + c;
          if (o + 4 > OFF_PA) return true;
        }
    return false;
  }
  static constexpr int nheld() {
    int n = 0;
    for (int j = 0; j < 16; ++j) n += held(j);
    return n;
  }
  static constexpr int OPI = IMG / 4;                        // pooled output pixels per image
};

constexpr int w4max(int a, int b) { return a > b ? a : b; }
constexpr int kW4Lds = 160 * 1024;
static_assert(W4Pair<W4A3, W4B4>::LDS == kW4Lds && W4Pair<W4A5, W4B6>::LDS == kW4Lds, "one LDS plan");

// Diagnostic builds only (tools/clock: -DQCN_W4_STAMP): s_memtime of lane 0
// of wave 0 at the phase start and after each step of every tile, plain
// vector stores into a buffer nothing else reads.  The product library
// compiles none of it.
#ifdef QCN_W4_STAMP
__device__ unsigned long long g_w4_stamp[4096][2][32];   // s_memtime
__device__ unsigned long long g_w4_rt[4096][2][2];       // s_memrealtime at phase start / end
QCN_DEV void w4_stamp(int ph, int idx) {
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  const unsigned lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if ((threadIdx.x >> 6) == 0 && lane == 0 && blockIdx.x < 4096 && idx < 32) {
    volatile unsigned long long* d = &g_w4_stamp[blockIdx.x][ph][idx];
    *d = t + lane;
  }
}
QCN_DEV void w4_rt(int ph, int idx) {
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  const unsigned lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if ((threadIdx.x >> 6) == 0 && lane == 0 && blockIdx.x < 4096) {
    volatile unsigned long long* d = &g_w4_rt[blockIdx.x][ph][idx];
    *d = t + lane;
  }
}
#define W4_RT(i) w4_rt(PH, (i))
#define W4_STAMP(i) w4_stamp(PH, (i))
#else
#define W4_STAMP(i)
#define W4_RT(i)
#endif

// The MFMA as inline asm with the accumulator TIED in place ("+a"): with the
// builtin the register allocator rotates the 256 accumulators between AGPR
// tuples around the last K-step (dst != srcC needs a spare tuple) and spills.
// The hazard recognizer does not see these: every VALU read of a result is
// placed behind mfma_drain(); dependent MFMAs on one tuple are 64 apart.
QCN_DEV void mfma_acc(v4i& c, const v4i& a, const v4i& b) {
  asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
QCN_DEV void mfma_first(v4i& c, const v4i& a, const v4i& b) {
  asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
}
// wait states before VALU reads results of the MFMAs just issued
QCN_DEV void mfma_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory"); }

// One conv over a staged patch: C::NCH K-steps of 64 MFMAs.  ga[s & 1] holds
// step s's four A fragments (step 0's issued by the caller or by the previous
// job); step s + 1's are issued early in step s; the NEXT job's first chunk
// comes from wrn into slot 0 (early in the last step when S is even, after it
// otherwise).  B fragments are single-buffered: block j's fragment of step
// s + 1 is read right after its fourth MFMA of step s, 60 MFMAs before its
// use.  Step 0 starts from an inline 0 (the zero-point correction is added in
// the epilogue: no AGPR initialisation).  The last step runs cout-block-major:
// after the 16 MFMAs of cout block i its accumulators are final, and epi(i)
// (with pre(i) issued just before those MFMAs, e.g. the epilogue constants'
// LDS loads) consumes them right there, so the AGPR -> VGPR copies of each
// accumulator sit next to its use.  lb: this lane's patch offset
// (C::at(wp, 0, p) + 16 g); voff: ((wc 64 + p) 64 + 16 g).
template <class C, class Pre, class Epi>
QCN_DEV void pipe_w4(const uint8_t* patch, wt_rsrc_t wr, wt_rsrc_t wrn, int voff, int lb,
                     v4i (&acc)[4][16], v4i (&ga)[2][4], Pre&& pre, Epi&& epi) {
  constexpr int CBK = C::kCin / 64, S = C::NCH;
  auto rd_b = [&](int s, int j) {
    const int tap = s / CBK, cb = s % CBK;
    return *reinterpret_cast<const v4i*>(patch + lb + C::jofs(j) + C::delta(tap, j) + cb * 64);
  };
  auto issue = [&](wt_rsrc_t r, int s, int slot) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, s * C::WBUF + i * 1024, 0);
      ga[slot][i] = (v4i){(int)v[0], (int)v[1], (int)v[2], (int)v[3]};
    }
  };
  v4i fb[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) fb[j] = rd_b(0, j);
  static_for<S - 1>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    static_for<64>([&](auto mc) {
      constexpr int m = decltype(mc)::value, j = m >> 2, i = m & 3;
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (s == 0) mfma_first(acc[i][j], ga[s & 1][i], fb[j]);
      else mfma_acc(acc[i][j], ga[s & 1][i], fb[j]);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (m == 1) {
        issue(wr, s + 1, (s + 1) & 1);   // slot (s + 1) & 1 was step s - 1's: all its MFMAs have issued
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (i == 3) {
        fb[j] = rd_b(s + 1, j);
        __builtin_amdgcn_sched_barrier(0);
      }
    });
  });
  constexpr int s = S - 1;
  static_for<4>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    pre(ic);
    __builtin_amdgcn_sched_barrier(0);
    static_for<16>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      if constexpr (s == 0) mfma_first(acc[i][j], ga[s & 1][i], fb[j]);
      else mfma_acc(acc[i][j], ga[s & 1][i], fb[j]);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (i == 0 && j == 1 && (S & 1) == 0) {   // slot 0 is free (this step reads slot 1)
        issue(wrn, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    });
    mfma_drain();
    epi(ic);
    __builtin_amdgcn_sched_barrier(0);
  });
  if constexpr ((S & 1) == 1) {
    issue(wrn, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// A value the compiler cannot see through: per-tile address math derived
// from it is recomputed where it is used instead of being hoisted out of the
// tile loop and held (spilled) across the MFMA jobs
QCN_DEV int fresh(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// Zero-point halo of every segment of patch C at base (only the CIN bytes a
// pixel's reads touch), 16-B stores spread over the 256 threads.
template <class C>
QCN_DEV void w4_halo(uint8_t* base, uint32_t pad, int tid) {
  constexpr int HS = 2 * C::PCOLS + 2 * (C::PROWS - 2), CH = C::kCin / 16;
  constexpr int TOTAL = C::SEGS * HS * CH;
#pragma unroll
  for (int k = 0; k < (TOTAL + 255) / 256; ++k) {
    const int e = tid + 256 * k;
    if (TOTAL % 256 == 0 || e < TOTAL) {
      const int c = e % CH, hs = (e / CH) % HS, sg = e / (CH * HS);
      int pr, pc;
      if (hs < C::PCOLS) { pr = 0; pc = hs; }
      else if (hs < 2 * C::PCOLS) { pr = C::PROWS - 1; pc = hs - C::PCOLS; }
      else { const int r = hs - 2 * C::PCOLS; pr = 1 + (r >> 1); pc = (r & 1) ? C::PCOLS - 1 : 0; }
      *reinterpret_cast<uint4*>(base + C::slot(sg, pr, pc) + c * 16) = make_uint4(pad, pad, pad, pad);
    }
  }
}

// One pair phase: conv A (+ requant) -> conv B (+ pooled requant) over this
// workgroup's images, SEGS per tile.  Image of segment sg of tile k:
// b + (k SEGS + sg) G; a phantom segment of a ragged last tile reads the
// tile's first image (this workgroup's) and stores nothing.  PH: phase index
// (stamps only).
template <class CA, class CB, int FA, int FB, bool KMAJOR, int PH>
QCN_DEV void w4_pair_body(int b, int G, const uint8_t* __restrict__ x, int nimg, int x_zp,
                          const int8_t* __restrict__ wa, const ConvEpi& epa, int xb_zp,
                          const int8_t* __restrict__ wb, const ConvEpi& epb, uint8_t* __restrict__ y) {
  using P = W4Pair<CA, CB>;
  constexpr int SEGS = P::SEGS, IMG = P::IMG, W = CA::W, CH16 = P::CH16, COUT = P::COUT;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave % CA::WCO, wp = wave / CA::WCO;
  const int mine = b < nimg ? (nimg - 1 - b) / G + 1 : 0;   // images b, b + G, ...
  const int T = (mine + SEGS - 1) / SEGS;
  auto img_of = [&](int k, int sg) {
    const int n = b + (k * SEGS + sg) * G;
    return n < nimg ? n : b + k * SEGS * G;
  };
  auto in_src = [&](int k, int q, int t) {
    const int p = t + 256 * q;
    const int n = img_of(k, p / (IMG * CH16));
    return x + ((long)n * IMG + (p / CH16) % IMG) * CA::kCin + (p % CH16) * 16;
  };
  auto in_dst = [&](int q, int t) {
    const int p = t + 256 * q;
    const int pix = (p / CH16) % IMG;
    return CA::slot(p / (IMG * CH16), pix / W + 1, pix % W + 1) + (p % CH16) * 16;
  };
  W4_RT(0);
  W4_STAMP(0);
  uint4 sv[8];   // a tile's input: eight 16-B pieces per thread
  if (T > 0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) sv[q] = *reinterpret_cast<const uint4*>(in_src(0, q, tid));
  }
  float* eka = reinterpret_cast<float*>(lds + P::OFF_EA);
  float* ekb = reinterpret_cast<float*>(lds + P::OFF_EB);
  const int* cra = reinterpret_cast<const int*>(lds + P::OFF_CA);
  const int* crb = reinterpret_cast<const int*>(lds + P::OFF_CB);
  {  // epilogue tables of both convs (u | v | mult, corr): one float4 of each
     // array per thread below COUT / 4, plain loads (no runtime selection
     // between the two ConvEpi arguments, which would be copied to scratch)
    if (tid < COUT / 4) {
      const int o = tid;
      float4* ea = reinterpret_cast<float4*>(lds + P::OFF_EA);
      float4* eb = reinterpret_cast<float4*>(lds + P::OFF_EB);
      const float4 ua = reinterpret_cast<const float4*>(epa.u)[o], va = reinterpret_cast<const float4*>(epa.v)[o],
                   ma = reinterpret_cast<const float4*>(epa.mult)[o];
      const float4 ub = reinterpret_cast<const float4*>(epb.u)[o], vb = reinterpret_cast<const float4*>(epb.v)[o],
                   mb = reinterpret_cast<const float4*>(epb.mult)[o];
      const int4 ca = reinterpret_cast<const int4*>(epa.corr)[o], cb = reinterpret_cast<const int4*>(epb.corr)[o];
      ea[o] = ua;
      ea[COUT / 4 + o] = va;
      ea[COUT / 2 + o] = ma;
      eb[o] = ub;
      eb[COUT / 4 + o] = vb;
      eb[COUT / 2 + o] = mb;
      reinterpret_cast<int4*>(lds + P::OFF_CA)[o] = ca;
      reinterpret_cast<int4*>(lds + P::OFF_CB)[o] = cb;
    }
  }
  if (T == 0) return;   // (uniform; the launcher never makes such a workgroup)

  const int p16 = lane & 15, g = lane >> 4;
  const wt_rsrc_t wra = wt_rsrc(wa), wrb = wt_rsrc(wb);
  const int voff = (wc * 64 + p16) * 64 + g * 16;
  const uint32_t pada = xor80(splat_u8(x_zp)), padb = xor80(splat_u8(xb_zp));
  v4i acc[4][16];
  v4i ga[2][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(wra, voff, i * 1024, 0);
    ga[0][i] = (v4i){(int)v[0], (int)v[1], (int)v[2], (int)v[3]};
  }
  // lane-derived addressing from a laundered lane id (recomputed per tile,
  // not hoisted and held live across the MFMA jobs)
  struct Lane {
    int g, ek, la, lb, hb, q;
  };
  auto lanes = [&]() {
    int lz = lane;
    asm volatile("" : "+v"(lz));
    Lane L;
    const int pz = lz & 15;
    L.g = lz >> 4;
    L.ek = wc * 64 + 4 * L.g;
    L.la = CA::at(wp, 0, pz) + 16 * L.g;
    L.lb = CB::at(wp, 0, pz) + 16 * L.g;
    L.hb = CA::template out_at<CB>(wp, 0, pz) + wc * 64 + 4 * L.g;
    L.q = wp * 64 + pz;
    return L;
  };
  // Epilogue constants of cout block i (4 channels per lane: 16 i + 4 g ..),
  // loaded just before the block's last 16 MFMAs
  EpiG K;
  int4 cr;
  auto pre_a = [&](auto ic) {
    const int ek = wc * 64 + 4 * (fresh(lane) >> 4) + 16 * decltype(ic)::value;
    K = load_epig(eka, COUT, ek);
    cr = *reinterpret_cast<const int4*>(cra + ek);   // zero-point correction
  };
  auto pre_b = [&](auto ic) {
    const int ek = wc * 64 + 4 * (fresh(lane) >> 4) + 16 * decltype(ic)::value;
    K = load_epig(ekb, COUT, ek);
    cr = *reinterpret_cast<const int4*>(crb + ek);
  };
  auto crr = [&](int r) { return r == 0 ? cr.x : (r == 1 ? cr.y : (r == 2 ? cr.z : cr.w)); };
  // conv A's requant of cout block i: one dword (4 channels) per pixel block,
  // kept in registers until every wave has finished reading patch A (patch B
  // aliases it), then written at the block's constant offset
  uint8_t* pa = lds + P::OFF_PA;
  uint8_t* pb = lds + P::OFF_PB;
  constexpr int NH = P::nheld() > 0 ? P::nheld() : 1;
  uint32_t res[4][NH];
  auto epi_a = [&](auto ic) {
    constexpr int i = decltype(ic)::value;
    const int hb = lanes().hb;
    int h = 0;
    static_for<16>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      uint32_t wd = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) wd = rq_elem<FA>(acc[i][j][r] + crr(r), K, r, epa, wd);
      if constexpr (P::held(j)) res[i][h++] = xor80(wd);
      else *reinterpret_cast<uint32_t*>(pb + hb + CA::template out_jofs<CB>(j) + 16 * i) = xor80(wd);
    });
  };
  auto put_a = [&](const Lane& L) {
    static_for<4>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      int h = 0;
      static_for<16>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (P::held(j))
          *reinterpret_cast<uint32_t*>(pb + L.hb + CA::template out_jofs<CB>(j) + 16 * i) = res[i][h++];
      });
    });
  };
  // conv B's pooled requant: per cout block i and group gq of 16 pooled
  // pixels, the max over the four quadrant blocks (+ corr: max(a_q + c) =
  // max(a_q) + c), requant; after the last cout block, per group a 4 x 4
  // dword transpose across the lane groups (two permlane32 + two permlane16
  // swaps) and one 16-B write-through store of 16 channels per lane
  uint32_t d[4][4];   // [gq][i]
  auto epi_b = [&](auto ic) {
    constexpr int i = decltype(ic)::value;
    static_for<4>([&](auto gc) {
      constexpr int gq = decltype(gc)::value;
      uint32_t wd = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int a = max(max(acc[i][4 * gq][r], acc[i][4 * gq + 1][r]), max(acc[i][4 * gq + 2][r], acc[i][4 * gq + 3][r]));
        wd = rq_elem<FB>(a + crr(r), K, r, epb, wd);
      }
      d[gq][i] = wd;
    });
  };
  auto put_b = [&](const Lane& L, int k) {
    static_for<4>([&](auto gc) {
      constexpr int gq = decltype(gc)::value;
      const auto s02 = __builtin_amdgcn_permlane32_swap(d[gq][0], d[gq][2], false, false);
      const auto s13 = __builtin_amdgcn_permlane32_swap(d[gq][1], d[gq][3], false, false);
      const auto t01 = __builtin_amdgcn_permlane16_swap(s02[0], s13[0], false, false);
      const auto t23 = __builtin_amdgcn_permlane16_swap(s02[1], s13[1], false, false);
      const uint4 v = make_uint4(t01[0], t01[1], t23[0], t23[1]);   // channels co .. co + 15
      const int q = L.q + 16 * gq;
      const int sg = q / P::OPI, pix = q % P::OPI;
      const int co = wc * 64 + 16 * L.g;
      if (b + (k * SEGS + sg) * G < nimg) {
        const int n = b + (k * SEGS + sg) * G;
        if constexpr (KMAJOR) {   // [f / 32][image][32], f = pix * cout + channel (NHWC flatten)
          const int kc = (pix * COUT + co) / 32;
          store_wt16(wt_rsrc(y), (uint32_t)(((long)kc * nimg + n) * 32 + 16 * (L.g & 1)), v);
        } else {
          store_wt16(wt_rsrc(y + (long)n * P::OPI * COUT), (uint32_t)(pix * COUT + co), v);
        }
      }
    });
  };

#pragma unroll 1
  for (int k = 0; k < T; ++k) {
    // patch A: halos + tile k's input (patch B's last reader, conv B of tile
    // k - 1, has passed the barrier that closed the previous iteration)
    const int ta = fresh(tid);
    w4_halo<CA>(pa, pada, ta);
#pragma unroll
    for (int q = 0; q < 8; ++q)
      *reinterpret_cast<uint4*>(pa + in_dst(q, ta)) =
          make_uint4(xor80(sv[q].x), xor80(sv[q].y), xor80(sv[q].z), xor80(sv[q].w));
    lds_barrier();
    W4_STAMP(1 + 5 * k);
    if (k + 1 < T) {   // tile k + 1's input: loads now, held in registers until then
      const int tn = fresh(tid);
#pragma unroll
      for (int q = 0; q < 8; ++q) sv[q] = *reinterpret_cast<const uint4*>(in_src(k + 1, q, tn));
    }
    pipe_w4<CA>(pa, wra, wrb, voff, lanes().la, acc, ga, pre_a, epi_a);
    W4_STAMP(2 + 5 * k);
    lds_barrier();   // every wave's conv A reads of patch A done
    w4_halo<CB>(pb, padb, fresh(tid));
    put_a(lanes());
    lds_barrier();
    W4_STAMP(3 + 5 * k);
    pipe_w4<CB>(pb, wrb, wra, voff, lanes().lb, acc, ga, pre_b, epi_b);
    W4_STAMP(4 + 5 * k);
    put_b(lanes(), k);
    lds_barrier();   // every wave's conv B reads of patch B done
    W4_STAMP(5 + 5 * k);
  }
  W4_RT(1);
}

// The launch: phase 1 (conv3 + conv4, a2 -> a4), the phase boundary (every
// wave's a4 stores complete, then the workgroup barrier), phase 2 (conv5 +
// conv6, a4 -> a6).  Phase 2 reads only a4 images this workgroup wrote.
template <int EM, bool KMAJOR>
__global__ __launch_bounds__(256, 1)
void convs36_w4_kernel(const uint8_t* __restrict__ a2, int nimg, const int8_t* __restrict__ w2, ConvEpi e2, int z2,
                       const int8_t* __restrict__ w3, ConvEpi e3, int z3, const int8_t* __restrict__ w4, ConvEpi e4,
                       int z4, const int8_t* __restrict__ w5, ConvEpi e5, int z5, uint8_t* __restrict__ a4,
                       uint8_t* __restrict__ a6) {
  const int b = (int)blockIdx.x, G = (int)gridDim.x;
  w4_pair_body<W4A3, W4B4, EM, EM, false, 0>(b, G, a2, nimg, z2, w2, e2, z3, w3, e3, a4);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  w4_pair_body<W4A5, W4B6, EM, EM, KMAJOR, 1>(b, G, a4, nimg, z4, w4, e4, z5, w5, e5, a6);
}

}  // namespace qcn

#ifdef QCN_W4_STAMP
// diagnostic builds only: the stamps of the last launch, [wg][phase][32] and [wg][phase][2]
extern "C" int qcn_w4_stamps(void* mt, void* rt, int nwg) {
  if (!mt || !rt || nwg <= 0 || nwg > 4096) return QCN_ERR_ARG;
  if (hipMemcpyFromSymbol(mt, HIP_SYMBOL(qcn::g_w4_stamp), (size_t)nwg * 2 * 32 * 8) != hipSuccess) return QCN_ERR_HIP;
  if (hipMemcpyFromSymbol(rt, HIP_SYMBOL(qcn::g_w4_rt), (size_t)nwg * 2 * 2 * 8) != hipSuccess) return QCN_ERR_HIP;
  return QCN_OK;
}
#endif

#ifndef QCN_NO_ABI
extern "C" int qcn_convs36_u8s8(const uint8_t* a2, int nimg, const qcn_conv_layer_t* layers, uint8_t* a4,
                                uint8_t* a6, int kmajor, void* stream) {
  using namespace qcn;
  if (!a2 || !layers || !a4 || !a6 || nimg <= 0) return QCN_ERR_ARG;
  ConvEpi ep[4];
  for (int i = 0; i < 4; ++i) {
    const qcn_conv_layer_t& l = layers[i];
    if (!l.w || !l.u || !l.v || !l.mult || !l.corr) return QCN_ERR_ARG;
    if (l.x_zp < 0 || l.x_zp > 255 || l.y_zp < 0 || l.y_zp > 255) return QCN_ERR_ARG;
    if (i > 0 && l.x_zp != (layers[i - 1].qdq ? layers[i - 1].qdq->z2 : layers[i - 1].y_zp)) return QCN_ERR_ARG;
    ep[i] = ConvEpi{l.u, l.v, l.mult, l.corr, l.y_zp, l.relu ? l.y_zp : 0, 0, 0.f, 0, 0.f, 0, 0};
    if (l.qdq) set_qdq(ep[i], l.qdq);
  }
  ep[3].kmajor = kmajor ? 1 : 0;
  if ((long)nimg * 4096 > 0x7fffffffL) return QCN_ERR_UNSUPPORTED;   // 32-bit store offsets
  // conv3 .. conv6 all on the FBGEMM fast epilogue, or all on the one-fma QDQ form
  int em = 0;
  bool all1 = true, all2 = true;
  for (int i = 0; i < 4; ++i) {
    all1 = all1 && epi_mode(ep[i]) == 1;
    all2 = all2 && epi_mode(ep[i]) == 2;
  }
  if (all1) em = 1;
  else if (all2) em = 2;
  else return QCN_ERR_UNSUPPORTED;
  const int ncu = qcn_cu_count();
  if (ncu <= 0) return QCN_ERR_HIP;
  const int grid = nimg < ncu ? nimg : ncu;   // persistent: one workgroup per CU
  static bool attr_done[4][QCN_MAX_DEV] = {};
#define QCN_W4(EM_, KM_)                                                                                \
  if (em == EM_ && (kmajor != 0) == KM_) {                                                              \
    auto k = convs36_w4_kernel<EM_, KM_>;                                                               \
    if (!qcn_set_lds_once((const void*)k, kW4Lds, attr_done[(EM_ - 1) * 2 + KM_])) return QCN_ERR_HIP; \
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), kW4Lds, (hipStream_t)stream, a2, nimg, layers[0].w,     \
                       ep[0], layers[0].x_zp, layers[1].w, ep[1], layers[1].x_zp, layers[2].w, ep[2],   \
                       layers[2].x_zp, layers[3].w, ep[3], layers[3].x_zp, a4, a6);                     \
    return hipGetLastError() == hipSuccess ? QCN_OK : QCN_ERR_HIP;                                      \
  }
  QCN_W4(1, true) QCN_W4(1, false) QCN_W4(2, true) QCN_W4(2, false)
#undef QCN_W4
  return QCN_ERR_UNSUPPORTED;
}
#endif
