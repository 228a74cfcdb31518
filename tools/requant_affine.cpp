// Feasibility probe (host, diagnostic): can FBGEMM's requant of one output
// channel,
//   f(acc) = sat_u8(rne(fp32(fp32(fmaf(u, v, fp32(acc))) * m)))    (zp 0, lo 0)
// be reproduced EXACTLY for every int32 acc with |acc| < 2^24 by one fma,
//   g(acc) = sat_u8(rne(fmaf(fp32(acc), a, b))) ?
// Both are monotone staircases in acc (m, a > 0), so g == f everywhere iff
// their 255 thresholds T_k = min{acc : f(acc) >= k} agree, which is checked
// exactly (fmaf) at T_k - 1 and T_k.  Build: g++ -O2 -shared -fPIC.
#include <cmath>
#include <cstdint>

namespace {

float rne_sat(float x) {   // v_cvt_pk_u8_f32: round half to even, saturate to [0, 255]
  const float r = std::nearbyint(x);
  return std::fmin(std::fmax(r, 0.0f), 255.0f);
}

float f_ref(int acc, float u, float v, float m) {
  const float t = std::fmaf(u, v, (float)acc);
  return rne_sat(t * m);
}

float g_aff(int acc, float a, float b) { return rne_sat(std::fmaf((float)acc, a, b)); }

// smallest acc in [lo, hi] with f(acc) >= k (f monotone); hi + 1 if none
int threshold(int k, float u, float v, float m, int lo, int hi) {
  while (lo < hi) {
    const int mid = lo + (hi - lo) / 2;
    if (f_ref(mid, u, v, m) >= (float)k) hi = mid;
    else lo = mid + 1;
  }
  return f_ref(lo, u, v, m) >= (float)k ? lo : lo + 1;
}

}  // namespace

extern "C" {

// Returns 1 and (a, b) when an exact one-fma form exists, 0 otherwise.
int NSCAN = 32;
void requant_affine_scan(int n) { NSCAN = n; }
int requant_affine(float u, float v, float m, float* out) {
  if (!(m > 0.0f)) return 0;
  const int LO = -(1 << 24) + 1, HI = (1 << 24) - 1;
  static int T[256];
  for (int k = 1; k <= 255; ++k) T[k] = threshold(k, u, v, m, LO, HI);
  // simple scan of +-32 ulps around m
  float lo_m = m, hi_m = m;
  for (int i = 0; i < NSCAN; ++i) { lo_m = std::nextafterf(lo_m, 0.0f); hi_m = std::nextafterf(hi_m, 1e30f); }
  for (float ac = lo_m; ac <= hi_m; ac = std::nextafterf(ac, 1e30f)) {
    double L = -1e300, U = 1e300;
    for (int k = 1; k <= 255; ++k) {
      if (T[k] > HI || T[k] <= LO) continue;
      // g(T_k) >= k needs T_k ac + b >= k - 0.5 (ties aside); g(T_k - 1) <= k - 1 needs < k - 0.5
      L = std::fmax(L, (k - 0.5) - (double)T[k] * ac);
      U = std::fmin(U, (k - 0.5) - (double)(T[k] - 1) * ac);
    }
    if (!(L < U)) continue;
    // try a few fp32 b in [L, U)
    const float mids[3] = {(float)(0.5 * (L + U)), (float)(L + 0.25 * (U - L)), (float)(L + 0.75 * (U - L))};
    for (float b : mids) {
      bool ok = true;
      for (int k = 1; k <= 255 && ok; ++k) {
        if (T[k] > HI) continue;
        if (T[k] > LO) ok = g_aff(T[k] - 1, ac, b) == f_ref(T[k] - 1, u, v, m);
        if (ok) ok = g_aff(T[k], ac, b) == f_ref(T[k], u, v, m);
      }
      if (ok) {
        out[0] = ac;
        out[1] = b;
        return 1;
      }
    }
  }
  return 0;
}

// Exhaustive check of a form over [lo, hi] (diagnostic): number of mismatches.
long long requant_affine_check(float u, float v, float m, float a, float b, int lo, int hi) {
  long long bad = 0;
  for (int acc = lo; acc <= hi; ++acc) bad += g_aff(acc, a, b) != f_ref(acc, u, v, m);
  return bad;
}

}  // extern "C"

extern "C" {
// With the slope a fixed: 1 and *b when an exact form exists for this channel.
int requant_affine_fixed(float u, float v, float m, float a, float* b_out) {
  const int LO = -(1 << 24) + 1, HI = (1 << 24) - 1;
  int T[256];
  for (int k = 1; k <= 255; ++k) T[k] = threshold(k, u, v, m, LO, HI);
  double L = -1e300, U = 1e300;
  for (int k = 1; k <= 255; ++k) {
    if (T[k] > HI || T[k] <= LO) continue;
    L = std::fmax(L, (k - 0.5) - (double)T[k] * a);
    U = std::fmin(U, (k - 0.5) - (double)(T[k] - 1) * a);
  }
  if (!(L < U)) return 0;
  const float mids[5] = {(float)(0.5 * (L + U)), (float)(L + 0.25 * (U - L)), (float)(L + 0.75 * (U - L)),
                         (float)(L + 0.1 * (U - L)), (float)(L + 0.9 * (U - L))};
  for (float b : mids) {
    bool ok = true;
    for (int k = 1; k <= 255 && ok; ++k) {
      if (T[k] > HI) continue;
      if (T[k] > LO) ok = g_aff(T[k] - 1, a, b) == f_ref(T[k] - 1, u, v, m);
      if (ok) ok = g_aff(T[k], a, b) == f_ref(T[k], u, v, m);
    }
    if (ok) { *b_out = b; return 1; }
  }
  return 0;
}
}
