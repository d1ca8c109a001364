// tpe_device.hpp -- device helpers shared by the fit and scoring kernels.
#pragma once
#include <math.h>

#include "tpe_internal.hpp"

namespace tpe {

// numpy.maximum / numpy.minimum: NaN propagates from either side.
__device__ __forceinline__ double np_maximum(double a, double b) {
  if (a != a) return a;
  if (b != b) return b;
  return a >= b ? a : b;
}
__device__ __forceinline__ double np_minimum(double a, double b) {
  if (a != a) return a;
  if (b != b) return b;
  return a <= b ? a : b;
}

// ------------------------------------------------------------------------
// Cross-lane data movement on DPP (VALU operand modifiers, a few cycles)
// instead of ds_bpermute (an LDS round trip per step).  Patterns: quad_perm
// xor 1 / xor 2, row_half_mirror (lane i <- 7 - i in its 8), row_mirror
// (i <- 15 - i in its 16), row_shr:n, row_bcast:15 / :31 (gfx9 family).
// ------------------------------------------------------------------------
enum : int {
  kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140,
  kDppShr1 = 0x111, kDppShr2 = 0x112, kDppShr4 = 0x114, kDppShr8 = 0x118,
  kDppBcast15 = 0x142, kDppBcast31 = 0x143
};
// lanes without a source (row_shr) or in a disabled row read 0
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ int dpp(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWS, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  const int lo = dpp<CTRL>((int)(uint32_t)v), hi = dpp<CTRL>((int)(uint32_t)(v >> 32));
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
  return __builtin_bit_cast(double, dpp64<CTRL>(__builtin_bit_cast(uint64_t, v)));
}
// the value of one lane as a wave-uniform scalar
__device__ __forceinline__ int lane_value(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t lane_value64(uint64_t v, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}
// wave-wide reductions (every lane must be active); results wave-uniform
__device__ __forceinline__ int wave_sum(int v) {
  v += dpp<kDppXor1>(v);
  v += dpp<kDppXor2>(v);
  v += dpp<kDppHalfMirror>(v);
  v += dpp<kDppMirror>(v);  // every lane: its row's sum
  return lane_value(v, 0) + lane_value(v, 16) + lane_value(v, 32) + lane_value(v, 48);
}
__device__ __forceinline__ uint64_t wave_and(uint64_t v) {
  v &= dpp64<kDppXor1>(v);
  v &= dpp64<kDppXor2>(v);
  v &= dpp64<kDppHalfMirror>(v);
  v &= dpp64<kDppMirror>(v);
  return lane_value64(v, 0) & lane_value64(v, 16) & lane_value64(v, 32) & lane_value64(v, 48);
}
__device__ __forceinline__ uint64_t wave_or(uint64_t v) {
  v |= dpp64<kDppXor1>(v);
  v |= dpp64<kDppXor2>(v);
  v |= dpp64<kDppHalfMirror>(v);
  v |= dpp64<kDppMirror>(v);
  return lane_value64(v, 0) | lane_value64(v, 16) | lane_value64(v, 32) | lane_value64(v, 48);
}
// inclusive prefix sum over the wave's lanes
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += dpp<kDppShr1>(v);
  v += dpp<kDppShr2>(v);
  v += dpp<kDppShr4>(v);
  v += dpp<kDppShr8>(v);
  v += dpp<kDppBcast15, 0xA>(v);
  v += dpp<kDppBcast31, 0xC>(v);
  return v;
}

// normal_cdf, hyperopt/tpe.py:96-101 (no FMA contraction: bit-level parity).
__device__ __forceinline__ double normal_cdf(double x, double mu, double sigma) {
#pragma clang fp contract(off)
  const double bottom = np_maximum(1.4142135623730951 * sigma, kEPS);
  const double z = (x - mu) / bottom;
  return 0.5 * (1.0 + erf(z));
}

// Total order of numpy argsort on float64 as an unsigned key: ascending,
// -0.0 == +0.0, every NaN after +inf and equal to each other (ties are then
// broken by position by the callers, i.e. a stable sort).
__device__ __forceinline__ uint64_t sort_key(double v) {
  if (v != v) return ~0ull;
  if (v == 0.0) return 0x8000000000000000ull;
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

// (key, position) lexicographic order
__device__ __forceinline__ bool kp_less(uint64_t ka, uint32_t pa, uint64_t kb, uint32_t pb) {
  return ka < kb || (ka == kb && pa < pb);
}

// numpy argmax order over (score, global index): a NaN wins at its first
// index, otherwise the larger score, ties to the lower index (tpe.py:756).
// (branch-free: the callers take their records with selects, so no
// exec-masked branch carries a winner's value -- DESIGN §3, the finalize
// re-read build whose branchy select handed a row-1 winner the row-0 value)
__device__ __forceinline__ bool better(double sa, int64_t ia, double sb, int64_t ib) {
  const bool na = sa != sa, nb = sb != sb;
  const bool lt = ia < ib;
  const bool by_score = (sa != sb) ? (sa > sb) : lt;    // neither NaN
  const bool by_nan = (na && nb) ? lt : na;             // a NaN ranks first
  return (ia >= 0) & ((ib < 0) | ((na | nb) ? by_nan : by_score));
}

// a <- (sb, vb, ib) when that record is better (numpy argmax order), by selects
__device__ __forceinline__ void take_better(double &s, double &v, int64_t &i, double os, double ov,
                                            int64_t oi) {
  const bool b = better(os, oi, s, i);
  s = b ? os : s;
  v = b ? ov : v;
  i = b ? oi : i;
}

// (the reduction carries (score, index) only; the winner's value comes from
// the lane that held the winning record -- candidate indices are unique
// across the lanes, so that lane is the one whose own index won; with no
// valid record anywhere every lane keeps its own (NaN, NaN, -1))
__device__ __forceinline__ void wave_best(double &s, double &v, int64_t &i) {
  const int64_t i0 = i;
  const double v0 = v;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double os = __shfl_xor(s, o, 64);
    const int64_t oi = __shfl_xor(i, o, 64);
    const bool b = better(os, oi, s, i);
    s = b ? os : s;
    i = b ? oi : i;
  }
  const uint64_t m = __ballot(i0 == i && i >= 0);
  v = m ? __shfl(v0, (int)__builtin_ctzll(m), 64) : v0;
}

// activity of a conditional hp: OR over its (parent active and parent value
// == branch) conditions (hyperopt/vectorize.py:20-38 routing)
__device__ __forceinline__ bool hp_active(const tpe_hp &H, const Partial *res,
                                          const int32_t *cp, const int32_t *cb) {
  if (H.cond_count == 0) return true;
  for (int c = 0; c < H.cond_count; ++c) {
    const Partial &r = res[cp[H.cond_begin + c]];
    if (r.active && r.index >= 0 && r.value == (double)cb[H.cond_begin + c]) return true;
  }
  return false;
}

// Per-component scoring coefficients (Coef, 32 B) of a continuous mixture.
//  LSE (q = None): the log-density term in log2 units as a quadratic in the
//   centred candidate y' = y - center (center = prior_mu of the hp):
//     t = c - (a (y' - mu'))^2 = alpha + y' (beta + gamma y'),
//   a = sqrt(log2(e) / 2) / max(sigma, EPS), mu' = mu - center,
//   c = log2(e) log(w / sqrt(2 pi sigma^2) / p_accept)      (GMM1_lpdf, tpe.py:138-144)
//   c = log2(e) (log w - log(max(sigma, EPS) sqrt(2 pi)))   (LGMM1_lpdf, tpe.py:193-202,
//       278-281: no p_accept; log x is subtracted per candidate).
//   Centring keeps alpha, beta y' and gamma y'^2 within ~(100 |mu'| / range)^2 of
//   t, i.e. cancellation costs < 1e-12 absolute in fp64.
//  ERF (q given): (mu, 1 / max(sqrt(2) sigma, EPS), w) for the CDF differences.
// The log-sum-exp envelope contribution of one component (its mu', c, a^2);
// neutral values for padding components.
struct EnvTerm {
  double m, c, a2;
};

__device__ __forceinline__ Coef make_coef(const tpe_hp &H, double w, double mu, double sigma,
                                          double pacc, EnvTerm *env = nullptr) {
#pragma clang fp contract(off)
  Coef c;
  c.w = 0.0;
  const double sp = np_maximum(sigma, kEPS);
  if (H.flags & TPE_HAS_Q) {
    const double s2 = np_maximum(1.4142135623730951 * sigma, kEPS);
    c.x = mu;
    c.y = 1.0 / s2;
    c.z = w;
    c.w = 6.6 * s2;  // dead-zone half-width for the chunk test (tpe_score.hip)
    return c;
  }
  const double L2E = 1.4426950408889634;  // log2(e)
  double cc;
  if (H.family == TPE_GMM) {
    const double Z = sqrt(2.0 * 3.141592653589793 * (sigma * sigma));
    cc = L2E * log(w / Z / pacc);
  } else {
    cc = L2E * (log(w) - log(sp * 2.5066282746310002));
  }
  const double a2 = (0.5 * L2E) / (sp * sp);   // a^2
  const double m = mu - H.prior_mu;            // mu'
  c.x = cc - a2 * (m * m);                     // alpha
  c.y = 2.0 * a2 * m;                          // beta
  c.z = -a2;                                   // gamma
  if (env) *env = EnvTerm{m, cc, a2};
  return c;
}

// The block envelope of the 8 consecutive components held by the 8 lanes
// (lane & 7) of this lane's group: reduced with xor shuffles (all 8 lanes
// must be active), written by the group's first lane into the block's w-row
// as 4 floats rounded outward (tpe_internal.hpp, kLseDeadBase).  NaN terms
// disable the skip of the block.
__device__ __forceinline__ void store_lse_envelope(Coef *table, int64_t k, EnvTerm e, bool valid,
                                                   const Coef &cf, Coef32 *t32,
                                                   float4 *te = nullptr) {
  // padding lanes (valid = false) contribute the neutral element
  double lo = valid ? e.m : INFINITY, hi = valid ? e.m : -INFINITY;
  double cm = !valid ? -INFINITY : (e.c == e.c) ? e.c : INFINITY, am = valid ? e.a2 : INFINITY;
  bool bad = valid && (!(e.m == e.m) || !(e.a2 == e.a2));
  static_assert(kCoefBlock == 8, "an envelope is one 8-lane DPP group");
  lo = fmin(lo, dppd<kDppXor1>(lo)); hi = fmax(hi, dppd<kDppXor1>(hi));
  cm = fmax(cm, dppd<kDppXor1>(cm)); am = fmin(am, dppd<kDppXor1>(am));
  bad |= dpp<kDppXor1>((int)bad) != 0;
  lo = fmin(lo, dppd<kDppXor2>(lo)); hi = fmax(hi, dppd<kDppXor2>(hi));
  cm = fmax(cm, dppd<kDppXor2>(cm)); am = fmin(am, dppd<kDppXor2>(am));
  bad |= dpp<kDppXor2>((int)bad) != 0;
  lo = fmin(lo, dppd<kDppHalfMirror>(lo)); hi = fmax(hi, dppd<kDppHalfMirror>(hi));
  cm = fmax(cm, dppd<kDppHalfMirror>(cm)); am = fmin(am, dppd<kDppHalfMirror>(am));
  bad |= dpp<kDppHalfMirror>((int)bad) != 0;
  // block-local fp32 form (Coef32): expand the quadratic about the block's
  // mu' midpoint in fp64, alpha relative to an integer block base
  bool wide = false;
  {
    const double cen = (lo <= hi) ? 0.5 * (lo + hi) : 0.0;
    const double al = valid ? cf.x + cen * (cf.y + cen * cf.z) : -INFINITY;
    const double be = valid ? cf.y + 2.0 * cen * cf.z : 0.0;
    double amax = (al == al) ? al : -INFINITY;
    amax = fmax(amax, dppd<kDppXor1>(amax));
    amax = fmax(amax, dppd<kDppXor2>(amax));
    amax = fmax(amax, dppd<kDppHalfMirror>(amax));
    const double base = (amax > -1.0e300 && amax < 1.0e300) ? floor(amax) : 0.0;
    // spread a^2 (mu' - centre)^2 of the block (NaN / inf: keep fp64 too)
    const double dm = e.m - cen;
    double sp = valid ? e.a2 * dm * dm : 0.0;
    if (!(sp <= kF32Spread)) sp = INFINITY;
    sp = fmax(sp, dppd<kDppXor1>(sp));
    sp = fmax(sp, dppd<kDppXor2>(sp));
    sp = fmax(sp, dppd<kDppHalfMirror>(sp));
    wide = !(sp <= kF32Spread);
    Coef32 *b = t32 + k / kCoefBlock;
    const int j = (int)(k % kCoefBlock);
    b->a[j] = (float)(al - base);
    b->b[j] = (float)be;
    b->c[j] = valid ? (float)cf.z : 0.0f;
    if (j == 0) {
      b->center = cen;
      b->base = (float)base;
      b->pad0 = 0.0f;
    }
  }
  if (k % kCoefBlock) return;
  float *out = reinterpret_cast<float *>(reinterpret_cast<double *>(table) + coef_off(k, 3));
  const float flo = (float)lo, fhi = (float)hi, fc = (float)cm, fa = (float)am;
  out[0] = ((double)flo > lo) ? nextafterf(flo, -INFINITY) : flo;
  out[1] = ((double)fhi < hi) ? nextafterf(fhi, INFINITY) : fhi;
  out[2] = ((double)fc < cm) ? nextafterf(fc, INFINITY) : fc;
  out[3] = ((double)fa > am) ? nextafterf(fa, 0.0f) : fa;
  if (bad) { out[2] = INFINITY; out[3] = 0.0f; }
  if (wide) out[3] = -out[3];  // the block keeps the fp64 quadratic in mode 3
  if (te) te[k / kCoefBlock] = make_float4(out[0], out[1], out[2], out[3]);  // (compact copy)
}

// reductions over the 16 lanes of a DPP row (every lane of the row active;
// xor / mirror steps: every lane ends with the same, bitwise, value)
__device__ __forceinline__ double row16_min(double v) {
  v = fmin(v, dppd<kDppXor1>(v));
  v = fmin(v, dppd<kDppXor2>(v));
  v = fmin(v, dppd<kDppHalfMirror>(v));
  return fmin(v, dppd<kDppMirror>(v));
}
__device__ __forceinline__ double row16_max(double v) {
  v = fmax(v, dppd<kDppXor1>(v));
  v = fmax(v, dppd<kDppXor2>(v));
  v = fmax(v, dppd<kDppHalfMirror>(v));
  return fmax(v, dppd<kDppMirror>(v));
}
__device__ __forceinline__ double row16_sum(double v) {
  v += dppd<kDppXor1>(v);
  v += dppd<kDppXor2>(v);
  v += dppd<kDppHalfMirror>(v);
  return v + dppd<kDppMirror>(v);
}

// reductions over the 8 lanes of a coefficient block (lane & 7; all 8 active)
__device__ __forceinline__ double row8_min(double v) {
  v = fmin(v, dppd<kDppXor1>(v));
  v = fmin(v, dppd<kDppXor2>(v));
  return fmin(v, dppd<kDppHalfMirror>(v));
}
__device__ __forceinline__ double row8_max(double v) {
  v = fmax(v, dppd<kDppXor1>(v));
  v = fmax(v, dppd<kDppXor2>(v));
  return fmax(v, dppd<kDppHalfMirror>(v));
}
__device__ __forceinline__ double row8_sum(double v) {
  v += dppd<kDppXor1>(v);
  v += dppd<kDppXor2>(v);
  return v + dppd<kDppHalfMirror>(v);
}
template <int CH> __device__ __forceinline__ double rowc_min(double v) {
  return CH == 8 ? row8_min(v) : row16_min(v);
}
template <int CH> __device__ __forceinline__ double rowc_max(double v) {
  return CH == 8 ? row8_max(v) : row16_max(v);
}
template <int CH> __device__ __forceinline__ double rowc_sum(double v) {
  return CH == 8 ? row8_sum(v) : row16_sum(v);
}

// The moment form (CoefM / CoefM8, tpe_internal.hpp) of the CH-component
// chunk held by this lane's DPP row of CH lanes (component k = lane's, k % CH
// = its place in the chunk): centre = mu' midpoint, T_k = t_k(centre) = c -
// a^2 d_k^2, rho_k = 2^(T_k - T*), q_k = 2 a^2 ln2 d_k, m_j = sum_k rho_k
// q_k^j / j! (j <= DEG) in fp64, stored fp32.  Eligible only when every valid
// component has the same a^2 (the same sigma) and the terms are finite; else
// xh = +inf.  Tables: 16 components / degree 9 (CoefM), 8 / 15 (CoefM8) and
// 16 / 15 (CoefM8 layout: the wide-window form of 16-wide plans).
template <int CH, int DEG, typename TB>
__device__ __forceinline__ void store_lse_moments_t(TB *tm, int64_t k, EnvTerm e, bool valid) {
  const double LN2 = 0.6931471805599453;
  const double lo = rowc_min<CH>(valid ? e.m : INFINITY), hi = rowc_max<CH>(valid ? e.m : -INFINITY);
  const double amin = rowc_min<CH>(valid ? e.a2 : INFINITY);
  const double amax = rowc_max<CH>(valid ? e.a2 : -INFINITY);
  const double cen = lo <= hi ? 0.5 * (lo + hi) : 0.0;
  const double d = valid ? e.m - cen : 0.0;
  const double T = valid ? e.c - e.a2 * (d * d) : -INFINITY;
  const double Tm = rowc_max<CH>(T == T ? T : INFINITY);
  const double hh = rowc_max<CH>(valid ? fabs(d) : 0.0);
  const bool ok = lo <= hi && amin == amax && amin > 0.0 && amin < 1.0e300 && Tm > -1.0e300 &&
                  Tm < 1.0e300 && hh < 1.0e300;
  const double rho = (valid && ok) ? exp2(T - Tm) : 0.0;
  const double q = 2.0 * amin * LN2 * d;
  float m[DEG + 1];
  double p = rho, fact = 1.0;
#pragma unroll
  for (int j = 0; j <= DEG; ++j) {
    if (j > 0) fact *= (double)j;
    m[j] = (float)(rowc_sum<CH>(p) / fact);
    p *= q;
  }
  if (k % CH) return;
  TB *b = tm + k / CH;
  const double base = ok ? floor(Tm) : 0.0;
  float xh = INFINITY;
  if (ok) {
    const double x = hh * 2.0 * amin * LN2;
    xh = (float)x;
    if ((double)xh < x) xh = nextafterf(xh, INFINITY);
  }
  b->center = cen;
  b->xh = xh;
  b->base = (float)base;
  b->cm = (float)(Tm - base);
  b->gam = (float)(-amin);
#pragma unroll
  for (int j = 0; j <= DEG; ++j) b->m[j] = m[j];
}
__device__ __forceinline__ void store_lse_moments(CoefM *tm, int64_t k, EnvTerm e, bool valid) {
  store_lse_moments_t<kMomChunk, kMomDeg>(tm, k, e, valid);
}
__device__ __forceinline__ void store_lse_moments8(CoefM8 *tm, int64_t k, EnvTerm e, bool valid) {
  store_lse_moments_t<kCoefBlock, kMom8Deg>(tm, k, e, valid);
}
__device__ __forceinline__ void store_lse_moments16h(CoefM8 *tm, int64_t k, EnvTerm e, bool valid) {
  store_lse_moments_t<kMomChunk, kMom8Deg>(tm, k, e, valid);
}

// Natural log of a finite x > 0 in ~30 VALU (OCML's fp64 log is ~70: its
// double-double tail buys the last half-ulp, which no caller here needs --
// candidate transforms y = log x, the EI ratio, bucketing keys): x = m 2^e
// with m in [1/sqrt2, sqrt2), log m = 2 atanh s, s = (m - 1) / (m + 1),
// |s| <= 0.1716, the odd series to s^21 (truncation < 2e-18 relative), the
// quotient by v_rcp_f64 and two Newton steps, e ln2 in two parts; within a
// few ulp of log x (tests/test_gpu_ops.py fast_log check).  Zero, negative,
// infinite and NaN x take the library log (same results as before).
__device__ __forceinline__ double fast_log(double x) {
  if (!(x > 0.0 && x < INFINITY)) return log(x);
  int e = __builtin_amdgcn_frexp_exp(x);
  double m = __builtin_amdgcn_frexp_mant(x);  // [0.5, 1)
  const bool lo = m < 0.70710678118654752440;
  m = lo ? 2.0 * m : m;
  e = lo ? e - 1 : e;
  const double n = m - 1.0, d = m + 1.0;  // (exact: m in [0.707, 1.414))
  double r = __builtin_amdgcn_rcp(d);
  r = fma(fma(-d, r, 1.0), r, r);
  r = fma(fma(-d, r, 1.0), r, r);
  double sq = n * r;
  sq = fma(fma(-d, sq, n), r, sq);  // s = n / d, corrected
  const double z = sq * sq;
  double p = 1.0 / 21.0;
  p = fma(p, z, 1.0 / 19.0);
  p = fma(p, z, 1.0 / 17.0);
  p = fma(p, z, 1.0 / 15.0);
  p = fma(p, z, 1.0 / 13.0);
  p = fma(p, z, 1.0 / 11.0);
  p = fma(p, z, 1.0 / 9.0);
  p = fma(p, z, 1.0 / 7.0);
  p = fma(p, z, 1.0 / 5.0);
  p = fma(p, z, 1.0 / 3.0);
  const double s2 = 2.0 * sq;
  const double lm = fma(s2 * z, p, s2);  // 2 s (1 + z p)
  const double fe = (double)e;
  return fma(fe, 6.93147180369123816490e-01, fma(fe, 1.90821492927058770002e-10, lm));
}
__device__ __forceinline__ double fast_log2(double x) {
  if (!(x > 0.0 && x < INFINITY)) return log2(x);
  int e = __builtin_amdgcn_frexp_exp(x);
  double m = __builtin_amdgcn_frexp_mant(x);
  const bool lo = m < 0.70710678118654752440;
  m = lo ? 2.0 * m : m;
  e = lo ? e - 1 : e;
  const double n = m - 1.0, d = m + 1.0;
  double r = __builtin_amdgcn_rcp(d);
  r = fma(fma(-d, r, 1.0), r, r);
  r = fma(fma(-d, r, 1.0), r, r);
  double sq = n * r;
  sq = fma(fma(-d, sq, n), r, sq);
  const double z = sq * sq;
  double p = 1.0 / 21.0;
  p = fma(p, z, 1.0 / 19.0);
  p = fma(p, z, 1.0 / 17.0);
  p = fma(p, z, 1.0 / 15.0);
  p = fma(p, z, 1.0 / 13.0);
  p = fma(p, z, 1.0 / 11.0);
  p = fma(p, z, 1.0 / 9.0);
  p = fma(p, z, 1.0 / 7.0);
  p = fma(p, z, 1.0 / 5.0);
  p = fma(p, z, 1.0 / 3.0);
  const double s2 = 2.0 * sq;
  const double lm = fma(s2 * z, p, s2);  // log m
  return fma(lm, 1.44269504088896340736, (double)e);
}

}  // namespace tpe
