// tpe_draw.hpp -- candidate sampling shared by the draw kernels
// (tpe_kernels.hip) and the scoring kernel's in-tile draws (tpe_score.hip).
#pragma once
#include <math.h>

#include "tpe_device.hpp"

namespace tpe {

// ------------------------------------------------------------------------
// counter-based Philox4x32-10 in registers
// ------------------------------------------------------------------------
struct U4 { uint32_t x, y, z, w; };
__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

struct Draw { double u0, u1, u2, u3; };
__device__ __forceinline__ Draw draw4(uint64_t seed, uint64_t gi, uint32_t stream,
                                      uint32_t it) {
  const U4 c0{(uint32_t)gi, (uint32_t)(gi >> 32), stream, 2u * it};
  const U4 c1{(uint32_t)gi, (uint32_t)(gi >> 32), stream, 2u * it + 1u};
  const U4 r0 = philox(c0, (uint32_t)seed, (uint32_t)(seed >> 32));
  const U4 r1 = philox(c1, (uint32_t)seed, (uint32_t)(seed >> 32));
  return Draw{u53(r0.x, r0.y), u53(r0.z, r0.w), u53(r1.x, r1.y), u53(r1.z, r1.w)};
}

// inverse CDF pick of a component with probability w[k] / wsum
__device__ __forceinline__ int pick(const double *__restrict__ w, int K, double t) {
  int k = 0;
  double acc = w[0];
  while (k < K - 1 && acc <= t) { ++k; acc += w[k]; }
  return k;
}

// the same pick on an inclusive CDF of the weights: the first k with
// cdf[k] > u * cdf[K-1] (binary search)
__device__ __forceinline__ int pick_cdf(const double *cdf, int K, double u) {
  const double t = u * cdf[K - 1];
  int lo = 0, hi = K - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cdf[mid] <= t) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// the rejection sampler's Philox pair and Box-Muller normal, out of line: its
// register footprint is what every kernel that can reach the fallback
// allocates, common path or not
__device__ __attribute__((noinline)) inline Draw draw4_ool(uint64_t seed, uint64_t gi,
                                                           uint32_t stream, uint32_t it) {
  return draw4(seed, gi, stream, it);
}
__device__ __attribute__((noinline)) inline double box_muller_ool(double u1, double u2) {
  return sqrt(-2.0 * log(1.0 - u1)) * cospi(2.0 * u2);
}

// One GMM1/LGMM1/categorical draw (tpe.py:62-93, 216-250; stochastic.py:104);
// cdf (optional): the weights' inclusive prefix sums.  The rejection sampler
// is the fallback for mixtures beyond the LDS table.
__device__ inline double draw_one(const tpe_hp &H, const MixInfo &I,
                           const double *__restrict__ w,
                           const double *__restrict__ mu,
                           const double *__restrict__ sg, uint64_t seed,
                           uint64_t gi, uint32_t stream, const double *cdf = nullptr) {
  if (H.family == TPE_CAT) {
    const Draw d = draw4(seed, gi, stream, 0);
    return (double)(cdf ? pick_cdf(cdf, I.K, d.u0) : pick(w, I.K, d.u0 * I.wsum));
  }
  const bool bounded = (H.flags & (TPE_HAS_LOW | TPE_HAS_HIGH)) != 0;
  double x = 0.0;
  bool ok = false;
  int k = 0;
  Draw d{};
#pragma unroll 1
  for (uint32_t it = 0; it < 64 && !ok; ++it) {
    d = draw4_ool(seed, gi, stream, it);
    k = cdf ? pick_cdf(cdf, I.K, d.u0) : pick(w, I.K, d.u0 * I.wsum);
    const double z = box_muller_ool(d.u1, d.u2);
    const double v = mu[k] + sg[k] * z;
    if (!bounded || (H.low <= v && v < H.high)) { x = v; ok = true; }
  }
  if (!ok) {
    // truncated inverse CDF of the last component (rejection budget spent)
    const double a = normal_cdf(H.low, mu[k], sg[k]);
    const double b = normal_cdf(H.high, mu[k], sg[k]);
    const double u = a + d.u3 * (b - a);
    double v = mu[k] + sg[k] * 1.4142135623730951 * erfinv(2.0 * u - 1.0);
    if (!(v >= H.low)) v = H.low;
    if (!(v < H.high)) v = nextafter(H.high, -INFINITY);
    x = v;
  }
  if (H.family == TPE_LGMM) x = exp(x);
  if (H.flags & TPE_HAS_Q) x = rint(x / H.q) * H.q;
  return x;
}

// ------------------------------------------------------------------------
// Table sampler (k_draw, k_sample).  The reference's truncated draw re-picks
// the component on every rejection (tpe.py:82-87, 237-242), so an accepted
// draw comes from component k with probability proportional to w_k * m_k,
// m_k = P_k(low <= x < high), distributed as N(mu_k, sigma_k) truncated to
// the bounds.  The table holds, per component, that pick weight as an
// inclusive CDF and the truncated inverse-CDF constants; a draw is then one
// pick (binary search) and one inverse CDF, with no divergent rejection loop.
// The inverse CDF works in the tail that keeps precision: for bounds in the
// upper half of component k it inverts the upper tail Q with erfcinv, in the
// lower half the lower tail Phi with erfcinv, else Phi with erfinv.
// ------------------------------------------------------------------------
template <int CAP>
struct DrawTableT {
  double cdf[CAP];   // inclusive CDF of the pick weights
  double base[CAP];  // Q(a) (mode 1), Phi(a) (modes 0, 2)
  double mass[CAP];  // m_k
  unsigned char mode[CAP];
  double wtot[16];   // per-wave totals of the scan (<= 1024 threads)
};
typedef DrawTableT<kTabCap> DrawTable;

// block-wide inclusive scan of a[0, K) in place: thread t scans a contiguous
// segment, then adds the exclusive scan of the segment totals (deterministic)
__device__ inline void block_inclusive_scan(double *a, int K, double *wtot) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, nt = blockDim.x;
  const int per = (K + nt - 1) / nt;
  const int k0 = min(K, t * per), k1 = min(K, k0 + per);
  double acc = 0.0;
  for (int k = k0; k < k1; ++k) { acc += a[k]; a[k] = acc; }
  double v = acc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double n = __shfl_up(v, o, 64);
    if (lane >= o) v += n;
  }
  if (lane == 63) wtot[wv] = v;
  __syncthreads();
  double off = v - acc;
  for (int w = 0; w < wv; ++w) off += wtot[w];
  for (int k = k0; k < k1; ++k) a[k] += off;
  __syncthreads();
}

// block-wide: the table of a (hp, mixture); K <= CAP
template <int CAP>
__device__ void build_table(const tpe_hp &H, int K, const double *__restrict__ w,
                            const double *__restrict__ mu, const double *__restrict__ sg,
                            DrawTableT<CAP> &T) {
  const bool bounded = H.family != TPE_CAT && (H.flags & (TPE_HAS_LOW | TPE_HAS_HIGH)) != 0;
#pragma unroll 1
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    double pw = w[k];
    if (bounded) {
      const double s2 = 1.4142135623730951 * sg[k];
      const double za = (H.low - mu[k]) / s2, zb = (H.high - mu[k]) / s2;
      double b, m;
      unsigned char md;
      if (za >= 0.0) {         // upper half: Q(z) = erfc(z) / 2
        b = 0.5 * erfc(za); m = b - 0.5 * erfc(zb); md = 1;
      } else if (zb <= 0.0) {  // lower half: Phi(z) = erfc(-z) / 2
        b = 0.5 * erfc(-za); m = 0.5 * erfc(-zb) - b; md = 2;
      } else {
        b = 0.5 * erfc(-za); m = 0.5 * erfc(-zb) - b; md = 0;
      }
      m = m > 0.0 ? m : 0.0;
      T.base[k] = b; T.mass[k] = m; T.mode[k] = md;
      pw *= m;
    }
    T.cdf[k] = pw;
  }
  __syncthreads();
  block_inclusive_scan(T.cdf, K, T.wtot);
}

// erfcinv(y) for y in (0, 1] (the tail-side inverse CDF of the table
// sampler; the value a sample takes, so ~4e-7 relative on the normal
// quantile is immaterial): Giles' single-precision erfinv polynomials
// ("Approximating the erfinv function", GPU Computing Gems, 2011) in
// w = -log(y (2 - y)), with w from the fp64 y by frexp + v_log_f32 (no
// cancellation in 1 - x, full range of y), both branches evaluated without
// divergence; beyond w = 36 (y < ~1e-16, outside the fitted range) the fp64
// OCML erfcinv.
// (the fp64 OCML erfcinv of the far tail out of line: inlined, its
// temporaries set the register allocation of every draw loop that can reach
// it -- k_draw_sorted went from 142 to 255 VGPRs)
__device__ __attribute__((noinline)) inline double erfcinv_ool(double y) { return erfcinv(y); }
__device__ __forceinline__ double erfcinv_fast(double y) {
  int e1, e2;
  const double m1 = frexp(y, &e1), m2 = frexp(2.0 - y, &e2);
  const float l2 = __builtin_amdgcn_logf((float)m1) + __builtin_amdgcn_logf((float)m2) +
                   (float)(e1 + e2);                   // log2(y (2 - y))
  const float w = -0.6931471805599453f * l2;
  if (!(w <= 36.0f)) return erfcinv_ool(y);
  const float wc = w - 2.5f;
  float pc = 2.81022636e-08f;
  pc = fmaf(pc, wc, 3.43273939e-07f);
  pc = fmaf(pc, wc, -3.5233877e-06f);
  pc = fmaf(pc, wc, -4.39150654e-06f);
  pc = fmaf(pc, wc, 0.00021858087f);
  pc = fmaf(pc, wc, -0.00125372503f);
  pc = fmaf(pc, wc, -0.00417768164f);
  pc = fmaf(pc, wc, 0.246640727f);
  pc = fmaf(pc, wc, 1.50140941f);
  // (the tail polynomial only when some lane of the wave needs it: w >= 5
  // means y < ~3.4e-3, so most waves skip it; a select, not a lane branch)
  float pt = pc;
  if (__builtin_amdgcn_ballot_w64(!(w < 5.0f))) {
    const float wt = __builtin_sqrtf(w) - 3.0f;
    pt = -0.000200214257f;
    pt = fmaf(pt, wt, 0.000100950558f);
    pt = fmaf(pt, wt, 0.00134934322f);
    pt = fmaf(pt, wt, -0.00367342844f);
    pt = fmaf(pt, wt, 0.00573950773f);
    pt = fmaf(pt, wt, -0.0076224613f);
    pt = fmaf(pt, wt, 0.00943887047f);
    pt = fmaf(pt, wt, 1.00167406f);
    pt = fmaf(pt, wt, 2.83297682f);
  }
  const double p = (double)(w < 5.0f ? pc : pt);
  return p * (1.0 - y);
}

// the first Philox block of draw (seed, gi, stream): computed by the caller,
// where the key (the suggestion's seed) is wave-uniform and its round
// schedule stays in scalar registers
__device__ __forceinline__ U4 draw_block0(uint64_t seed, uint64_t gi, uint32_t stream) {
  return philox(U4{(uint32_t)gi, (uint32_t)(gi >> 32), stream, 0u}, (uint32_t)seed,
                (uint32_t)(seed >> 32));
}

// (r0: the words of draw4's first Philox block, draw_block0: u0 picks, u1
// inverts; the second block -- u2 -- only for the unbounded Box-Muller)
template <int CAP>
__device__ double draw_table_from(const tpe_hp &H, int K, const double *__restrict__ mu,
                                  const double *__restrict__ sg, const DrawTableT<CAP> &T,
                                  U4 r0, uint64_t seed, uint64_t gi, uint32_t stream) {
  const double u0 = u53(r0.x, r0.y), u1 = u53(r0.z, r0.w);
  const int k = pick_cdf(T.cdf, K, u0);
  if (H.family == TPE_CAT) return (double)k;
  double x;
  if (H.flags & (TPE_HAS_LOW | TPE_HAS_HIGH)) {
    // one tail probability q and side: x = mu + side * sqrt2 sigma erfcinv(2q)
    const double s2 = 1.4142135623730951 * sg[k], b = T.base[k], m = T.mass[k];
    const int md = T.mode[k];
    double q, side;
    if (md == 1) { q = b - u1 * m; side = 1.0; }          // upper tail Q
    else {
      const double pp = b + u1 * m;                        // Phi
      if (md == 2 || pp < 0.5) { q = pp; side = -1.0; }
      else { q = 1.0 - pp; side = 1.0; }
    }
    x = mu[k] + side * s2 * erfcinv_fast(2.0 * q);
    if (!(x >= H.low)) x = H.low;  // rounding at the bounds / zero-mass picks
    if (!(x < H.high)) x = nextafter(H.high, -INFINITY);
  } else {
    const U4 c1{(uint32_t)gi, (uint32_t)(gi >> 32), stream, 1u};
    const U4 r1 = philox(c1, (uint32_t)seed, (uint32_t)(seed >> 32));
    const double u2 = u53(r1.x, r1.y);
    x = mu[k] + sg[k] * (sqrt(-2.0 * log(1.0 - u1)) * cospi(2.0 * u2));
  }
  if (H.family == TPE_LGMM) x = exp(x);
  if (H.flags & TPE_HAS_Q) x = rint(x / H.q) * H.q;
  return x;
}
template <int CAP>
__device__ double draw_table(const tpe_hp &H, int K, const double *__restrict__ mu,
                             const double *__restrict__ sg, const DrawTableT<CAP> &T,
                             uint64_t seed, uint64_t gi, uint32_t stream) {
  return draw_table_from(H, K, mu, sg, T, draw_block0(seed, gi, stream), seed, gi, stream);
}

// pick_cdf's index without its loop, for tables of <= CAP components: the
// number of k < K - 1 with cdf[k] <= t (the CDF is nondecreasing, so that
// count is the first k with cdf[k] > t, capped at K - 1 -- pick_cdf's value),
// by a fixed ladder of halving steps (one LDS read and a select each)
template <int CAP>
__device__ __forceinline__ int pick_cdf_ladder(const double *cdf, int K, double t) {
  static_assert((CAP & (CAP - 1)) == 0, "power-of-two table");
  int lo = 0;
#pragma unroll
  for (int step = CAP / 2; step > 0; step >>= 1) {
    const int j = lo + step;
    // (the read is in the table whatever K is: no branch around it)
    const bool ok = (j <= K - 1) & (cdf[min(j, CAP) - 1] <= t);
    lo = ok ? j : lo;
  }
  return lo;
}

// The bounded continuous draw of draw_table_from (GMM / LGMM, truncated to
// [low, high)) for the sorted-draw loop, inline: the descriptor fields are
// wave-uniform arguments (scalar registers, no per-draw descriptor loads or
// call), the pick is the loop-free ladder, the tail branch a select.  The
// arithmetic is draw_table_from's, operation for operation, so the values
// are the same bits (the regeneration tests compare every winner with
// tpe_sample's draw_table).  cdf_last = T.cdf[K - 1]; high_prev =
// nextafter(high, -inf).
template <int CAP>
__device__ __forceinline__ double draw_bounded_inline(const DrawTableT<CAP> &T, int K,
                                                      double cdf_last,
                                                      const double *__restrict__ mu,
                                                      const double *__restrict__ sg, double low,
                                                      double high, double high_prev, bool logn,
                                                      bool hasq, double qv, U4 r0) {
  const double u0 = u53(r0.x, r0.y), u1 = u53(r0.z, r0.w);
  const int k = pick_cdf_ladder<CAP>(T.cdf, K, u0 * cdf_last);
  const double s2 = 1.4142135623730951 * sg[k], b = T.base[k], m = T.mass[k];
  const int md = T.mode[k];
  // (draw_table_from's codegen: u1 m once, b -/+ it unfused; x by one fma)
  double pu, pp;
  {
#pragma clang fp contract(off)
    const double um = u1 * m;
    pu = b - um;
    pp = b + um;
  }
  const bool lower = md != 1 && (md == 2 || pp < 0.5);
  const double q = md == 1 ? pu : lower ? pp : 1.0 - pp;
  const double side = lower ? -1.0 : 1.0;
  double x = fma(side * s2, erfcinv_fast(2.0 * q), mu[k]);
  if (!(x >= low)) x = low;
  if (!(x < high)) x = high_prev;
  if (logn) x = exp(x);
  if (hasq) x = rint(x / qv) * qv;
  return x;
}

// s is wave-uniform: select the inline seed with an unrolled compare chain
// (a dynamic index into the by-value argument would copy it to scratch)
__device__ __forceinline__ uint64_t suggestion_seed(const ScoreArgs &A, int s) {
  if (s >= A.n_inline_seeds) return A.seeds[s];
  uint64_t v = A.seed_inline[0];
#pragma unroll
  for (int i = 1; i < kInlineSeeds; ++i) v = (s == i) ? A.seed_inline[i] : v;
  return v;
}

// one table draw, out of line: inlined into the grid-stride loop below, the
// inverse CDFs are specialised per descriptor branch and the kernel grows to
// 256 VGPRs
template <int CAP>
__device__ __attribute__((noinline)) double draw_table_ool(const tpe_hp *Hp, int K,
                                                          const double *mu, const double *sg,
                                                          const DrawTableT<CAP> *T, U4 r0,
                                                          uint64_t seed, uint64_t gi,
                                                          uint32_t stream) {
  return draw_table_from(*Hp, K, mu, sg, *T, r0, seed, gi, stream);
}

// the per-draw rejection sampler, out of line (small register footprint for
// the table kernels that fall back to it)
__device__ __attribute__((noinline)) inline double draw_one_ool(
    const tpe_hp *Hp, const MixInfo *I, const double *w, const double *mu, const double *sg,
    uint64_t seed, uint64_t gi, uint32_t stream) {
  return draw_one(*Hp, *I, w, mu, sg, seed, gi, stream);
}

// Active-slot grids (ScoreArgs::compact).  Lane i of the wave tests slot
// s0 + i (+ 64 per round) of the range [s0, s0 + n) for suggestion s; the
// j-th active one (in slot order), or -1 when fewer are active.  Every lane
// of the wave calls it (the result is wave-uniform).
__device__ __forceinline__ int active_slot(const ScoreArgs &A, int s, int s0, int n, int j) {
  const int lane = threadIdx.x & 63;
  const Partial *res = A.results + (int64_t)s * A.n_hp;
  int seen = 0;
  for (int b = 0; b < n; b += 64) {
    const int i = b + lane;
    const bool act = i < n && hp_active(A.hps[A.level_hps[s0 + i]], res, A.cond_parent,
                                        A.cond_branch);
    uint64_t m = __ballot(act);
    const int c = __popcll(m);
    if (j < seen + c) {
      for (int k = seen; k < j; ++k) m &= m - 1;
      return s0 + b + __builtin_ctzll(m);
    }
    seen += c;
  }
  return -1;
}
// the same over the union of suggestions 0 .. n_sug - 1 (value lattices are
// shared by every suggestion of a call)
__device__ __forceinline__ int active_slot_any(const ScoreArgs &A, int n_sug, int s0, int n,
                                               int j) {
  const int lane = threadIdx.x & 63;
  int seen = 0;
  for (int b = 0; b < n; b += 64) {
    const int i = b + lane;
    bool act = false;
    if (i < n) {
      const tpe_hp &H = A.hps[A.level_hps[s0 + i]];
      for (int s = 0; s < n_sug && !act; ++s)
        act = hp_active(H, A.results + (int64_t)s * A.n_hp, A.cond_parent, A.cond_branch);
    }
    uint64_t m = __ballot(act);
    const int c = __popcll(m);
    if (j < seen + c) {
      for (int k = seen; k < j; ++k) m &= m - 1;
      return s0 + b + __builtin_ctzll(m);
    }
    seen += c;
  }
  return -1;
}
// the slot of draw / bucket grid row `row` of suggestion s over slots
// [s0, s0 + n): the row itself, or with compact grids the row-th active slot
// (-1: none; without compaction the caller still tests activity)
__device__ __forceinline__ int row_slot(const ScoreArgs &A, int s, int s0, int n, int row) {
  return A.compact ? active_slot(A, s, s0, n, row) : s0 + row;
}

// One draw block (k_draw<true>, or a draw row of the fused k_lattice): the
// below mixture's table of (suggestion s, level slot) in LDS, then a
// grid-stride pass over the chunk's candidates bx * blockDim + t (+ stride).
// Large draws use several candidates per thread so one table build serves
// 2048 draws.  K > CAP (a stale host routing decision) falls back to the
// rejection sampler: the same distribution, never a silent NaN.
template <int CAP>
__device__ void draw_block(const ScoreArgs &A, int bx, int row, int s, DrawTableT<CAP> &T,
                           int64_t stride) {
  const int slot = row_slot(A, s, 0, A.n_slots, row);
  if (slot < 0) return;
  const int hp = A.level_hps[slot];
  const tpe_hp H = A.hps[hp];
  if (!A.compact && !hp_active(H, A.results + (int64_t)s * A.n_hp, A.cond_parent, A.cond_branch))
    return;
  const int64_t sb = 2 * (int64_t)hp;
  const double *bw = A.mw + sb * A.kcap, *bmu = A.mmu + sb * A.kcap, *bsg = A.msig + sb * A.kcap;
  const int K = A.info[sb].K;
  const bool tab = K >= 1 && K <= CAP;
  if (tab) build_table(H, K, bw, bmu, bsg, T);
  const uint64_t seed = suggestion_seed(A, s);
  double *out = const_cast<double *>(A.cand) + (int64_t)s * A.cand_sstride + (int64_t)slot * A.n_cand;
#pragma unroll 1
  for (int64_t li = (int64_t)bx * blockDim.x + threadIdx.x; li < A.n_cand; li += stride)
    out[li] = tab ? draw_table_ool<CAP>(A.hps + hp, K, bmu, bsg, &T,
                                        draw_block0(seed, (uint64_t)(A.cand_begin + li), (uint32_t)hp),
                                        seed, (uint64_t)(A.cand_begin + li), (uint32_t)hp)
                  : draw_one_ool(A.hps + hp, A.info + sb, bw, bmu, bsg, seed,
                                 (uint64_t)(A.cand_begin + li), (uint32_t)hp);
}

// ------------------------------------------------------------------------
// Value-bucketed draws (k_draw_sorted; k_fit's fused small draws).  NT
// threads draw kSortedBlock consecutive candidates of one (suggestion, slot)
// and, for the per-candidate log-sum-exp and erf kinds, write them grouped
// into kSortBuckets equal-width value buckets of the block's range (log scale
// for LGMM), with their chunk positions.  A scoring tile (64 or 128
// consecutive candidates) then spans a narrow value range, so whole
// component blocks / chunks of a mixture are provably negligible for the wave
// and skipped (tpe_score.hip).  The candidate values are those of the
// unsorted draw (counter = global index); only their order changes, and the
// argmax tie-break uses the original index.  The scatter is stable, so the
// layout does not depend on NT or on thread timing.
// ------------------------------------------------------------------------
constexpr int kSortBuckets = 256;

// Stable counting scatter by an 8-bit bucket: element i of [0, n) goes to
// position dest(i) = (elements of lower buckets) + (elements of its bucket
// with a lower index), independent of thread timing (an atomic-increment
// scatter orders a bucket's elements by arrival, so which scoring tile a
// candidate lands in -- and the log-sum-exp block skip of that tile --
// would vary from run to run).  Wave w takes elements [w * per, ...) in
// order; per (wave, bucket) counts from 8-ballot lane matching, one scan
// over (bucket, wave), then the same walk writes the destinations.
// cnt: NW * 256 ints of LDS; every thread of the block calls it.
// (per bit: the lane's bit sign-extended, its ballot, and the lanes that
// differ in it -- ballot xor the lane's own bit -- or-ed into a mismatch
// mask; three 32-bit ops per half instead of a 64-bit select per bit)
__device__ __forceinline__ uint64_t lanes_equal8(uint32_t d, bool v) {
  uint32_t mlo = 0u, mhi = 0u;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const uint32_t x = (uint32_t)__builtin_amdgcn_sbfe((int)d, b, 1);  // 0 or ~0
    const uint64_t bb = __ballot(x != 0u);
    mlo |= (uint32_t)bb ^ x;
    mhi |= (uint32_t)(bb >> 32) ^ x;
  }
  return __ballot(v) & ~(((uint64_t)mhi << 32) | mlo);
}

// counts, then per (bucket, wave) output bases in cnt (16-bit halves); every
// thread of the block calls it.  Returns the wave's row range [r0, r1).
template <int NW>
__device__ __forceinline__ void bucket_bases(const unsigned char *bk, int n, uint32_t *cnt,
                                             int &r0, int &r1) {
  // counts and bases per (wave, bucket) are < 2^16 (n <= kSortedBlock): two
  // buckets per 32-bit LDS word, bucket b in half b & 1 of word b >> 1
  static_assert(kSortedBlock < 65536, "16-bit bucket counts");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int per = ((n + NW * 64 - 1) / (NW * 64)) * 64;
  r0 = w * per;
  r1 = min(n, r0 + per);
  uint32_t *mine = cnt + w * (kSortBuckets / 2);
  for (int b = lane; b < kSortBuckets / 2; b += 64) mine[b] = 0u;
  // (a wave's LDS ops complete in order: no barrier between its own rows)
  // counts: one LDS atomic per element into the wave's own bins (the order
  // of the adds does not matter; the ranks below keep the scatter stable)
  for (int base = r0; base < r1; base += 64) {
    const int i = base + lane;
    if (i < r1) {
      const unsigned d = bk[i];
      __hip_atomic_fetch_add(&mine[d >> 1], 1u << ((d & 1) * 16), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __syncthreads();
  // bucket b (thread b of the first 256): its total over the waves, a block
  // scan of the totals, then the (bucket, wave) bases in place (the even
  // thread of each pair writes the pair's word)
  static_assert(NW * 64 >= 256, "one thread per bucket");
  __shared__ int wtot[4];
  const int hb = (threadIdx.x & 1) * 16;
  int tot = 0;
  if (threadIdx.x < 256)
    for (int q = 0; q < NW; ++q) tot += (int)((cnt[q * 128 + (threadIdx.x >> 1)] >> hb) & 0xffffu);
  int x = tot;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63 && w < 4) wtot[w] = x;
  __syncthreads();
  if (threadIdx.x < 256) {
    int acc = x - tot;
    for (int q = 0; q < w; ++q) acc += wtot[q];
    for (int q = 0; q < NW; ++q) {
      const uint32_t word = cnt[q * 128 + (threadIdx.x >> 1)];
      const int c = (int)((word >> hb) & 0xffffu);
      const int acc1 = __shfl_xor(acc, 1, 64);  // (the pair's other bucket)
      if (!(threadIdx.x & 1)) cnt[q * 128 + (threadIdx.x >> 1)] = (uint32_t)acc | ((uint32_t)acc1 << 16);
      acc += c;
    }
  }
  __syncthreads();
}

// the destination of element i of the wave's current row (its bucket's base
// for the wave plus its rank among the row's earlier lanes of that bucket),
// and the bucket's base moved past the row's members
__device__ __forceinline__ int bucket_rank(uint32_t *mine, uint32_t d, bool v) {
  const int lane = threadIdx.x & 63;
  const uint64_t mt = lanes_equal8(d, v);
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int sh = (int)(d & 1) * 16;
  const int p = (int)((mine[d >> 1] >> sh) & 0xffffu) + __popcll(mt & lt);
  // (leaders of the two buckets of one word may update it together: atomic)
  if (v && lane == __ffsll((long long)mt) - 1)
    __hip_atomic_fetch_add(&mine[d >> 1], (uint32_t)__popcll(mt) << sh, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
  return p;
}

template <int NW, typename Dest>
__device__ __forceinline__ void stable_bucket_scatter(const unsigned char *bk, int n, uint32_t *cnt,
                                                      Dest dest) {
  int r0, r1;
  bucket_bases<NW>(bk, n, cnt, r0, r1);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t *mine = cnt + w * (kSortBuckets / 2);
  for (int base = r0; base < r1; base += 64) {
    const int i = base + lane;
    const bool v = i < r1;
    const uint32_t d = v ? bk[i] : 0u;
    const int p = bucket_rank(mine, d, v);
    if (v) dest(i, p);
  }
}

// The same order, written with coalesced stores: each lane keeps its rows'
// values and destinations in registers (at most MAXR rows per wave), the
// values are permuted inside LDS (xs, in place between barriers), written
// in destination order, and then xs holds the source positions for the
// position write.  (The scattered stores of stable_bucket_scatter -- 64
// lines per store instruction -- were a third of k_draw_sorted's time.)
template <int NW, int MAXR>
__device__ __forceinline__ void stable_bucket_permute(const unsigned char *bk, int n, uint32_t *cnt,
                                                      double *xs, double *__restrict__ out,
                                                      int32_t *__restrict__ po, int64_t base) {
  int r0, r1;
  bucket_bases<NW>(bk, n, cnt, r0, r1);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t *mine = cnt + w * (kSortBuckets / 2);
  double xv[MAXR];
  int pd[MAXR];
#pragma unroll
  for (int j = 0; j < MAXR; ++j) {
    pd[j] = -1;
    xv[j] = 0.0;
    if (r0 + 64 * j < r1) {  // (wave-uniform)
      const int i = r0 + 64 * j + lane;
      const bool v = i < r1;
      const uint32_t d = v ? bk[i] : 0u;
      const int p = bucket_rank(mine, d, v);
      if (v) { pd[j] = p; xv[j] = xs[i]; }
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < MAXR; ++j)
    if (pd[j] >= 0) xs[pd[j]] = xv[j];
  __syncthreads();
  for (int p = threadIdx.x; p < n; p += NW * 64) out[p] = xs[p];
  __syncthreads();
  int32_t *src = reinterpret_cast<int32_t *>(xs);
#pragma unroll
  for (int j = 0; j < MAXR; ++j)
    if (pd[j] >= 0) src[pd[j]] = r0 + 64 * j + lane;
  __syncthreads();
  for (int p = threadIdx.x; p < n; p += NW * 64) po[p] = (int32_t)(base + src[p]);
}


// Lookup slots (categorical, value lattice) drawn inside the scoring tile
// instead of by the sorted draw (ScoreArgs::lookup_draw): below mixtures of
// 1 .. kFuseTab components, whose LDS table the tile builds (DrawTableT<
// kFuseTab>; the table, hence every draw, is the one the draw kernels build
// for that K).  Both kernels decide from the same device-side K.
__device__ __forceinline__ bool lookup_inline(const ScoreArgs &A, int K) {
  return A.lookup_draw && K >= 1 && K <= kFuseTab;
}

// The bucketing key of a sorted block: the value, or for log-scale slots
// its fp32 log2 (v_log_f32 of the value rounded to fp32: buckets only group
// candidates, so the key needs no more than fp32 and one instruction --
// round 5's fp64 fast_log cost ~30 VALU, twice per LGMM candidate).  Draws
// and given candidates (k_sort_ext) bucket through this same function.
__device__ __forceinline__ double sort_key(double x, bool lg) {
  return lg ? (double)__builtin_amdgcn_logf((float)x) : x;
}

template <int CAP, int NT>
struct SortedDrawLds {
  DrawTableT<CAP> T;
  double xs[kSortedBlock];          // the block's draws, in draw order
  unsigned char bk[kSortedBlock];   // their buckets
  uint32_t cnt[NT / 64 * kSortBuckets / 2];  // stable scatter counts / bases (16-bit pairs)
  double red[2][NT / 64];
};

// One sorted block: candidates [base, base + kSortedBlock) of level slot
// `slot` for suggestion s (bucket: value-bucket them; lg: in log scale).
// EXT (k_sort_ext): the values come from src[slot][n_cand] instead of the
// draw (given candidates scored exactly as a large draw's are).  Every
// thread of the block calls it.
// FAST: the launch's drawn slots are all bounded continuous ones with a
// table (the host checks it, launch_draw_sorted): only the inline draw is
// compiled in -- no out-of-line draw call, whose calling convention would
// set the kernel's registers (143 VGPRs against ~60)
template <int CAP, int NT, bool EXT, bool FAST = false>
__device__ __forceinline__ void sorted_block_body(const ScoreArgs &A, int slot, int s,
                                                  int64_t base, bool bucket, bool lg,
                                                  int32_t *__restrict__ pos_out,
                                                  const double *__restrict__ src,
                                                  SortedDrawLds<CAP, NT> &L) {
  const int hp = A.level_hps[slot];
  const tpe_hp H = A.hps[hp];
  const int64_t sb = 2 * (int64_t)hp;
  const double *bw = A.mw + sb * A.kcap, *bmu = A.mmu + sb * A.kcap, *bsg = A.msig + sb * A.kcap;
  const int K = A.info[sb].K;
  const bool tab = !EXT && K >= 1 && K <= CAP;
  if constexpr (!EXT) {
    if (tab) build_table(H, K, bw, bmu, bsg, L.T);
  }
  const uint64_t seed = suggestion_seed(A, s);
  const int n = (int)min<int64_t>((int64_t)1 << A.sort_log2, A.n_cand - base);
  const int64_t off = (int64_t)s * A.cand_sstride + (int64_t)slot * A.n_cand + base;
  double *out = const_cast<double *>(A.cand) + off;
  const int t = threadIdx.x;
  double lo = INFINITY, hi = -INFINITY;
  // each candidate: to the output (unbucketed slot) or to the LDS staging
  // with its bucketing key folded into the block range
  auto emit = [&](int i, double x) {
    if (!bucket) {
      out[i] = x;
      return;
    }
    L.xs[i] = x;
    const double key = sort_key(x, lg);
    if (fabs(key) < INFINITY) { lo = fmin(lo, key); hi = fmax(hi, key); }
  };
  // bounded continuous slots with a table (config 4 / 5's hps): the table
  // draw inline with the descriptor in scalar registers (draw_bounded_inline,
  // the same values); everything else through the out-of-line draws
  const bool fast = FAST || (!EXT && tab && H.family != TPE_CAT && (H.flags & TPE_HAS_LOW) &&
                             (H.flags & TPE_HAS_HIGH));
  if (fast) {
    const double cdf_last = L.T.cdf[K - 1];
    const double high_prev = nextafter(H.high, -INFINITY);
    const bool logn = H.family == TPE_LGMM, hasq = (H.flags & TPE_HAS_Q) != 0;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll 1
    for (int i = t; i < n; i += NT) {
      const uint64_t gi = (uint64_t)(A.cand_begin + base + i);
      const U4 r0 = philox(U4{(uint32_t)gi, (uint32_t)(gi >> 32), (uint32_t)hp, 0u}, k0, k1);
      emit(i, draw_bounded_inline<CAP>(L.T, K, cdf_last, bmu, bsg, H.low, H.high, high_prev,
                                       logn, hasq, H.q, r0));
    }
  } else if constexpr (!FAST) {
#pragma unroll 1
    for (int i = t; i < n; i += NT) {
      const uint64_t gi = (uint64_t)(A.cand_begin + base + i);
      double x;
      if constexpr (EXT) {
        (void)gi; (void)seed; (void)bw;
        x = src[(int64_t)slot * A.n_cand + base + i];
      } else {
        x = tab ? draw_table_ool<CAP>(A.hps + hp, K, bmu, bsg, &L.T,
                                      draw_block0(seed, gi, (uint32_t)hp), seed, gi, (uint32_t)hp)
                : draw_one_ool(A.hps + hp, A.info + sb, bw, bmu, bsg, seed, gi, (uint32_t)hp);
      }
      emit(i, x);
    }
  }
  if (!bucket) return;
  // block range of the finite keys
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, o, 64));
    hi = fmax(hi, __shfl_xor(hi, o, 64));
  }
  const int lane = t & 63, wv = t >> 6;
  if (lane == 0) { L.red[0][wv] = lo; L.red[1][wv] = hi; }
  __syncthreads();
  lo = INFINITY; hi = -INFINITY;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) { lo = fmin(lo, L.red[0][w]); hi = fmax(hi, L.red[1][w]); }
  const double scale = hi > lo ? (double)kSortBuckets / (hi - lo) : 0.0;
  for (int i = t; i < n; i += NT) {
    const double key = sort_key(L.xs[i], lg);
    int b = kSortBuckets - 1;
    if (fabs(key) < INFINITY) b = min(kSortBuckets - 1, max(0, (int)((key - lo) * scale)));
    L.bk[i] = (unsigned char)b;
  }
  __syncthreads();
  // scatter into the block's slice, stable
  int32_t *po = pos_out + off;
  if constexpr (NT >= 512) {
    stable_bucket_permute<NT / 64, kSortedBlock / NT>(L.bk, n, L.cnt, L.xs, out, po, base);
  } else {
    stable_bucket_scatter<NT / 64>(L.bk, n, L.cnt, [&](int i, int p) {
      out[p] = L.xs[i];
      po[p] = (int32_t)(base + i);
    });
  }
}

}  // namespace tpe
