// tpe_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the TPE hot path.
//
// Reference semantics (pminervini/hyperopt, hyperopt/tpe.py); the split and
// the Parzen fits are in tpe_fit.hip.
//   k_draw   : candidate draw (GMM1/LGMM1/categorical,   tpe.py:62-93, 216-250
//               counter-based Philox in registers), below/above lpdf
//               (log-sum-exp or linear erf-CDF sum), EI and block argmax
//                                                         tpe.py:684-698, 749-759
//   k_reduce / k_merge : grid / cross-device argmax with numpy semantics
//
// Layout: one 64-lane wave owns 64 candidates; mixture components are read
// with wave-uniform addresses (scalar loads -> SGPR operands), so no LDS or
// VGPRs are spent on them and HBM traffic per pair is ~0.
#include <math.h>

#include <algorithm>

#include "tpe_device.hpp"

namespace tpe {

constexpr int kSortMax = 8192;  // candidates per bucketing chunk

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

// One GMM1/LGMM1/categorical draw (tpe.py:62-93, 216-250; stochastic.py:104)
__device__ double draw_one(const tpe_hp &H, const MixInfo &I,
                           const double *__restrict__ w,
                           const double *__restrict__ mu,
                           const double *__restrict__ sg, uint64_t seed,
                           uint64_t gi, uint32_t stream) {
  if (H.family == TPE_CAT) {
    const Draw d = draw4(seed, gi, stream, 0);
    return (double)pick(w, I.K, d.u0 * I.wsum);
  }
  const bool bounded = (H.flags & (TPE_HAS_LOW | TPE_HAS_HIGH)) != 0;
  double x = 0.0;
  bool ok = false;
  int k = 0;
  Draw d{};
  for (uint32_t it = 0; it < 64 && !ok; ++it) {
    d = draw4(seed, gi, stream, it);
    k = pick(w, I.K, d.u0 * I.wsum);
    const double z = sqrt(-2.0 * log(1.0 - d.u1)) * cospi(2.0 * d.u2);
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
// scoring inner loops
// ------------------------------------------------------------------------
// log-sum-exp slice in log2 units: m = max_k t_k, s = sum_k 2^(t_k - m),
// t_k = c_k - ((y - mu_k) a_k)^2.  Exponent arguments and the accumulator are
// fp64; 2^(t-m) in [0,1] is one v_exp_f32 (rel. err ~1e-7 per term).
__device__ __forceinline__ void lse_slice(const Coef *__restrict__ c, int k0, int k1, int ks,
                                          double y, double &m_out, double &s_out) {
  double m = -INFINITY;
#pragma unroll 4
  for (int k = k0; k < k1; k += ks) {
    const double z = (y - c[k].x) * c[k].y;
    m = fmax(m, fma(-z, z, c[k].z));
  }
  double s = 0.0;
  if (m != -INFINITY || !(fabs(y) < INFINITY)) {
#pragma unroll 4
    for (int k = k0; k < k1; k += ks) {
      const double z = (y - c[k].x) * c[k].y;
      const double t = fma(-z, z, c[k].z);
      s += (double)__builtin_amdgcn_exp2f((float)(t - m));
    }
  }
  m_out = m;
  s_out = s;
}

// linear-space sum of w_k (Phi_k(ub) - Phi_k(lb)), tpe.py:146-160 / 284-299.
// Components with both bounds beyond 6.5 sigma on one side contribute an
// exact 0 in float64 (erf saturates to +-1), so they are skipped.
template <bool LOGN>
__device__ __forceinline__ double erf_slice(const Coef *__restrict__ c, int k0,
                                            int k1, int ks, double ub, double lb) {
#pragma clang fp contract(off)
  double prob = 0.0;
  for (int k = k0; k < k1; k += ks) {
    const double zu = (ub - c[k].x) * c[k].y;
    const double zl = (lb - c[k].x) * c[k].y;
    const bool dead = (zu >= 6.5 && zl >= 6.5) || (zu <= -6.5 && zl <= -6.5);
    if (!dead) {
      const double wk = c[k].z;
      double cu, cl;
      if (LOGN) {
        cu = .5 + .5 * erf(zu);
        cl = .5 + .5 * erf(zl);
      } else {
        cu = 0.5 * (1.0 + erf(zu));
        cl = 0.5 * (1.0 + erf(zl));
      }
      double inc = wk * cu;
      inc -= wk * cl;
      prob += inc;
    }
  }
  return prob;
}

__device__ __forceinline__ bool better(double sa, int64_t ia, double sb, int64_t ib) {
  if (ia < 0) return false;
  if (ib < 0) return true;
  const bool na = sa != sa, nb = sb != sb;
  if (na || nb) return (na && nb) ? ia < ib : na;
  if (sa != sb) return sa > sb;
  return ia < ib;
}

__device__ __forceinline__ void wave_best(double &s, double &v, int64_t &i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double os = __shfl_xor(s, o, 64);
    const double ov = __shfl_xor(v, o, 64);
    const int64_t oi = __shfl_xor(i, o, 64);
    if (better(os, oi, s, i)) { s = os; v = ov; i = oi; }
  }
}

__device__ __forceinline__ void slice_bounds(int K, int part, int parts, int &k0, int &k1) {
  const int per = (K + parts - 1) / parts;
  k0 = min(K, part * per);
  k1 = min(K, k0 + per);
}

__device__ __forceinline__ bool hp_active(const tpe_hp &H, const Partial *res,
                                          const int32_t *cp, const int32_t *cb) {
  if (H.cond_count == 0) return true;
  for (int c = 0; c < H.cond_count; ++c) {
    const Partial &r = res[cp[H.cond_begin + c]];
    if (r.active && r.index >= 0 && r.value == (double)cb[H.cond_begin + c]) return true;
  }
  return false;
}

__device__ __forceinline__ uint64_t suggestion_seed(const ScoreArgs &A, int s) {
  return s < kInlineSeeds && A.n_inline_seeds > s ? A.seed_inline[s] : A.seeds[s];
}

// Candidate draws of one level (all its hps): grid = (blocks, hps of the
// level, suggestions), one candidate per thread per step.  Counter = (global
// candidate index, hp id, iteration), key = suggestion seed, so the
// candidate set does not depend on how [0, n_cand) is chunked or sharded.
__global__ __launch_bounds__(256) void k_draw(ScoreArgs A) {
  const int slot = blockIdx.y, s = blockIdx.z;
  const int hp = A.level_hps[slot];
  const tpe_hp H = A.hps[hp];
  if (!hp_active(H, A.results + (int64_t)s * A.n_hp, A.cond_parent, A.cond_branch)) return;
  const int64_t sb = 2 * (int64_t)hp;
  const MixInfo ib = A.info[sb];
  const double *bw = A.mw + sb * A.kcap, *bmu = A.mmu + sb * A.kcap, *bsg = A.msig + sb * A.kcap;
  const uint64_t seed = suggestion_seed(A, s);
  double *out = const_cast<double *>(A.cand) + (int64_t)s * A.cand_sstride + (int64_t)slot * A.n_cand;
  for (int64_t li = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; li < A.n_cand;
       li += (int64_t)gridDim.x * blockDim.x)
    out[li] = draw_one(H, ib, bw, bmu, bsg, seed, (uint64_t)(A.cand_begin + li), (uint32_t)hp);
}

// Bucket each 8192-candidate chunk of the erf-kind hps by value (counting
// sort into 256 equal-width buckets of the chunk's range, in the coordinate
// the erf argument is linear in), keeping each candidate's original
// position.  A wave then holds neighbouring candidates and a mixture
// component far from all of them (both erf saturated) is skipped by the
// whole wave.  Order inside a bucket is irrelevant: every candidate is
// scored on its own and the argmax tie-break uses the original index.
constexpr int kBuckets = 256;
__global__ __launch_bounds__(1024) void k_bucket(ScoreArgs A, int32_t *__restrict__ pos_out) {
  extern __shared__ __attribute__((aligned(16))) double dyn_lds[];
  __shared__ int hist[kBuckets];
  __shared__ double red_lo[16], red_hi[16];
  const int slot = blockIdx.y, s = blockIdx.z;
  const int hp = A.level_hps[slot];
  const tpe_hp H = A.hps[hp];
  const int kind = score_kind(H);
  if (kind != KIND_ERF_G && kind != KIND_ERF_L) return;
  if (!hp_active(H, A.results + (int64_t)s * A.n_hp, A.cond_parent, A.cond_branch)) return;
  const int64_t base = (int64_t)blockIdx.x * kSortMax;
  if (base >= A.n_cand) return;
  const int n = (int)min<int64_t>(kSortMax, A.n_cand - base);
  const int64_t off = (int64_t)s * A.cand_sstride + (int64_t)slot * A.n_cand + base;
  double *cand = const_cast<double *>(A.cand) + off;
  double *xs = dyn_lds;                                        // [8192] values
  unsigned char *bk = reinterpret_cast<unsigned char *>(dyn_lds + kSortMax);  // [8192]
  const bool lg = kind == KIND_ERF_L;
  double lo = INFINITY, hi = -INFINITY;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double x = cand[i];
    xs[i] = x;
    const double t = lg ? log(fmax(x, 1e-300)) : x;
    if (t == t && fabs(t) < INFINITY) { lo = fmin(lo, t); hi = fmax(hi, t); }
  }
  for (int b = threadIdx.x; b < kBuckets; b += blockDim.x) hist[b] = 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, o, 64));
    hi = fmax(hi, __shfl_xor(hi, o, 64));
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { red_lo[wid] = lo; red_hi[wid] = hi; }
  __syncthreads();
  lo = INFINITY; hi = -INFINITY;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { lo = fmin(lo, red_lo[w]); hi = fmax(hi, red_hi[w]); }
  const double scale = hi > lo ? (double)kBuckets / (hi - lo) : 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double x = xs[i];
    const double t = lg ? log(fmax(x, 1e-300)) : x;
    int b = kBuckets - 1;
    if (t == t && fabs(t) < INFINITY) b = min(kBuckets - 1, max(0, (int)((t - lo) * scale)));
    bk[i] = (unsigned char)b;
    atomicAdd(&hist[b], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int b = 0; b < kBuckets; ++b) { const int c = hist[b]; hist[b] = acc; acc += c; }
  }
  __syncthreads();
  int32_t *po = pos_out + off;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int p = atomicAdd(&hist[bk[i]], 1);
    cand[p] = xs[i];
    po[p] = (int32_t)(base + i);
  }
}

// Scoring kernel, one instantiation per lpdf kind so each keeps its own
// register budget (the erf path must not cap the log-sum-exp path's
// occupancy).  grid = (candidate-tile blocks, hps of the group, suggestions);
// 4 waves per block; with ks > 1 the waves of a 64-candidate group split the
// components and combine their partial sums through LDS.
constexpr int kScoreWaves = 16;  // 1024-thread scoring blocks

template <int KIND>
__global__ __launch_bounds__(1024) void k_score(ScoreArgs A, const Coef *__restrict__ coef,
                                               const double *__restrict__ cand_all) {
  constexpr bool LSE = KIND == KIND_LSE_G || KIND == KIND_LSE_L;
  constexpr bool ERF = KIND == KIND_ERF_G || KIND == KIND_ERF_L;
  constexpr bool CAT = KIND == KIND_CAT;
  constexpr bool LOGN = KIND == KIND_LSE_L || KIND == KIND_ERF_L;
  __shared__ double red[kScoreWaves][4][64];
  __shared__ double bs[kScoreWaves], bv[kScoreWaves];
  __shared__ int64_t bi[kScoreWaves];
  const int slot = blockIdx.y, s = blockIdx.z;
  const int hp = A.level_hps[slot];
  const tpe_hp H = A.hps[hp];
  Partial *pbase = A.partial + ((int64_t)s * A.n_hp + hp) * A.pstride;
  Partial *pout = pbase + blockIdx.x;

  const bool act = A.force_active || hp_active(H, A.results + (int64_t)s * A.n_hp,
                                                  A.cond_parent, A.cond_branch);
  if (!act) {   // every block writes the same "inactive" record
    if (threadIdx.x == 0) A.results[(int64_t)s * A.n_hp + hp] = Partial{NAN, NAN, -1, 0, 0};
    return;
  }
  const int64_t sb = 2 * (int64_t)hp, sa = sb + 1;
  const MixInfo ib = A.info[sb], ia = A.info[sa];
  const Coef *__restrict__ cb = coef + sb * A.kcap;
  const Coef *__restrict__ ca = coef + sa * A.kcap;
  const int64_t coff = (int64_t)s * A.cand_sstride + (int64_t)(A.cand_slot0 + slot) * A.n_cand;
  const double *__restrict__ cand = cand_all + coff;
  const int32_t *__restrict__ cpos = A.cand_pos ? A.cand_pos + coff : nullptr;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ks = A.ks, groups = kScoreWaves / ks;
  const int grp = wave / ks, kp = wave % ks;
  const int TC = 64 * groups;
  // wave kp of a candidate group takes components kp, kp+ks, ... (strided, so
  // the live components of sorted candidates spread over the group's waves);
  // wave-uniform bounds -> scalar (SGPR) component loads
  const int kb0 = __builtin_amdgcn_readfirstlane(kp), kb1 = __builtin_amdgcn_readfirstlane(ib.K);
  const int ka0 = kb0, ka1 = __builtin_amdgcn_readfirstlane(ia.K);
  const int kst = __builtin_amdgcn_readfirstlane(ks);

  double best_s = NAN, best_v = NAN;
  int64_t best_i = -1;
  for (int tile = blockIdx.x; tile < A.tiles; tile += gridDim.x) {
    const int64_t li = (int64_t)tile * TC + grp * 64 + lane;
    const bool valid = li < A.n_cand;
    const double x = valid ? cand[li] : 0.0;
    double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
    if constexpr (LSE) {
      const double y = LOGN ? log(x) : x;
      lse_slice(cb, kb0, kb1, kst, y, p0, p1);
      lse_slice(ca, ka0, ka1, kst, y, p2, p3);
    } else if constexpr (ERF) {
      const double hq = H.q / 2.0;
      double ub, lb;
      if constexpr (!LOGN) {
        ub = (H.flags & TPE_HAS_HIGH) ? np_minimum(x + hq, H.high) : x + hq;
        lb = (H.flags & TPE_HAS_LOW) ? np_maximum(x - hq, H.low) : x - hq;
      } else {
        const double u = (H.flags & TPE_HAS_HIGH) ? np_minimum(x + hq, exp(H.high)) : x + hq;
        double l = (H.flags & TPE_HAS_LOW) ? np_maximum(x - hq, exp(H.low)) : x - hq;
        l = np_maximum(0.0, l);
        ub = u < 0.0 ? NAN : log(np_maximum(u, kEPS));
        lb = log(np_maximum(l, kEPS));
      }
      p0 = erf_slice<LOGN>(cb, kb0, kb1, kst, ub, lb);
      p2 = erf_slice<LOGN>(ca, ka0, ka1, kst, ub, lb);
    }
    if (!CAT && ks > 1) {
      red[wave][0][lane] = p0; red[wave][1][lane] = p1;
      red[wave][2][lane] = p2; red[wave][3][lane] = p3;
      __syncthreads();
    }
    if (kp == 0 && valid) {
      double lpb, lpa;
      if constexpr (LSE) {
        double mb = p0, smb = p1, ma = p2, sma = p3;
        for (int j = 1; j < ks; ++j) {
          const int wv = grp * ks + j;
          const double m2 = red[wv][0][lane], s2 = red[wv][1][lane];
          const double m4 = red[wv][2][lane], s4 = red[wv][3][lane];
          if (m2 > mb) { smb = smb * exp2(mb - m2) + s2; mb = m2; }
          else if (m2 != -INFINITY || s2 != s2) smb += s2 * exp2(m2 - mb);
          if (m4 > ma) { sma = sma * exp2(ma - m4) + s4; ma = m4; }
          else if (m4 != -INFINITY || s4 != s4) sma += s4 * exp2(m4 - ma);
        }
        const double LN2 = 0.6931471805599453;
        lpb = (mb == -INFINITY) ? NAN : (mb + log2(smb)) * LN2;
        lpa = (ma == -INFINITY) ? NAN : (ma + log2(sma)) * LN2;
        if constexpr (LOGN) { const double lx = log(x); lpb -= lx; lpa -= lx; }
      } else if constexpr (ERF) {
        double pb = p0, pa = p2;
        for (int j = 1; j < ks; ++j) {
          pb += red[grp * ks + j][0][lane];
          pa += red[grp * ks + j][2][lane];
        }
        lpb = log(pb) - ib.log_pacc;
        lpa = log(pa) - ia.log_pacc;
      } else {
        const int64_t c = (int64_t)x;
        const bool in = (x >= 0.0) && (c < ib.K) && ((double)c == x);
        lpb = in ? cb[c].x : NAN;
        lpa = in ? ca[c].x : NAN;
      }
      const int64_t lo = cpos ? (int64_t)cpos[li] : li;   // original position
      if (A.out_lb) A.out_lb[lo] = lpb;
      if (A.out_la) A.out_la[lo] = lpa;
      const int64_t gi = A.cand_begin + lo;
      const double sc = lpb - lpa;
      if (better(sc, gi, best_s, best_i)) { best_s = sc; best_v = x; best_i = gi; }
    }
    if (!CAT && ks > 1) __syncthreads();
  }
  wave_best(best_s, best_v, best_i);
  if (lane == 0) { bs[wave] = best_s; bv[wave] = best_v; bi[wave] = best_i; }
  __syncthreads();
  __shared__ int last;
  if (threadIdx.x == 0) {
    for (int w = 1; w < kScoreWaves; ++w)
      if (better(bs[w], bi[w], best_s, best_i)) { best_s = bs[w]; best_v = bv[w]; best_i = bi[w]; }
    *pout = Partial{best_s, best_v, best_i, 1, 0};
    // publish the block record, then take an arrival ticket (agent-scope
    // release / acquire, cdna_hip_programming.md Guideline 16 counter form)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t *tk = A.ticket + (int64_t)s * A.n_hp + hp;
    const uint32_t t = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == gridDim.x - 1) ? 1 : 0;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (!last || wave != 0) return;
  // the last-arriving block reduces every block's record (k_reduce fused)
  double fs = NAN, fv = NAN;
  int64_t fi = -1;
  for (int i = lane; i < (int)gridDim.x; i += 64) {
    const Partial q = pbase[i];
    if (better(q.score, q.index, fs, fi)) { fs = q.score; fv = q.value; fi = q.index; }
  }
  wave_best(fs, fv, fi);
  if (lane == 0) {
    Partial *r = A.results + (int64_t)s * A.n_hp + hp;
    if (!(A.accumulate && better(r->score, r->index, fs, fi))) *r = Partial{fs, fv, fi, 1, 0};
  }
}

// grid reduce: one block per (slot, suggestion)
__global__ __launch_bounds__(64) void k_reduce(const int32_t *__restrict__ level_hps,
                                               int32_t n_slots, int32_t n_hp,
                                               int32_t grid_x, int32_t accumulate,
                                               const Partial *__restrict__ partial,
                                               Partial *__restrict__ results) {
  const int slot = blockIdx.x, s = blockIdx.y;
  const Partial *p = partial + ((int64_t)s * n_slots + slot) * grid_x;
  Partial *r = results + (int64_t)s * n_hp + level_hps[slot];
  double bs_ = NAN, bv_ = NAN;
  int64_t bi_ = -1;
  const int active = grid_x > 0 ? p[0].active : 1;
  for (int i = threadIdx.x; i < grid_x; i += 64)
    if (better(p[i].score, p[i].index, bs_, bi_)) { bs_ = p[i].score; bv_ = p[i].value; bi_ = p[i].index; }
  wave_best(bs_, bv_, bi_);
  if (threadIdx.x == 0) {
    if (accumulate && better(r->score, r->index, bs_, bi_)) return;
    *r = Partial{bs_, bv_, active ? bi_ : -1, active, 0};
  }
}

// cross-device merge of gathered [world][S][P] results
__global__ __launch_bounds__(64) void k_merge(const int32_t *__restrict__ level_hps,
                                              int32_t n_slots, int32_t n_suggest,
                                              int32_t n_hp, int32_t world,
                                              const Partial *__restrict__ g,
                                              Partial *__restrict__ results) {
  const int slot = blockIdx.x, s = blockIdx.y;
  const int hp = level_hps[slot];
  double bs_ = NAN, bv_ = NAN;
  int64_t bi_ = -1;
  int active = 0;
  for (int r = threadIdx.x; r < world; r += 64) {
    const Partial q = g[((int64_t)r * n_suggest + s) * n_hp + hp];
    active |= q.active;
    if (better(q.score, q.index, bs_, bi_)) { bs_ = q.score; bv_ = q.value; bi_ = q.index; }
  }
  wave_best(bs_, bv_, bi_);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) active |= __shfl_xor(active, o, 64);
  if (threadIdx.x == 0)
    results[(int64_t)s * n_hp + hp] = Partial{bs_, bv_, active ? bi_ : -1, active, 0};
}

__global__ __launch_bounds__(256) void k_sample(const tpe_hp *__restrict__ hpd,
                                                const double *__restrict__ w,
                                                const double *__restrict__ mu,
                                                const double *__restrict__ sg,
                                                const MixInfo *__restrict__ info,
                                                uint64_t seed, uint32_t stream,
                                                int64_t offset, int64_t n,
                                                double *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const tpe_hp H = hpd[0];
  const MixInfo I = info[0];
  out[i] = draw_one(H, I, w, mu, sg, seed, (uint64_t)(offset + i), stream);
}

// ------------------------------------------------------------------------
// register-only microkernels for the roofline (tpe_microbench)
// ------------------------------------------------------------------------
template <int WHICH>
__global__ __launch_bounds__(256) void k_micro(int iters, double *sink) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (WHICH == 0) {  // v_exp_f32 throughput, 8 independent chains
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.001f * (t + j);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = __builtin_amdgcn_exp2f(-v[j]);
    }
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j];
    if (acc == 12345.f) sink[t] = acc;
  } else if constexpr (WHICH == 1) {  // fp64 FMA throughput, 8 chains
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 1e-3 * (t + j);
    const double b = 0.999999, c = 1e-7;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fma(v[j], b, c);
    }
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j];
    if (acc == 12345.0) sink[t] = acc;
  } else {  // OCML fp64 erf throughput, 4 chains
    double v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = 1e-3 * (t + j);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = erf(v[j]) - 0.25;
    }
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc += v[j];
    if (acc == 12345.0) sink[t] = acc;
  }
}


hipError_t launch_micro(int which, int blocks, int iters, double *sink, hipStream_t st) {
  switch (which) {
    case 0: k_micro<0><<<blocks, 256, 0, st>>>(iters, sink); break;
    case 1: k_micro<1><<<blocks, 256, 0, st>>>(iters, sink); break;
    default: k_micro<2><<<blocks, 256, 0, st>>>(iters, sink); break;
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------------
// launch wrappers
// ------------------------------------------------------------------------
hipError_t launch_score(const ScoreArgs &a, int32_t kind, int32_t grid_x, hipStream_t st) {
  if (a.n_slots <= 0) return hipSuccess;
  if (a.n_suggest <= 0) return hipSuccess;
  const dim3 g(grid_x, a.n_slots, a.n_suggest);
  switch (kind) {
    case KIND_LSE_G: k_score<KIND_LSE_G><<<g, 1024, 0, st>>>(a, a.coef, a.cand); break;
    case KIND_LSE_L: k_score<KIND_LSE_L><<<g, 1024, 0, st>>>(a, a.coef, a.cand); break;
    case KIND_ERF_G: k_score<KIND_ERF_G><<<g, 1024, 0, st>>>(a, a.coef, a.cand); break;
    case KIND_ERF_L: k_score<KIND_ERF_L><<<g, 1024, 0, st>>>(a, a.coef, a.cand); break;
    default: k_score<KIND_CAT><<<g, 1024, 0, st>>>(a, a.coef, a.cand); break;
  }
  return hipGetLastError();
}

hipError_t launch_draw(const ScoreArgs &a, hipStream_t st) {
  if (a.n_slots <= 0 || a.n_suggest <= 0 || a.n_cand <= 0) return hipSuccess;
  const int64_t want = (a.n_cand + 255) / 256;
  const int64_t cap = std::max<int64_t>(1, 8192 / ((int64_t)a.n_slots * a.n_suggest));
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min(want, cap));
  k_draw<<<dim3(gx, a.n_slots, a.n_suggest), 256, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_bucket(const ScoreArgs &a, int32_t *pos_out, hipStream_t st) {
  if (a.n_slots <= 0 || a.n_suggest <= 0 || a.n_cand <= 0) return hipSuccess;
  const unsigned gx = (unsigned)((a.n_cand + kSortMax - 1) / kSortMax);
  k_bucket<<<dim3(gx, a.n_slots, a.n_suggest), 1024, (size_t)kSortMax * 9, st>>>(a, pos_out);
  return hipGetLastError();
}

hipError_t launch_reduce(const int32_t *level_hps, int32_t n_slots, int32_t n_suggest,
                         int32_t n_hp, int32_t grid_x, int32_t accumulate,
                         const Partial *partial, Partial *results, hipStream_t st) {
  if (n_slots <= 0 || n_suggest <= 0) return hipSuccess;
  k_reduce<<<dim3(n_slots, n_suggest), 64, 0, st>>>(level_hps, n_slots, n_hp, grid_x, accumulate,
                                                    partial, results);
  return hipGetLastError();
}

hipError_t launch_merge(const int32_t *level_hps, int32_t n_slots, int32_t n_suggest,
                        int32_t n_hp, int32_t world, const Partial *gathered,
                        Partial *results, hipStream_t st) {
  if (n_slots <= 0 || n_suggest <= 0) return hipSuccess;
  k_merge<<<dim3(n_slots, n_suggest), 64, 0, st>>>(level_hps, n_slots, n_suggest, n_hp, world,
                                                   gathered, results);
  return hipGetLastError();
}

hipError_t launch_sample(const tpe_hp *hp_dev, const double *mw, const double *mmu,
                         const double *msig, const MixInfo *info, uint64_t seed,
                         uint64_t stream, int64_t offset, int64_t n, double *out,
                         hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = (n + 255) / 256;
  k_sample<<<(unsigned)blocks, 256, 0, st>>>(hp_dev, mw, mmu, msig, info, seed, (uint32_t)stream,
                                             offset, n, out);
  return hipGetLastError();
}

}  // namespace tpe
