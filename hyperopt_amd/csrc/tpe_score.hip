// tpe_score.hip -- below/above lpdf of every candidate, EI and argmax, gfx950.
//
// Reference (pminervini/hyperopt, hyperopt/tpe.py):
//   GMM1_lpdf   tpe.py:104-166     LGMM1_lpdf  tpe.py:259-301
//   categorical_lpdf tpe.py:50-57  broadcast_best tpe.py:749-759 (EI argmax)
//
// Work decomposition.  A block of 16 waves owns a tile of 64 candidates of
// one (suggestion, hp): every wave holds the same 64 candidates, one per lane.
// The components of both mixtures are staged in LDS (batches of 1024, 32 KB)
// and wave w takes the components with index = w (mod 16) of each mixture,
// reading them by broadcast, so a (candidate, component) pair costs only VALU
// work, and the few live components of a quantized mixture (those near the
// tile's candidates) are spread over all 16 waves.  Each wave reduces its
// share per batch (log-sum-exp: a max pass and a sum pass; quantized: a
// linear sum) and merges batches in order; then one wave per mixture merges
// the 16 wave partials in wave order.  The reduction tree depends on (K_b,
// K_a) only, so scores are bitwise independent of the grid, of candidate
// chunking and of multi-GPU sharding.
//
// Log-sum-exp (q = None): t = alpha + y'(beta + gamma y') (two fp64 FMAs, see
// make_coef), 2^(t - max) with v_exp_f32 on the fp64 difference, fp64
// accumulation.  Quantized: the reference's sum_k w (Phi(ub) - Phi(lb)) in
// fp64 with OCML erf, in its operation order; a component whose two erf
// arguments are beyond 6.5 on one side contributes an exact 0 and is skipped
// when every lane of the wave agrees.
#include <math.h>

#include "tpe_device.hpp"

namespace tpe {

constexpr int kWaves = 16;     // waves per scoring block (all share the 64 candidates)
constexpr int kStage = 1024;   // components staged in LDS per batch (32 KB)

struct LseAcc {
  double m, s;  // max and sum of 2^(t - m), log2 units
};

// merge b into a (a then b): the order every path uses
__device__ __forceinline__ void lse_merge(LseAcc &a, const LseAcc &b) {
  if (b.m == -INFINITY && b.s == 0.0) return;
  if (a.m == -INFINITY && a.s == 0.0) { a = b; return; }
  const bool nan = a.m != a.m || b.m != b.m;
  const double M = nan ? NAN : fmax(a.m, b.m);
  a.s = a.s * (double)__builtin_amdgcn_exp2f((float)(a.m - M)) +
        b.s * (double)__builtin_amdgcn_exp2f((float)(b.m - M));
  a.m = M;
}

// the components i = first, first + st, ... < hi of an LDS batch, log-sum-exp:
// a max pass and a sum pass (log2 units)
__device__ __forceinline__ LseAcc lse_strided(const Coef *__restrict__ cs, int first, int hi,
                                              int st, double y) {
  double m = -INFINITY;
  bool nan = y != y;
#pragma unroll 4
  for (int k = first; k < hi; k += st) {
    const double cx = cs[k].x, cy = cs[k].y, cz = cs[k].z;
    const double t = fma(fma(cz, y, cy), y, cx);
    nan |= t != t;
    m = fmax(m, t);
  }
  LseAcc r{m, 0.0};
  if (nan) { r.m = NAN; r.s = NAN; return r; }
  if (m == -INFINITY) return r;  // no terms, or every term -inf
  double s = 0.0;
#pragma unroll 4
  for (int k = first; k < hi; k += st) {
    const double cx = cs[k].x, cy = cs[k].y, cz = cs[k].z;
    const double t = fma(fma(cz, y, cy), y, cx);
    s += (double)__builtin_amdgcn_exp2f((float)(t - m));
  }
  r.s = s;
  return r;
}

// the same components, quantized: sum_k w (Phi(ub) - Phi(lb)),
// tpe.py:146-160 (GMM: 0.5 * (1 + erf)) / 284-299 (LGMM: .5 + .5 * erf)
// CENSUS counts, per lane, the valid pairs, the live ones and the ones
// evaluated (live for some lane of the wave) -- roofline accounting only.
struct Census {
  uint32_t total, live, exec;
};

template <bool LOGN, bool CENSUS>
__device__ __forceinline__ double erf_strided(const Coef *__restrict__ cs, int first, int hi,
                                              int st, double ub, double lb, bool valid,
                                              Census &cen) {
#pragma clang fp contract(off)
  double prob = 0.0;
  for (int k = first; k < hi; k += st) {
    const double cx = cs[k].x, cy = cs[k].y;
    const double zu = (ub - cx) * cy;
    const double zl = (lb - cx) * cy;
    const bool dead = !valid || (zu >= 6.5 && zl >= 6.5) || (zu <= -6.5 && zl <= -6.5);
    const bool skip = __all(dead);
    if constexpr (CENSUS) {
      cen.total += valid ? 1u : 0u;
      cen.live += dead ? 0u : 1u;
      cen.exec += (valid && !skip) ? 1u : 0u;
    }
    if (skip) continue;  // exact zeros for every lane of the wave
    const double w = cs[k].z;
    double cu, cl;
    if (LOGN) {
      cu = .5 + .5 * erf(zu);
      cl = .5 + .5 * erf(zl);
    } else {
      cu = 0.5 * (1.0 + erf(zu));
      cl = 0.5 * (1.0 + erf(zl));
    }
    double inc = w * cu;
    inc -= w * cl;
    prob += inc;
  }
  return prob;
}

struct ScoreSmem {
  Coef stage[kStage];              // 32 KB: one batch of components
  double2 wpart[2][kWaves][64];    // 32 KB: per-wave partials (below, above)
};

template <int KIND, bool CENSUS>
__device__ __forceinline__ void score_tile(const ScoreArgs &A, ScoreSmem &sm) {
  constexpr bool LSE = KIND == KIND_LSE_G || KIND == KIND_LSE_L;
  constexpr bool ERF = KIND == KIND_ERF_G || KIND == KIND_ERF_L;
  constexpr bool CAT = KIND == KIND_CAT;
  constexpr bool LOGN = KIND == KIND_LSE_L || KIND == KIND_ERF_L;
  Coef *stage = sm.stage;
  auto &wpart = sm.wpart;
  const int slot = blockIdx.y, s = blockIdx.z, tile = blockIdx.x;
  const int hp = A.level_hps[slot];
  const tpe_hp H = A.hps[hp];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool act = A.force_active || hp_active(H, A.results + (int64_t)s * A.n_hp,
                                                  A.cond_parent, A.cond_branch);
  if (!act) {  // one record says "inactive"; no tickets are taken
    if (blockIdx.x == 0 && threadIdx.x == 0)
      A.results[(int64_t)s * A.n_hp + hp] = Partial{NAN, NAN, -1, 0, 0};
    return;
  }
  const int64_t sb = 2 * (int64_t)hp, sa = sb + 1;
  const MixInfo ib = A.info[sb], ia = A.info[sa];
  const Coef *__restrict__ cb = A.coef + sb * A.kcap;
  const Coef *__restrict__ ca = A.coef + sa * A.kcap;
  const int64_t coff = (int64_t)s * A.cand_sstride + (int64_t)(A.cand_slot0 + slot) * A.n_cand;
  const double *__restrict__ cand = A.cand + coff;
  // only the quantized kinds' candidates are value-bucketed (k_bucket)
  const int32_t *__restrict__ cpos = (ERF && A.cand_pos) ? A.cand_pos + coff : nullptr;
  const int64_t li = (int64_t)tile * 64 + lane;
  const bool valid = li < A.n_cand;
  const double x = valid ? cand[li] : (LOGN ? 1.0 : 0.0);

  // candidate-side transforms, once per candidate
  double y = 0.0, ub = 0.0, lb = 0.0;
  if constexpr (LSE) {
    y = (LOGN ? log(x) : x) - H.prior_mu;
  } else if constexpr (ERF) {
    const double hq = H.q / 2.0;
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
  }

  double2 res_b = make_double2(0.0, 0.0), res_a = res_b;  // lane's merged results (wave 0)
  if constexpr (!CAT) {
    // components: below [0, Kb) then above [Kb, Kb + Ka), staged in batches
    // of kStage; wave w owns the components of each mixture with index
    // k = w (mod kWaves) -- live erf components spread over the waves
    const int Kb = ib.K, Kt = ib.K + ia.K;
    LseAcc lacc[2] = {{-INFINITY, 0.0}, {-INFINITY, 0.0}};
    double pacc[2] = {0.0, 0.0};
    Census cen{0u, 0u, 0u};
    for (int b0 = 0; b0 < Kt; b0 += kStage) {
      const int nb = min(kStage, Kt - b0);
      __syncthreads();  // the previous batch is consumed
      for (int i = threadIdx.x; i < nb; i += blockDim.x) {
        const int k = b0 + i;
        stage[i] = k < Kb ? cb[k] : ca[k - Kb];
      }
      __syncthreads();
#pragma unroll
      for (int mix = 0; mix < 2; ++mix) {
        // this batch's part of mixture `mix`, in batch-local indices [lo, hi)
        const int lo = max(0, (mix ? Kb : 0) - b0), hi = min(nb, (mix ? Kt : Kb) - b0);
        if (lo >= hi) continue;
        // first owned index >= lo: mixture-relative index = w (mod kWaves)
        const int mbase = (mix ? Kb : 0) - b0;             // batch-local index of mixture k = 0
        int first = lo + ((wave - (lo - mbase)) % kWaves + kWaves) % kWaves;
        if constexpr (LSE) {
          lse_merge(lacc[mix], lse_strided(stage, first, hi, kWaves, y));
        } else {
          pacc[mix] += erf_strided<LOGN, CENSUS>(stage, first, hi, kWaves, ub, lb, valid, cen);
        }
      }
    }
    if constexpr (CENSUS && ERF) {
      unsigned long long c3[3] = {cen.total, cen.live, cen.exec};
#pragma unroll
      for (int q = 0; q < 3; ++q) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c3[q] += __shfl_xor(c3[q], o, 64);
        if (lane == 0) atomicAdd(A.census + q, c3[q]);
      }
    }
    if constexpr (LSE) {
      wpart[0][wave][lane] = make_double2(lacc[0].m, lacc[0].s);
      wpart[1][wave][lane] = make_double2(lacc[1].m, lacc[1].s);
    } else {
      wpart[0][wave][lane] = make_double2(pacc[0], 0.0);
      wpart[1][wave][lane] = make_double2(pacc[1], 0.0);
    }
    __syncthreads();
    // wave 0 merges the below partials, wave 1 the above ones, in wave order
    double2 r = make_double2(0.0, 0.0);
    if (wave < 2) {
      r = wpart[wave][0][lane];
      for (int w = 1; w < kWaves; ++w) {
        const double2 v = wpart[wave][w][lane];
        if constexpr (LSE) {
          LseAcc t{r.x, r.y};
          lse_merge(t, LseAcc{v.x, v.y});
          r = make_double2(t.m, t.s);
        } else {
          r.x += v.x;
        }
      }
      if (wave == 1) wpart[1][1][lane] = r;  // slot already consumed by wave 1
    }
    __syncthreads();
    res_b = r;
    res_a = wpart[1][1][lane];
  }
  if (wave != 0) return;

  // ---- finalize the tile (wave 0): lpdfs, EI, argmax (numpy semantics)
  double best_s = NAN, best_v = NAN;
  int64_t best_i = -1;
  if (valid) {
    double lpb, lpa;
    if constexpr (LSE) {
      const double LN2 = 0.6931471805599453;
      lpb = (res_b.x == -INFINITY) ? NAN : (res_b.x + log2(res_b.y)) * LN2;
      lpa = (res_a.x == -INFINITY) ? NAN : (res_a.x + log2(res_a.y)) * LN2;
      if constexpr (LOGN) { const double lx = log(x); lpb -= lx; lpa -= lx; }
    } else if constexpr (ERF) {
      lpb = log(res_b.x) - ib.log_pacc;
      lpa = log(res_a.x) - ia.log_pacc;
    } else {
      const int64_t c = (int64_t)x;
      const bool in = (x >= 0.0) && (c < ib.K) && ((double)c == x);
      lpb = in ? cb[c].x : NAN;
      lpa = in ? ca[c].x : NAN;
    }
    const int64_t lo = cpos ? (int64_t)cpos[li] : li;  // original position
    if (A.out_lb) A.out_lb[lo] = lpb;
    if (A.out_la) A.out_la[lo] = lpa;
    best_s = lpb - lpa;
    best_v = x;
    best_i = A.cand_begin + lo;
  }
  wave_best(best_s, best_v, best_i);
  Partial *pbase = A.partial + ((int64_t)s * A.n_hp + hp) * A.pstride;
  int is_last = 0;
  if (lane == 0) {
    pbase[tile] = Partial{best_s, best_v, best_i, 1, 0};
    // publish the tile record, then take an arrival ticket (agent release /
    // acquire, cdna_hip_programming.md Guideline 16 counter form)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t *tk = A.ticket + (int64_t)s * A.n_hp + hp;
    const uint32_t t = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = (t == (uint32_t)A.tiles - 1) ? 1 : 0;
    if (is_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  is_last = __shfl(is_last, 0, 64);
  if (!is_last) return;
  double fs = NAN, fv = NAN;
  int64_t fi = -1;
  for (int i = lane; i < A.tiles; i += 64) {
    const Partial q = pbase[i];
    if (better(q.score, q.index, fs, fi)) { fs = q.score; fv = q.value; fi = q.index; }
  }
  wave_best(fs, fv, fi);
  if (lane == 0) {
    Partial *r = A.results + (int64_t)s * A.n_hp + hp;
    if (!(A.accumulate && better(r->score, r->index, fs, fi))) *r = Partial{fs, fv, fi, 1, 0};
  }
}

// One launch scores every hp of a level (grid.y), each block dispatching on its
// hp's lpdf kind, so log-sum-exp, quantized and categorical tiles share the
// GPU without stream forks.  Without quantized hps the kernel is built for
// <= 64 VGPRs (8 waves per SIMD); with them it keeps OCML erf's registers
// (4 waves per SIMD) rather than spilling.
template <bool ERFK, bool CENSUS>
__global__ __launch_bounds__(kWaves * 64, ERFK ? 4 : 8) void k_score(ScoreArgs A) {
  __shared__ ScoreSmem sm;
  const tpe_hp &H = A.hps[A.level_hps[blockIdx.y]];
  switch (score_kind(H)) {
    case KIND_LSE_G: score_tile<KIND_LSE_G, CENSUS>(A, sm); break;
    case KIND_LSE_L: score_tile<KIND_LSE_L, CENSUS>(A, sm); break;
    case KIND_ERF_G: if constexpr (ERFK) score_tile<KIND_ERF_G, CENSUS>(A, sm); break;
    case KIND_ERF_L: if constexpr (ERFK) score_tile<KIND_ERF_L, CENSUS>(A, sm); break;
    default: score_tile<KIND_CAT, CENSUS>(A, sm); break;
  }
}

hipError_t launch_score(const ScoreArgs &a, bool has_erf, hipStream_t st) {
  if (a.n_slots <= 0 || a.n_suggest <= 0 || a.tiles <= 0) return hipSuccess;
  const dim3 g((unsigned)a.tiles, a.n_slots, a.n_suggest);
  if (has_erf) {
    if (a.census) k_score<true, true><<<g, kWaves * 64, 0, st>>>(a);
    else k_score<true, false><<<g, kWaves * 64, 0, st>>>(a);
  } else {
    k_score<false, false><<<g, kWaves * 64, 0, st>>>(a);
  }
  return hipGetLastError();
}

}  // namespace tpe
