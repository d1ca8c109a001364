// tpe_score.hip -- below/above lpdf of every candidate, EI and argmax, gfx950.
//
// Reference (pminervini/hyperopt, hyperopt/tpe.py):
//   GMM1_lpdf   tpe.py:104-166     LGMM1_lpdf  tpe.py:259-301
//   categorical_lpdf tpe.py:50-57  broadcast_best tpe.py:749-759 (EI argmax)
//
// Work decomposition.  A block of kWaves waves owns a tile of 64 * kR
// candidates of one (suggestion, hp); every wave holds the same candidates,
// kR per lane (candidate r * 64 + lane of the tile).  The components of both
// mixtures are cut into chunks of kChunk; wave w takes the chunks w (mod
// kWaves) and reads their coefficients with wave-uniform scalar loads (SGPR
// operands: a (candidate, component) pair costs only VALU work, no LDS or
// VGPR traffic).  Each wave reduces its share (log-sum-exp: single pass with
// an integer exponent; quantized: a linear sum), then 2 * kR waves (one per
// mixture and candidate row) merge the wave partials in wave order.  The
// reduction tree depends on (K_b, K_a) only, so scores are bitwise
// independent of the grid, of candidate chunking and of multi-GPU sharding.
//
// Log-sum-exp (q = None): t = alpha + y'(beta + gamma y') (two fp64 FMAs, see
// make_coef), 2^(t - m) with v_exp_f32 on the fp64 difference, fp32 group
// sums added in fp64.  With value-bucketed candidates (large draws) a block
// of 8 components whose envelope proves all its terms below 2^-(27 + log2 K)
// of every lane's largest term is skipped (lse_window, kLseDeadBase): the
// lpdf moves by at most 2^-26 ~ 1.5e-8 relative.  Quantized: the reference's
// sum_k w (Phi(ub) - Phi(lb)) in fp64 with OCML erf, in its operation order;
// a component whose two erf arguments are beyond 6.5 on one side contributes
// an exact 0 and is skipped when every candidate of the wave agrees.
#include <math.h>

#include <algorithm>
#include <type_traits>

#include "tpe_device.hpp"
#include "tpe_draw.hpp"

namespace tpe {

constexpr int kWaves = 8;       // waves per scoring block (all share the tile)
constexpr int kRMax = 2;        // candidate rows (per lane) of the widest non-categorical tile
constexpr int kChunk = 16;      // components per ownership chunk
static_assert(2 * kRMax <= kWaves, "one merging wave per (mixture, candidate row)");

// A log-sum-exp partial in log2 units: value = m + log2(s).  The exponent m
// is kept integer-valued (or -inf), so every rescale of s to a new exponent is
// an exact power-of-two ldexp; the only rounding is in the terms themselves.
struct LseAcc {
  double m, s;
};

// merge b into a (a then b): the order every path uses
__device__ __forceinline__ void lse_merge(LseAcc &a, const LseAcc &b) {
  if (b.m == -INFINITY && b.s == 0.0) return;
  if (a.m == -INFINITY && a.s == 0.0) { a = b; return; }
  if (a.m != a.m || b.m != b.m) { a = LseAcc{NAN, NAN}; return; }
  const double M = fmax(a.m, b.m);
  a.s = ldexp(a.s, (int)fmax(a.m - M, -2100.0)) + ldexp(b.s, (int)fmax(b.m - M, -2100.0));
  a.m = M;
}

// Coefficients read through the constant address space: the component loops
// below index them with wave-uniform addresses, so they compile to scalar
// loads (s_load into SGPRs, one per wave, no LDS or VGPR traffic per lane).
typedef const double __attribute__((address_space(4))) KDbl;

// global (not flat) words of the in-launch tile hand-off
typedef uint64_t __attribute__((address_space(1))) gu64;
typedef uint32_t __attribute__((address_space(1))) gu32;
__device__ __forceinline__ uint64_t dbits(double x) { return __builtin_bit_cast(uint64_t, x); }
__device__ __forceinline__ double bitsd(uint64_t x) { return __builtin_bit_cast(double, x); }

// a wave-uniform table pointer as a scalar (the compiler cannot always prove it)
__device__ __forceinline__ KDbl *uniform_ptr(const Coef *p) {
  const uint64_t u = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return (KDbl *)(((uint64_t)hi << 32) | lo);
}

// Component ownership: a mixture's components are cut into chunks of kChunk
// consecutive indices and wave w owns the chunks c = w (mod kWaves), scanning
// them in order; `c0` is the wave's first chunk.

constexpr int kGroup = kCoefBlock;  // components per scalar-load group: one table block
static_assert(kChunk % kGroup == 0, "groups tile the chunks");

struct CoefGroup {
  double x[kGroup], y[kGroup], z[kGroup];
};

// three 64-B scalar loads: the x, y, z rows of the table block at k (whole
// blocks are allocated, entries past the mixture are masked by the caller)
__device__ __forceinline__ void load_group(KDbl *__restrict__ cs, int k, CoefGroup &g) {
  KDbl *b = cs + (((unsigned)k >> 3) << 5);  // k >= 0: coef_off(k, 0) of a block start
#pragma unroll
  for (int j = 0; j < kGroup; ++j) {
    g.x[j] = b[j];
    g.y[j] = b[kCoefBlock + j];
    g.z[j] = b[2 * kCoefBlock + j];
  }
}

// prune mode 3: the block-local fp32 form of the same terms (Coef32)
typedef const Coef32 __attribute__((address_space(4))) KC32;
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ KC32 *uniform_ptr32(const Coef32 *p) {
  const uint64_t u = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return (KC32 *)(((uint64_t)hi << 32) | lo);
}
struct CoefGroup32 {
  double m;
  float A;
  float a[kGroup], b[kGroup], c[kGroup];
};
// two 64-B scalar loads: the block of component k
__device__ __forceinline__ void load_group32(KC32 *__restrict__ t, int k, CoefGroup32 &g) {
  KC32 *b = t + ((unsigned)k >> 3);  // k >= 0: block k / kCoefBlock
  static_assert(kCoefBlock == 8, "block shift");
  g.m = b->center;
  g.A = b->base;
#pragma unroll
  for (int j = 0; j < kGroup; ++j) {
    g.a[j] = b->a[j];
    g.b[j] = b->b[j];
    g.c[j] = b->c[j];
  }
}

// the same from a round's first block rb and a block offset j < 64 (wave
// tiles): a 32-bit offset on a per-round base, no 64-bit address arithmetic
// per block
__device__ __forceinline__ void load_block32(KC32 *__restrict__ rb, uint32_t j, CoefGroup32 &g) {
  KC32 *b = rb + j;
  g.m = b->center;
  g.A = b->base;
#pragma unroll
  for (int q = 0; q < kGroup; ++q) {
    g.a[q] = b->a[q];
    g.b[q] = b->b[q];
    g.c[q] = b->c[q];
  }
}
// The moment form of a 16-component chunk (CoefM, tpe_internal.hpp): one
// 64-B scalar load per chunk
typedef const CoefM __attribute__((address_space(4))) KCM;
__device__ __forceinline__ KCM *uniform_ptrm(const CoefM *p) {
  const uint64_t u = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return (KCM *)(((uint64_t)hi << 32) | lo);
}
struct MomGroup {
  double c;
  float A, cm, g;
  float m[kMomDeg + 1];
};
__device__ __forceinline__ void load_mom(KCM *__restrict__ rb, uint32_t j, MomGroup &g) {
  KCM *b = rb + j;
  g.c = b->center;
  g.A = b->base;
  g.cm = b->cm;
  g.g = b->gam;
#pragma unroll
  for (int q = 0; q <= kMomDeg; ++q) g.m[q] = b->m[q];
}
// a chunk's terms for the two candidate rows of a lane, but the exponential:
// v = fp32(y' - centre), arg = -a^2 v^2 + (T* - A) + (A - M) (A - M exact),
// and the degree-kMomDeg polynomial in v by Horner on packed fp32 pairs (the
// coefficients are scalar operands); the chunk's sum is 2^arg * p
__device__ __forceinline__ void mom_terms(const MomGroup &g, float Mf, const double (&y)[2],
                                          f2v &arg, f2v &p) {
  const float off = g.cm + (g.A - Mf);
  const f2v v = {(float)(y[0] - g.c), (float)(y[1] - g.c)};
  arg = __builtin_elementwise_fma(f2v{g.g, g.g}, v * v, f2v{off, off});
  p = __builtin_elementwise_fma(f2v{g.m[kMomDeg], g.m[kMomDeg]}, v,
                                f2v{g.m[kMomDeg - 1], g.m[kMomDeg - 1]});
#pragma unroll
  for (int q = kMomDeg - 2; q >= 0; --q) p = __builtin_elementwise_fma(p, v, f2v{g.m[q], g.m[q]});
}
// one candidate row (one-row wave tiles): two chunks a, b packed instead of
// two rows, the same arithmetic per (candidate, chunk)
__device__ __forceinline__ void mom_terms2(const MomGroup &a, const MomGroup &b, float Mf, double y,
                                           f2v &arg, f2v &p) {
  const f2v off = {a.cm + (a.A - Mf), b.cm + (b.A - Mf)};
  const f2v v = {(float)(y - a.c), (float)(y - b.c)};
  arg = __builtin_elementwise_fma(f2v{a.g, b.g}, v * v, off);
  p = __builtin_elementwise_fma(f2v{a.m[kMomDeg], b.m[kMomDeg]}, v,
                                f2v{a.m[kMomDeg - 1], b.m[kMomDeg - 1]});
#pragma unroll
  for (int q = kMomDeg - 2; q >= 0; --q) p = __builtin_elementwise_fma(p, v, f2v{a.m[q], b.m[q]});
}
__device__ __forceinline__ void mom_sum(const f2v &arg, const f2v &p, float (&bs)[2]) {
  bs[0] = __builtin_amdgcn_exp2f(arg.x) * p.x;
  bs[1] = __builtin_amdgcn_exp2f(arg.y) * p.y;
}
// The 8-wide moment form (CoefM8, one coefficient block, degree kMom8Deg):
// the same arithmetic with 16 coefficients; one entry = two 64-B scalar loads
typedef const CoefM8 __attribute__((address_space(4))) KCM8;
__device__ __forceinline__ KCM8 *uniform_ptrm8(const CoefM8 *p) {
  const uint64_t u = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return (KCM8 *)(((uint64_t)hi << 32) | lo);
}
struct Mom8Group {
  double c;
  float A, cm, g;
  float m[kMom8Deg + 1];
};
__device__ __forceinline__ void load_mom8(KCM8 *__restrict__ rb, uint32_t j, Mom8Group &g) {
  KCM8 *b = rb + j;
  g.c = b->center;
  g.A = b->base;
  g.cm = b->cm;
  g.g = b->gam;
#pragma unroll
  for (int q = 0; q <= kMom8Deg; ++q) g.m[q] = b->m[q];
}
// two candidate rows of a lane against one block
__device__ __forceinline__ void mom8_terms(const Mom8Group &g, float Mf, const double (&y)[2],
                                           f2v &arg, f2v &p) {
  const float off = g.cm + (g.A - Mf);
  const f2v v = {(float)(y[0] - g.c), (float)(y[1] - g.c)};
  arg = __builtin_elementwise_fma(f2v{g.g, g.g}, v * v, f2v{off, off});
  p = __builtin_elementwise_fma(f2v{g.m[kMom8Deg], g.m[kMom8Deg]}, v,
                                f2v{g.m[kMom8Deg - 1], g.m[kMom8Deg - 1]});
#pragma unroll
  for (int q = kMom8Deg - 2; q >= 0; --q) p = __builtin_elementwise_fma(p, v, f2v{g.m[q], g.m[q]});
}
// one candidate row against two blocks a, b packed
__device__ __forceinline__ void mom8_terms2(const Mom8Group &a, const Mom8Group &b, float Mf,
                                            double y, f2v &arg, f2v &p) {
  const f2v off = {a.cm + (a.A - Mf), b.cm + (b.A - Mf)};
  const f2v v = {(float)(y - a.c), (float)(y - b.c)};
  arg = __builtin_elementwise_fma(f2v{a.g, b.g}, v * v, off);
  p = __builtin_elementwise_fma(f2v{a.m[kMom8Deg], b.m[kMom8Deg]}, v,
                                f2v{a.m[kMom8Deg - 1], b.m[kMom8Deg - 1]});
#pragma unroll
  for (int q = kMom8Deg - 2; q >= 0; --q) p = __builtin_elementwise_fma(p, v, f2v{a.m[q], b.m[q]});
}

// Tables staged in LDS (the one-row wave-tile kernel, k_score_wave1): a
// mixture's block envelopes and block-local fp32 blocks copied once per
// workgroup, so the component loops of its 8 waves read them at LDS latency
// instead of waiting on one scalar-load batch per block (the small launches
// that kernel serves are latency-bound, not VALU-bound).  The values are the
// global tables' bit for bit: staging changes no result.
#ifdef TPE_STAMPS
// diagnostic build only (tools/score_stamps.py): per wave of suggestion 0's
// wave tiles, [0] component blocks evaluated by the one-exponent loops, [1]
// their attempts, [2] fallbacks to the exact loop, [3] blocks the exact loop
// evaluated
__device__ unsigned g_wave_info[8192][8][4];
#define WINFO(i, v)                                                                      \
  do {                                                                                   \
    if ((threadIdx.x & 63) == 0 && blockIdx.y == 0 && blockIdx.x < 8192)                 \
      g_wave_info[blockIdx.x][threadIdx.x >> 6][i] += (unsigned)(v);                     \
  } while (0)
// per wave (wave tiles), lane 0 of every wave of the blocks of suggestion 0:
// [0] start of the component loops, [1] their end, [2] after the candidate
// loads, [3] after the below mixture, [4] after the above mixture's window,
// [5] after pass 1 of the one-exponent loop, [6] after its tightening, [7]
// after pass 2 (the guard passed), [8] after the finalize's wave argmax
constexpr int kWaveStamps = 10;
__device__ unsigned long long g_wave_stamps[8192][8][kWaveStamps];
#define WSTAMP(i)                                                                        \
  do {                                                                                   \
    if ((threadIdx.x & 63) == 0 && blockIdx.y == 0 && blockIdx.x < 8192)                 \
      g_wave_stamps[blockIdx.x][threadIdx.x >> 6][i] = wall_clock64();                   \
  } while (0)
#else
#define WINFO(i, v) do {} while (0)
#define WSTAMP(i) do {} while (0)
#endif
typedef const float4 __attribute__((address_space(3))) LF4;
typedef const Coef32 __attribute__((address_space(3))) LC32;
struct Stage {
  LF4 *env;    // [blocks] envelopes (the Coef w-rows' first 16 B)
  LC32 *c32;   // [blocks] block-local fp32 blocks
  const float4 *genv;  // the slot's compact envelope table (CoefEnv, global; null: w-rows)
  int tight = 1;       // tighten the threshold from the top block (ScoreArgs::lse_tight)
};
constexpr int kStageBlocks = 224;  // blocks of both mixtures a workgroup stages (32 KB)
struct StageSmem {
  float4 env[kStageBlocks];
  Coef32 c32[kStageBlocks];
};
__device__ __forceinline__ void load_block32_lds(LC32 *__restrict__ rb, uint32_t j, CoefGroup32 &g) {
  LC32 *b = rb + j;
  g.m = b->center;
  g.A = b->base;
#pragma unroll
  for (int q = 0; q < kGroup; ++q) {
    g.a[q] = b->a[q];
    g.b[q] = b->b[q];
    g.c[q] = b->c[q];
  }
}
// the envelope of the block starting at component k0 (global table or stage)
// (unstaged: the compact envelope table when given -- a round's 64 envelopes
// are 1 KB contiguous, 8 cache lines, against 64 lines of the Coef w-rows at
// a 256-B stride)
template <bool STG>
__device__ __forceinline__ float4 block_env(const double *tb, const Stage &st, int k0) {
  if constexpr (STG) {
    const float __attribute__((address_space(3))) *e =
        (const float __attribute__((address_space(3))) *)(st.env + (k0 >> 3));
    return make_float4(e[0], e[1], e[2], e[3]);
  }
  else if (st.genv) return st.genv[k0 >> 3];
  else return *reinterpret_cast<const float4 *>(tb + coef_off(k0, 3));
}

// the lowest set bit of m, or 0 when m is empty (the caller then reloads
// block 0 of the round: a valid address, its values unused)
__device__ __forceinline__ uint32_t low_bit(uint64_t m) {
  return (uint32_t)max(__ffsll((long long)m) - 1, 0);
}

// Single-pass log-sum-exp over the wave's chunks of a mixture of nb
// components against the lane's KR candidates (log2 units, t = alpha +
// y'(beta + gamma y'), make_coef).  Per group of kGroup components: the group
// max lifts the integer exponent m to ceil(max) if larger (exact ldexp rescale
// of s), then s += 2^(t - m) with v_exp_f32 on the fp64 difference (every
// term <= 1, the largest > 1/2).  A NaN term makes its 2^(t - m) NaN, which
// reaches the lpdf as the reference's NaN (logsum_rows, tpe.py:37-40); fmax
// drops it from the exponent, so a lane whose terms are all NaN keeps
// m = -inf and scores NaN as well.
template <int KR>
__device__ __forceinline__ void lse_terms(const CoefGroup &g, const double (&y)[KR],
                                          const double (&y2)[KR], double (&t)[KR][kGroup]) {
#pragma unroll
  for (int r = 0; r < KR; ++r)
#pragma unroll
    for (int j = 0; j < kGroup; ++j)
      // alpha + beta y' + gamma y'^2, one scalar coefficient per FMA
      t[r][j] = fma(g.z[j], y2[r], fma(g.y[j], y[r], g.x[j]));
}
template <int KR>
__device__ __forceinline__ void lse_fold(const double (&t)[KR][kGroup], double (&m)[KR],
                                         double (&s)[KR]) {
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    // group max as a tree (fmax drops NaN terms)
    double mx[kGroup];
#pragma unroll
    for (int j = 0; j < kGroup; ++j) mx[j] = t[r][j];
#pragma unroll
    for (int w = kGroup / 2; w > 0; w >>= 1)
#pragma unroll
      for (int j = 0; j < w; ++j) mx[j] = fmax(mx[j], mx[j + w]);
    // lift the integer exponent; s == 0 while m == -inf, and the clamp turns
    // the -inf / NaN differences of that state into a harmless ldexp of 0
    const double mn = fmax(m[r], ceil(mx[0]));
    s[r] = ldexp(s[r], (int)fmax(m[r] - mn, -2100.0));
    m[r] = mn;
    const double ms = mn == -INFINITY ? 0.0 : mn;  // all terms -inf / NaN so far
    // terms 2^(t - m) <= 1 summed as an fp32 tree (<= kGroup), then in fp64
    float e[kGroup];
#pragma unroll
    for (int j = 0; j < kGroup; ++j) e[j] = __builtin_amdgcn_exp2f((float)(t[r][j] - ms));
#pragma unroll
    for (int w = kGroup / 2; w > 0; w >>= 1)
#pragma unroll
      for (int j = 0; j < w; ++j) e[j] += e[j + w];
    s[r] += (double)e[0];
  }
}

// Envelope rounds: the wave's chunks c = c0 (mod STRIDE) in increasing order,
// 32 chunks (64 blocks of kGroup components) per round, lane l testing block
// l of the round -- block (l & 1) of chunk r0 + STRIDE (l >> 1) -- so one
// ballot lists the round's live blocks in evaluation order (chunk j's block 0
// before its block 1 before chunk j + 1) and the next one is one bit scan.
template <int STRIDE>
__device__ __forceinline__ int round_k(int r0, int j) {
  return ((r0 + STRIDE * (j >> 1)) * 2 + (j & 1)) * kGroup;
}
// the next live block of a round: its first component, popped from the mask
template <int STRIDE>
__device__ __forceinline__ bool next_live(uint64_t &m, int r0, int &kg) {
  if (!m) return false;
  const int j = __builtin_ctzll(m);
  m &= m - 1;
  kg = round_k<STRIDE>(r0, j);
  return true;
}

// The wave's pruning window for one mixture (lse_chunks' PRUNE mode): the
// candidate range [lo, hi] (y' units) and the threshold below which a block's
// bound proves every term an fp32 zero.
struct LseWindow {
  float lo, hi, thr;
};

// Census of the log-sum-exp work (roofline accounting only): valid pairs and
// the ones in evaluated (not skipped) blocks.
struct LseCensus {
  uint32_t total, exec, shift;  // shift: the evaluated ones in the one-exponent form
  uint32_t f32;                 // the evaluated ones in the fp32 per-group-lift form
  uint32_t retry;               // one-exponent pairs evaluated again by a second attempt
  uint32_t wide;                // one-exponent pairs of wide blocks (fp64 loop, mode 3)
  uint32_t mom;                 // one-exponent pairs evaluated in the moment form (CoefM / CoefM8)
  uint32_t mom8;                // of those, in the 8-wide form (CoefM8)
  uint32_t momh;                // of those, in the 16-wide degree-15 form (CoefMH)
};

// A block's envelope bound over the wave's candidate range [lo, hi]: the
// largest term any of its components can reach there (log2 units).
__device__ __forceinline__ float envelope_bound(const float4 e, const LseWindow &win) {
  const float d = fmaxf(0.0f, fmaxf(e.x - win.hi, win.lo - e.y));
  return fmaf(-fabsf(e.w), d * d, e.z);  // (the sign of e.w flags a wide block, Coef32)
}

// The wave's chunks c = c0 (mod STRIDE) of a mixture of nb components, in
// increasing order, one envelope round (round_k: 64 blocks) at a time: lane l
// tests block l of the round against the window (one vector load of its
// envelope, tpe_internal.hpp kLseDeadBase), a ballot gives the round's live
// blocks, and only those are evaluated, in the same order as the full loop.
// prune = false: every block is live.
// The same fold from the block-local fp32 form (prune mode 3, Coef32, blocks
// that are not wide): z = t - A by two packed fp32 FMAs per component pair
// (lse_terms_z, before the next block's coefficients are loaded), then the
// group max in fp32, the integer lift m = max(m, A + ceil(max z)) in fp64 as
// before, and 2^(z + (A - m)) with A - m an exact integer (lse_fold_z).
template <int KR>
__device__ __forceinline__ void lse_terms_z(const CoefGroup32 &g, const double (&y)[KR],
                                            float (&z)[KR][kGroup]) {
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    const float u = (float)(y[r] - g.m);
    const f2v u2 = {u, u};
#pragma unroll
    for (int j = 0; j < kGroup; j += 2) {
      const f2v a2 = {g.a[j], g.a[j + 1]}, b2 = {g.b[j], g.b[j + 1]}, c2 = {g.c[j], g.c[j + 1]};
      const f2v t = __builtin_elementwise_fma(__builtin_elementwise_fma(c2, u2, b2), u2, a2);
      z[r][j] = t.x;
      z[r][j + 1] = t.y;
    }
  }
}
template <int KR>
__device__ __forceinline__ void lse_fold_z(const float (&z)[KR][kGroup], float A, double (&m)[KR],
                                           double (&s)[KR]) {
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    float mx[kGroup];
#pragma unroll
    for (int j = 0; j < kGroup; ++j) mx[j] = z[r][j];
#pragma unroll
    for (int w = kGroup / 2; w > 0; w >>= 1)
#pragma unroll
      for (int j = 0; j < w; ++j) mx[j] = fmaxf(mx[j], mx[j + w]);
    const double mn = fmax(m[r], (double)A + (double)ceilf(mx[0]));
    s[r] = ldexp(s[r], (int)fmax(m[r] - mn, -2100.0));
    m[r] = mn;
    const double ms = mn == -INFINITY ? 0.0 : mn;
    const float off = (float)((double)A - ms);
    const f2v o2 = {off, off};
    float e[kGroup];
#pragma unroll
    for (int j = 0; j < kGroup; j += 2) {
      const f2v zz = f2v{z[r][j], z[r][j + 1]} + o2;
      e[j] = __builtin_amdgcn_exp2f(zz.x);
      e[j + 1] = __builtin_amdgcn_exp2f(zz.y);
    }
    const float t0 = (e[0] + e[2]) + (e[1] + e[3]);
    const float t1 = (e[4] + e[6]) + (e[5] + e[7]);
    s[r] += (double)(t0 + t1);
  }
}

// F32 (prune mode 3): blocks that are not wide take lse_terms_z / lse_fold_z in the
// pipelined loop, wide ones (the sign of their envelope's a^2) the fp64 fold
// in a second loop after each round.
template <int KR, bool CENSUS, int STRIDE = kWaves, bool F32 = false, bool STG = false>
__device__ __forceinline__ void lse_chunks(KDbl *__restrict__ cs, const Coef *__restrict__ cv,
                                           int c0, int nb, const double (&y)[KR],
                                           LseAcc (&out)[KR], bool prune, LseWindow win,
                                           int nvalid, LseCensus &cen,
                                           KC32 *__restrict__ c32 = nullptr, Stage stg = {}) {
  const int lane = threadIdx.x & 63;
  double m[KR], s[KR], y2[KR];
#pragma unroll
  for (int r = 0; r < KR; ++r) { m[r] = -INFINITY; s[r] = 0.0; y2[r] = y[r] * y[r]; }
  const int nch = (nb + kChunk - 1) / kChunk;
  for (int r0 = c0; r0 < nch; r0 += STRIDE * 32) {
    const int k0 = round_k<STRIDE>(r0, lane);
    const bool has = r0 + STRIDE * (lane >> 1) < nch && k0 < nb;
    bool live = has, wide = false;
    if ((prune || F32) && has) {
      const double *t = reinterpret_cast<const double *>(cv);
      const float4 e = block_env<STG>(t, stg, k0);
      if (prune) live = envelope_bound(e, win) >= win.thr;
      wide = __builtin_signbit(e.w);
    }
    if constexpr (CENSUS) {
      const int n = has ? min(kGroup, nb - k0) : 0;
      uint32_t tot = (uint32_t)n, ex = (uint32_t)(live ? n : 0);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        tot += __shfl_xor(tot, o, 64);
        ex += __shfl_xor(ex, o, 64);
      }
      cen.total += tot * (uint32_t)nvalid;
      cen.exec += ex * (uint32_t)nvalid;
      if constexpr (F32) {
        uint32_t fx = (uint32_t)(live && !wide ? n : 0);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) fx += __shfl_xor(fx, o, 64);
        cen.f32 += fx * (uint32_t)nvalid;
      }
    }
    uint64_t mk = __ballot(live && !(F32 && wide));
    if (STRIDE == 1) WINFO(3, __builtin_popcountll(__ballot(live)));
    // live blocks in order (the padding components of a last block have
    // alpha = -inf, make_coef_pad, so no tail masking is needed);
    // software-pipelined: the next live block's coefficients are loaded into
    // the same scalar registers once this block's terms are formed, so the
    // load overlaps the block's max / exp / sum (scalar loads complete out of
    // order, so only one batch may be in flight)
    int kg = 0;
    bool have = next_live<STRIDE>(mk, r0, kg);
    if constexpr (F32) {
      CoefGroup32 g32;
      if (have) {
        if constexpr (STG) load_block32_lds(stg.c32, (unsigned)kg >> 3, g32);
        else load_group32(c32, kg, g32);
      }
      while (have) {
        float z[KR][kGroup];
        lse_terms_z<KR>(g32, y, z);
        const float A = g32.A;
        have = next_live<STRIDE>(mk, r0, kg);
        if constexpr (STG) load_block32_lds(stg.c32, (unsigned)kg >> 3, g32);
        else load_group32(c32, kg, g32);
        __builtin_amdgcn_sched_barrier(0);
        lse_fold_z<KR>(z, A, m, s);
      }
      uint64_t xk = __ballot(live && wide);
      while (next_live<STRIDE>(xk, r0, kg)) {
        CoefGroup g;
        load_group(cs, kg, g);
        double t[KR][kGroup];
        lse_terms<KR>(g, y, y2, t);
        lse_fold<KR>(t, m, s);
      }
    } else {
      CoefGroup cgp;
      if (have) load_group(cs, kg, cgp);
      while (have) {
        double t[KR][kGroup];
        lse_terms<KR>(cgp, y, y2, t);
        have = next_live<STRIDE>(mk, r0, kg);  // (kg kept after the last)
        load_group(cs, kg, cgp);  // unconditional: no branch merge of the registers
        __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the fold
        lse_fold<KR>(t, m, s);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    if (y[r] != y[r]) out[r] = LseAcc{NAN, NAN};
    else if (m[r] == -INFINITY) out[r] = s[r] == 0.0 ? LseAcc{-INFINITY, 0.0} : LseAcc{NAN, NAN};
    else out[r] = LseAcc{m[r], s[r]};
  }
}

// Shifted log-sum-exp over the live blocks (value-bucketed tiles): one
// exponent M for the whole wave instead of a per-group max and lift.  M =
// ceil(largest live block bound over the wave's range) + 1 is an upper bound
// of every term of every lane, so t - M <= 0 and alpha - M is folded into
// the coefficients once per component (shared by the lane's candidates): a
// pair costs 2 fp64 FMA + cvt + v_exp_f32 + an fp32 add.  Accuracy guard: the
// fp32 rounding of t - M costs |t - M| * 2^-24 relative per term, so every
// valid lane's sum must be >= 2^-4 (its dominant terms within ~4 of M, error
// <= 3e-7); otherwise (a spread-out tile) the wave returns false and the
// exact per-group-lift loop runs instead.
// t - M = (alpha - M) + beta y' + gamma y'^2 as fma(gamma, y'^2, fma(beta, y',
// alpha - M)): each FMA reads one scalar (SGPR) coefficient, so no VALU move
// of a second one is needed (one scalar operand per VALU instruction).
template <int KR>
__device__ __forceinline__ void lse_terms_shifted(const CoefGroup &g, double M,
                                                  const double (&y)[KR], const double (&y2)[KR],
                                                  float (&d)[KR][kGroup]) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    double am[kGroup / 2];
#pragma unroll
    for (int j = 0; j < kGroup / 2; ++j) am[j] = g.x[4 * h + j] - M;
#pragma unroll
    for (int r = 0; r < KR; ++r)
#pragma unroll
      for (int j = 0; j < kGroup / 2; ++j)
        d[r][4 * h + j] = (float)fma(g.z[4 * h + j], y2[r], fma(g.y[4 * h + j], y[r], am[j]));
  }
}
// a lane's group sum is (h0 tree) + (h1 tree) over the halves of 4 components
template <int KR>
__device__ __forceinline__ void lse_fold_shifted(const float (&d)[KR][kGroup], double (&s)[KR]) {
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    float e[kGroup];
#pragma unroll
    for (int j = 0; j < kGroup; ++j) e[j] = __builtin_amdgcn_exp2f(d[r][j]);
    const float t0 = (e[0] + e[2]) + (e[1] + e[3]);
    const float t1 = (e[4] + e[6]) + (e[5] + e[7]);
    s[r] += (double)(t0 + t1);
  }
}
// the same block's terms summed in fp32 only (bs), for a caller that adds two
// blocks' sums in fp32 before the fp64 accumulation
template <int KR>
__device__ __forceinline__ void lse_block_sum(const float (&d)[KR][kGroup], float (&bs)[KR]) {
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    float e[kGroup];
#pragma unroll
    for (int j = 0; j < kGroup; ++j) e[j] = __builtin_amdgcn_exp2f(d[r][j]);
    const float t0 = (e[0] + e[2]) + (e[1] + e[3]);
    const float t1 = (e[4] + e[6]) + (e[5] + e[7]);
    bs[r] = t0 + t1;
  }
}

// Mode 3: t - M of the block in fp32, u = fp32(y' - center) once per
// (candidate, block), then t - M = fma(fma(gamma, u, beta), u, (A - M) +
// alpha) on packed fp32 pairs of components (v_pk_fma_f32): the fp64 FMAs
// and the cvt of every pair become half a packed FMA each.  A - M is an
// exact integer difference and alpha, beta u, gamma u^2 are O(1) for the
// terms that matter, so the rounding stays at the level of the fp32 t - M
// the fp64 form feeds v_exp_f32 (tools/fp32_pair_error.py: max 2.4e-8
// relative lpdf error at config 4 against 1.2e-8 for the fp64 form).
template <int KR>
__device__ __forceinline__ void lse_terms_f32(const CoefGroup32 &g, float Mf,
                                              const double (&y)[KR], float (&d)[KR][kGroup]) {
  // t - M = gamma u^2 + (beta u + (alpha + (A - M))): each packed FMA reads
  // one scalar (SGPR) coefficient pair -- alpha + (A - M) is formed once per
  // block in VGPRs and shared by the rows, u^2 once per row -- so no VALU
  // move of a second coefficient pair is needed (one scalar operand per VOP3P)
  const float am = g.A - Mf;
  const f2v am2 = {am, am};
  f2v a2m[kGroup / 2];
#pragma unroll
  for (int j = 0; j < kGroup; j += 2) a2m[j / 2] = f2v{g.a[j], g.a[j + 1]} + am2;
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    const float u = (float)(y[r] - g.m);
    const f2v u2 = {u, u};
    const f2v uu2 = u2 * u2;
#pragma unroll
    for (int j = 0; j < kGroup; j += 2) {
      const f2v b2 = {g.b[j], g.b[j + 1]}, c2 = {g.c[j], g.c[j + 1]};
      const f2v t = __builtin_elementwise_fma(c2, uu2, __builtin_elementwise_fma(b2, u2, a2m[j / 2]));
      d[r][j] = t.x;
      d[r][j + 1] = t.y;
    }
  }
}

// MW: the moment width of the launch (16: CoefM chunks in cmv, 8: CoefM8
// blocks in cmv8; the kernels are instantiated per width, tpe_internal.hpp)
template <int KR, bool CENSUS, int STRIDE = kWaves, bool F32 = false, bool STG = false, int MW = 16>
__device__ __forceinline__ bool lse_chunks_shifted(KDbl *__restrict__ cs,
                                                   const Coef *__restrict__ cv, int c0, int nb,
                                                   const double (&y)[KR], const bool (&valid)[KR],
                                                   LseAcc (&out)[KR], LseWindow win, int nvalid,
                                                   LseCensus &cen, KC32 *__restrict__ c32 = nullptr,
                                                   const CoefM *__restrict__ cmv = nullptr,
                                                   const CoefM8 *__restrict__ cmv8 = nullptr,
                                                   Stage stg = {}, float env_cmax = 0.0f,
                                                   float env_amin = 0.0f, int probe = -1,
                                                   const CoefM8 *__restrict__ cmvh = nullptr) {
  const int lane = threadIdx.x & 63;
  const int nch = (nb + kChunk - 1) / kChunk;
  const double *tb = reinterpret_cast<const double *>(cv);
  // Live-range search (wave tiles, tables with envelope extremes, MixInfo):
  // every block but the probe's whose envelope bound reaches thr lies within
  // H = sqrt((cmax - thr) / amin) of the window [lo, hi] (its bound is at
  // most cmax - amin d^2).  The blocks' mu' ranges are sorted, so one coarse
  // round -- lane l tests block l S, S = ceil(blocks / 64) -- brackets the
  // blocks whose range meets [lo - H, hi + H]: passes 1 and 2 take only the
  // rounds covering them, and the probe's block (the prior, sigma =
  // prior_sigma: live for every wave, in the middle of the table) is tested
  // and summed on its own when it lies outside them.  (Config 4: pass 1 over
  // ~4 rounds instead of 20, pass 2 no longer spans the rounds between the
  // window and the prior.)
  int rbeg = c0, rend = nch;  // pass-1 rounds [rbeg, rend) (chunk indices)
  int pbk = -1;               // the probe's block, when outside those rounds
  if constexpr (STRIDE == 1) {
    if (env_amin > 0.0f && win.thr > -INFINITY && env_cmax < INFINITY) {
      const float h2 = fmaxf(0.0f, (env_cmax - win.thr) / env_amin);
      const float H = __builtin_sqrtf(h2) * 1.0001f + 1.0e-6f;  // (rounded outward)
      const float L = win.lo - H, R = win.hi + H;
      const int nblk = (nb + kGroup - 1) / kGroup, S = (nblk + 63) / 64;
      const int bq = lane * S;
      bool f = false, g = false;
      if (bq < nblk) {
        const float4 e = block_env<STG>(tb, stg, bq * kGroup);
        f = e.y >= L;  // (monotone in the block: a suffix of the lanes)
        g = e.x <= R;  //                           (a prefix)
      }
      const uint64_t mf = __ballot(f), mg = __ballot(g);
      // first block that can meet [L, R]: after the last tested block left of
      // L (the blocks past the last tested one are untested: a lane beyond
      // it stands for them); last: before the first tested block right of R
      // (none when block 0 already is)
      const int lastlane = (nblk - 1) / S;
      const int j1 = mf ? __builtin_ctzll(mf) : lastlane + 1;
      const int bfirst = j1 == 0 ? 0 : (j1 - 1) * S + 1;
      const int blast = mg ? min(nblk - 1, (64 - __builtin_clzll(mg)) * S - 1) : -1;
      if (bfirst > blast) {
        rbeg = rend = 0;
      } else {
        rbeg = (bfirst >> 1) & ~31;
        rend = min(nch, ((blast >> 1) & ~31) + 32);
      }
      const int pb = probe >= 0 ? probe / kGroup : -1;
      if (pb >= 0 && ((pb >> 1) < rbeg || (pb >> 1) >= rend)) pbk = pb;
    }
  }
  // pass 1: the largest live block bound of the wave's chunks, and the block
  // (and the first and last round with a live block: pass 2, whose
  // threshold is only ever tightened, has no live block outside them)
  float bmax = -INFINITY;
  int barg = -1, rf = -1, rl = -1;
  bool probe_live = false;
  if (pbk >= 0) {  // (every lane: a wave-uniform test)
    const float b = envelope_bound(block_env<STG>(tb, stg, pbk * kGroup), win);
    probe_live = b >= win.thr;
    if (probe_live && lane == 0) { bmax = b; barg = pbk * kGroup; }
  }
  for (int r0 = rbeg; r0 < rend; r0 += STRIDE * 32) {
    const int k0 = round_k<STRIDE>(r0, lane);
    bool lv = false;
    if (r0 + STRIDE * (lane >> 1) < nch && k0 < nb) {
      const float b = envelope_bound(block_env<STG>(tb, stg, k0), win);
      lv = b >= win.thr;
      if (lv && b > bmax) { bmax = b; barg = k0; }
    }
    if (__ballot(lv)) {
      rf = rf < 0 ? r0 : rf;
      rl = r0;
    }
  }
  float wmax = bmax;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wmax = fmaxf(wmax, __shfl_xor(wmax, o, 64));
  if (STRIDE == 1) WSTAMP(5);
  if (!(wmax > -INFINITY && wmax < INFINITY)) return false;  // non-finite envelope
  {
    // a tighter skip threshold: every lane's largest term is at least its
    // largest term in the block of the highest bound (exact t, log2 units),
    // usually several units above the probe's (the wide prior) that
    // lse_window started from; the skip bound then holds as before
    const uint64_t at = __ballot(bmax == wmax && barg >= 0);
    const int kb = __shfl(barg, at ? __builtin_ctzll(at) : 0, 64);
    if (kb >= 0 && stg.tight) {
      const int kbu = __builtin_amdgcn_readfirstlane(kb);
      double lo = INFINITY;
      bool done = false;
      if constexpr (F32) {
        // a block that is not wide: its block-local fp32 form, t = A + z
        // (the maximum term is within ~1 of A, fp32 rounding ~1e-6 on it; a
        // margin of 1/64 keeps the bound a lower bound)
        const float4 e = block_env<STG>(tb, stg, kbu);
        if (!__builtin_signbit(e.w)) {
          CoefGroup32 g32;
          if constexpr (STG) load_block32_lds(stg.c32, (unsigned)kbu >> 3, g32);
          else load_group32(c32, kbu, g32);
          float lo32 = INFINITY;
#pragma unroll
          for (int r = 0; r < KR; ++r) {
            if (!valid[r]) continue;
            float z[1][kGroup];
            const double yr[1] = {y[r]};
            lse_terms_z<1>(g32, yr, z);
            float mx = z[0][0];
#pragma unroll
            for (int j = 1; j < kGroup; ++j) mx = fmaxf(mx, z[0][j]);
            lo32 = fminf(lo32, mx);
          }
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) lo32 = fminf(lo32, __shfl_xor(lo32, o, 64));
          lo = (double)g32.A + (double)lo32 - 0.015625;
          done = true;
        }
      }
      if (!done) {
        CoefGroup g;
        load_group(cs, kbu, g);
#pragma unroll
        for (int r = 0; r < KR; ++r) {
          if (!valid[r]) continue;
          double mx = -INFINITY;
#pragma unroll
          for (int j = 0; j < kGroup; ++j)
            mx = fmax(mx, fma(g.z[j], y[r] * y[r], fma(g.y[j], y[r], g.x[j])));
          lo = fmin(lo, mx);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) lo = fmin(lo, __shfl_xor(lo, o, 64));
      }
      const float dead = kLseDeadBase + (float)(32 - __builtin_clz((unsigned)max(nb - 1, 1)));
      const float t2 = (float)(lo - (double)dead) - 1.0f;
      if (lo > -1.0e30 && lo < 1.0e30 && t2 > win.thr)
        win.thr = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, t2)));
    }
  }
  bmax = wmax;
  if (STRIDE == 1) WSTAMP(6);
  // pass 2 with M = ceil(bmax) + 1 for every lane; a lane whose sum comes
  // out below 2^-4 re-centres on its own sum (M + ceil(log2 s) + 1, the sum
  // then in (1/4, 1/2]) and the wave runs once more; failing that (or a sum
  // that underflowed), the exact loop
  double M = __builtin_amdgcn_readfirstlane((int)ceil((double)bmax)) + 1.0;
  double s[KR], y2[KR];
#pragma unroll
  for (int r = 0; r < KR; ++r) y2[r] = y[r] * y[r];
  for (int attempt = 0;; ++attempt) {
    WINFO(1, 1);
#pragma unroll
    for (int r = 0; r < KR; ++r) s[r] = 0.0;
    // the rounds pass 1 found live (every round in census builds, whose
    // totals count the skipped blocks too; none when only the probe's block
    // is live)
    const int rb = CENSUS ? c0 : (rf < 0 ? 0 : rf), re = CENSUS ? nch : rl + 1;
    for (int r0 = rb; r0 < re; r0 += STRIDE * 32) {
      const int k0 = round_k<STRIDE>(r0, lane);
      const bool has = r0 + STRIDE * (lane >> 1) < nch && k0 < nb;
      bool live = false, wide = false;
      float bnd = -INFINITY;  // the block's envelope bound over the window
      if (has) {
        const float4 e = block_env<STG>(tb, stg, k0);
        bnd = envelope_bound(e, win);
        live = bnd >= win.thr;
        wide = __builtin_signbit(e.w);
      }
      if constexpr (CENSUS) {
        const int n = has ? min(kGroup, nb - k0) : 0;
        uint32_t tot = (uint32_t)n, ex = (uint32_t)(live ? n : 0);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          tot += __shfl_xor(tot, o, 64);
          ex += __shfl_xor(ex, o, 64);
        }
        if (attempt == 0) cen.total += tot * (uint32_t)nvalid;
        cen.exec += ex * (uint32_t)nvalid;
        cen.shift += ex * (uint32_t)nvalid;
        if (attempt > 0) cen.retry += ex * (uint32_t)nvalid;
        if constexpr (F32) {
          uint32_t wx = (uint32_t)(live && wide ? n : 0);
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) wx += __shfl_xor(wx, o, 64);
          cen.wide += wx * (uint32_t)nvalid;
        }
      }
      // (mode 3: the live wide blocks -- kF32Spread, flagged by the sign of
      // their envelope's a^2 -- go to a second, fp64 loop after the round)
      uint64_t mk = __ballot(live && !(F32 && wide));
      WINFO(0, __builtin_popcountll(__ballot(live)));
      // software-pipelined as in lse_chunks
      int kg = 0;
      bool have = next_live<STRIDE>(mk, r0, kg);
      if constexpr (F32 && STRIDE == 1) {
        // wave tiles: block 2 r0 + j of the round for each live bit j, in
        // order; one bit scan and a 32-bit offset per block (SALU)
        const float Mf = (float)M;  // an integer (< 2^24 in magnitude): exact
        KC32 *rb = c32 + 2 * r0;
        LC32 *rbl = STG ? stg.c32 + 2 * r0 : nullptr;
        // chunks in the moment form (CoefM): lane 2i tests chunk r0 + i -- its
        // sigmas equal and x = |v| xh <= kMomXLim over the wave's whole
        // candidate range -- and the chunk is taken when either of its two
        // blocks is live; its blocks then leave the pair and wide loops
        // (the moment form packs the lane's two candidate rows, or two chunks
        // of its one row in one-row tiles)
        constexpr uint64_t kEven = 0x5555555555555555ull;
        // Eligibility: the truncation bound tau(x) = x^(D+1) / (D+1)! e^x (D =
        // kMomDeg) relative to the chunk's terms, which are at most 2^bound
        // (the larger of its two blocks' envelope bounds) against the lane's
        // largest term >= 2^L, L = thr + dead + 1 (lse_window): taken when x
        // <= kMomXLim (tau <= 7.1e-9 whatever the chunk weighs) or when
        // log2 tau + bound <= thr + 1, i.e. tau 2^(bound - L) <= 2^-dead, the
        // skipped blocks' budget per component -- far chunks of a wide halo
        // qualify at larger x -- and x <= kMomXCap (fp32 Horner conditioning
        // e^(2x) bounded).  8-wide (MW 8): lane l tests its own block (one
        // CoefM8 entry per block, degree kMom8Deg), the chunk is the block.
        uint64_t cmask = 0, cmaskh = 0;
        if constexpr (MW == 8) {
          bool elig = false;
          if (KR <= 2 && cmv8 && has) {
            const CoefM8 *q = cmv8 + (2 * r0 + lane);
            const float cf = (float)q->center;
            const float x = fmaxf(fabsf(win.lo - cf), fabsf(win.hi - cf)) * q->xh;
            const float l2tau = (float)(kMom8Deg + 1) * __builtin_amdgcn_logf(x) +
                                x * 1.44269504f - kMom8Log2Fact;
            elig = x <= kMom8XLim || (x <= kMomXCap && l2tau + bnd <= win.thr + 1.0f);
          }
          cmask = __ballot(live && elig);
        } else {
          // (with the degree-15 table, CoefMH: the chunks the degree-9 form
          // leaves out take it when its own bound allows -- x <= kMom8XLim,
          // or the weighted criterion at degree 15)
          const float bnd1 = __builtin_bit_cast(float, dpp<kDppXor1>(__builtin_bit_cast(int, bnd)));
          bool elig = false, eligh = false;
          if (KR <= 2 && cmv && has && !(lane & 1)) {
            const CoefM *q = cmv + (r0 + (lane >> 1));
            const float cf = (float)q->center;
            const float x = fmaxf(fabsf(win.lo - cf), fabsf(win.hi - cf)) * q->xh;
            const float lx = __builtin_amdgcn_logf(x), xl = x * 1.44269504f;
            const float bb = fmaxf(bnd, bnd1);
            const float l2tau = (float)(kMomDeg + 1) * lx + xl - kMomLog2Fact;
            elig = x <= kMomXLim || (x <= kMomXCap && l2tau + bb <= win.thr + 1.0f);
            if (cmvh && !elig) {
              const float l2tauh = (float)(kMom8Deg + 1) * lx + xl - kMom8Log2Fact;
              eligh = x <= kMom8XLim || (x <= kMomXCap && l2tauh + bb <= win.thr + 1.0f);
            }
          }
          const uint64_t lm = __ballot(live);
          cmask = (lm | (lm >> 1)) & __ballot(elig) & kEven;
          cmaskh = (lm | (lm >> 1)) & __ballot(eligh) & kEven;
        }
        const uint64_t cmall = cmask | cmaskh;
        const uint64_t cover = MW == 8 ? cmask : cmall | (cmall << 1);
        if constexpr (CENSUS) {
          const int n = (cmall >> lane) & 1 ? min(MW == 8 ? kGroup : kMomChunk, nb - k0) : 0;
          const int nh = (cmaskh >> lane) & 1 ? min(kMomChunk, nb - k0) : 0;
          uint32_t mx = (uint32_t)n, mh = (uint32_t)nh;
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) {
            mx += __shfl_xor(mx, o, 64);
            mh += __shfl_xor(mh, o, 64);
          }
          cen.mom += mx * (uint32_t)nvalid;
          cen.momh += mh * (uint32_t)nvalid;
          if (MW == 8) cen.mom8 += mx * (uint32_t)nvalid;
          if constexpr (MW != 8) {
            // (the chunk's blocks counted as evaluated whether or not both were live)
            const uint64_t lm = __ballot(live);
            uint32_t lx = (uint32_t)(has && (((cover & ~lm) >> lane) & 1) ? min(kGroup, nb - k0) : 0);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) lx += __shfl_xor(lx, o, 64);
            cen.exec += lx * (uint32_t)nvalid;
            cen.shift += lx * (uint32_t)nvalid;
          }
        }
        if constexpr (MW == 8 && KR == 2) {
          // two blocks per iteration, both loaded at its top (no group live
          // across the back edge: a loop-carried 21-SGPR group was spilled to
          // VGPR lanes every iteration); their fp32 sums added in fp32 and
          // converted once (as the pair loop below).  The second of an odd
          // last pair is block 0 of the round again, a valid address, its sum
          // dropped.
          KCM8 *rm = uniform_ptrm8(cmv8) + 2 * r0;
          uint64_t cm = cmask;
          while (cm) {
            Mom8Group ga, gb;
            load_mom8(rm, low_bit(cm), ga);
            cm &= cm - 1;
            const bool two = cm != 0;
            load_mom8(rm, low_bit(cm), gb);
            cm &= cm - 1;
            f2v a0, p0, a1, p1;
            mom8_terms(ga, Mf, y, a0, p0);
            mom8_terms(gb, Mf, y, a1, p1);
            float b0[2], b1[2];
            mom_sum(a0, p0, b0);
            mom_sum(a1, p1, b1);
#pragma unroll
            for (int r = 0; r < KR; ++r) s[r] += (double)(two ? b0[r] + b1[r] : b0[r]);
          }
        } else if constexpr (MW == 8 && KR == 1) {
          // one row: blocks in pairs (the second of an odd last pair is block
          // 0 of the round again, a valid address, its sum dropped)
          KCM8 *rm = uniform_ptrm8(cmv8) + 2 * r0;
          uint64_t cm = cmask;
          while (cm) {
            Mom8Group ga, gb;
            load_mom8(rm, low_bit(cm), ga);
            cm &= cm - 1;
            const bool two = cm != 0;
            load_mom8(rm, low_bit(cm), gb);
            cm &= cm - 1;
            f2v a2, p2;
            mom8_terms2(ga, gb, Mf, y[0], a2, p2);
            float b2[2];
            mom_sum(a2, p2, b2);
            s[0] += (double)(two ? b2[0] + b2[1] : b2[0]);
          }
        } else if constexpr (KR == 2) {
          if (cmaskh) {
            // the degree-15 form of 16-component chunks (CoefMH), as the
            // 8-wide loop above with a chunk index
            KCM8 *rh = uniform_ptrm8(cmvh) + r0;
            uint64_t cm = cmaskh;
            bool hm = true;
            Mom8Group g;
            load_mom8(rh, low_bit(cm) >> 1, g);
            while (hm) {
              f2v a0, p0;
              mom8_terms(g, Mf, y, a0, p0);
              cm &= cm - 1;
              hm = cm != 0;
              load_mom8(rh, low_bit(cm) >> 1, g);
              __builtin_amdgcn_sched_barrier(0);
              float b0[2];
              mom_sum(a0, p0, b0);
              if (!hm) {
#pragma unroll
                for (int r = 0; r < KR; ++r) s[r] += (double)b0[r];
                break;
              }
              f2v a1, p1;
              mom8_terms(g, Mf, y, a1, p1);
              cm &= cm - 1;
              hm = cm != 0;
              load_mom8(rh, low_bit(cm) >> 1, g);
              __builtin_amdgcn_sched_barrier(0);
              float b1[2];
              mom_sum(a1, p1, b1);
#pragma unroll
              for (int r = 0; r < KR; ++r) s[r] += (double)(b0[r] + b1[r]);
            }
          }
          KCM *rm = uniform_ptrm(cmv) + r0;
          uint64_t cm = cmask;
          bool hm = cm != 0;
          MomGroup g;
          if (hm) load_mom(rm, low_bit(cm) >> 1, g);
          // two chunks per iteration, their fp32 sums added in fp32 and
          // converted once (as the pair loop below)
          while (hm) {
            f2v a0, p0;
            mom_terms(g, Mf, y, a0, p0);
            cm &= cm - 1;
            hm = cm != 0;
            load_mom(rm, low_bit(cm) >> 1, g);
            __builtin_amdgcn_sched_barrier(0);
            float b0[2];
            mom_sum(a0, p0, b0);
            if (!hm) {
#pragma unroll
              for (int r = 0; r < KR; ++r) s[r] += (double)b0[r];
              break;
            }
            f2v a1, p1;
            mom_terms(g, Mf, y, a1, p1);
            cm &= cm - 1;
            hm = cm != 0;
            load_mom(rm, low_bit(cm) >> 1, g);
            __builtin_amdgcn_sched_barrier(0);
            float b1[2];
            mom_sum(a1, p1, b1);
#pragma unroll
            for (int r = 0; r < KR; ++r) s[r] += (double)(b0[r] + b1[r]);
          }
        } else if constexpr (KR == 1) {
          // one row: chunks in pairs (the second of an odd last pair is chunk
          // 0 of the round again, a valid address, its sum dropped)
          KCM *rm = uniform_ptrm(cmv) + r0;
          uint64_t cm = cmask;
          while (cm) {
            MomGroup ga, gb;
            load_mom(rm, low_bit(cm) >> 1, ga);
            cm &= cm - 1;
            const bool two = cm != 0;
            load_mom(rm, low_bit(cm) >> 1, gb);
            cm &= cm - 1;
            f2v a2, p2;
            mom_terms2(ga, gb, Mf, y[0], a2, p2);
            float b2[2];
            mom_sum(a2, p2, b2);
            s[0] += (double)(two ? b2[0] + b2[1] : b2[0]);
          }
        }
        uint64_t m = __ballot(live && !wide) & ~cover;
        bool hv = m != 0;
        CoefGroup32 g32;
        auto ld32 = [&](uint32_t j) {
          if constexpr (STG) load_block32_lds(rbl, j, g32);
          else load_block32(rb, j, g32);
        };
        if (hv) ld32(low_bit(m));
        // two live blocks per iteration: their fp32 sums (terms <= 1, 16 of
        // them) are added in fp32 and converted once (tools/fp32_pair_error.py
        // blockf32_uu_pair: 2.3e-8 relative at config 4 against 2.2e-8)
        while (hv) {
          float d[KR][kGroup], b0[KR];
          lse_terms_f32<KR>(g32, Mf, y, d);
          m &= m - 1;
          hv = m != 0;
          ld32(low_bit(m));
          __builtin_amdgcn_sched_barrier(0);
          lse_block_sum<KR>(d, b0);
          if (!hv) {
#pragma unroll
            for (int r = 0; r < KR; ++r) s[r] += (double)b0[r];
            break;
          }
          float b1[KR];
          lse_terms_f32<KR>(g32, Mf, y, d);
          m &= m - 1;
          hv = m != 0;
          ld32(low_bit(m));
          __builtin_amdgcn_sched_barrier(0);
          lse_block_sum<KR>(d, b1);
#pragma unroll
          for (int r = 0; r < KR; ++r) s[r] += (double)(b0[r] + b1[r]);
        }
        uint64_t xk = __ballot(live && wide) & ~cover;
        while (next_live<STRIDE>(xk, r0, kg)) {
          CoefGroup g;
          load_group(cs, kg, g);
          float d[KR][kGroup];
          lse_terms_shifted<KR>(g, M, y, y2, d);
          lse_fold_shifted<KR>(d, s);
        }
      } else if constexpr (F32) {
        const float Mf = (float)M;  // an integer (< 2^24 in magnitude): exact
        CoefGroup32 g32;
        if (have) load_group32(c32, kg, g32);
        // two live blocks per iteration: their fp32 sums (terms <= 1, 16 of
        // them) are added in fp32 and converted once (tools/fp32_pair_error.py
        // blockf32_uu_pair: 2.3e-8 relative at config 4 against 2.2e-8)
        while (have) {
          float d[KR][kGroup], b0[KR];
          lse_terms_f32<KR>(g32, Mf, y, d);
          have = next_live<STRIDE>(mk, r0, kg);
          load_group32(c32, kg, g32);
          __builtin_amdgcn_sched_barrier(0);
          lse_block_sum<KR>(d, b0);
          if (!have) {
#pragma unroll
            for (int r = 0; r < KR; ++r) s[r] += (double)b0[r];
            break;
          }
          float b1[KR];
          lse_terms_f32<KR>(g32, Mf, y, d);
          have = next_live<STRIDE>(mk, r0, kg);
          load_group32(c32, kg, g32);
          __builtin_amdgcn_sched_barrier(0);
          lse_block_sum<KR>(d, b1);
#pragma unroll
          for (int r = 0; r < KR; ++r) s[r] += (double)(b0[r] + b1[r]);
        }
        uint64_t xk = __ballot(live && wide);
        while (next_live<STRIDE>(xk, r0, kg)) {
          CoefGroup g;
          load_group(cs, kg, g);
          float d[KR][kGroup];
          lse_terms_shifted<KR>(g, M, y, y2, d);
          lse_fold_shifted<KR>(d, s);
        }
      } else {
        CoefGroup cgp;
        if (have) load_group(cs, kg, cgp);
        while (have) {
          float d[KR][kGroup];
          lse_terms_shifted<KR>(cgp, M, y, y2, d);
          have = next_live<STRIDE>(mk, r0, kg);
          load_group(cs, kg, cgp);
          __builtin_amdgcn_sched_barrier(0);
          lse_fold_shifted<KR>(d, s);
        }
      }
    }
    // the probe's block on its own (outside the searched rounds; census
    // builds visit every round, it is in one of them)
    if (!CENSUS && pbk >= 0 && probe_live) {
      CoefGroup g;
      load_group(cs, pbk * kGroup, g);
      float d[KR][kGroup];
      lse_terms_shifted<KR>(g, M, y, y2, d);
      lse_fold_shifted<KR>(d, s);
    }
    bool ok = true;
    double smax = 0.0;
#pragma unroll
    for (int r = 0; r < KR; ++r)
      if (valid[r] && y[r] == y[r]) {
        ok &= s[r] >= 0.0625;
        smax = fmax(smax, s[r]);
      }
    if (__all(ok)) break;
    if (attempt > 0 || !__all(ok || smax >= 0x1p-100)) return false;
    // lanes that fit keep M (identical second pass); the others re-centre
    // ceil(log2 smax) from the exponent of smax = m 2^e (m in [1/2, 1)): e,
    // or e - 1 when smax is a power of two -- exactly the library's value,
    // without its polynomial constants held in (spilled) registers
    if (!ok) {
      const int e = __builtin_amdgcn_frexp_exp(smax);
      const double mt = __builtin_amdgcn_frexp_mant(smax);
      M += (double)(mt == 0.5 ? e - 1 : e) + 1.0;
    }
  }
#pragma unroll
  for (int r = 0; r < KR; ++r) out[r] = (y[r] != y[r]) ? LseAcc{NAN, NAN} : LseAcc{M, s[r]};
  if (STRIDE == 1) WSTAMP(7);
  return true;
}

// Mixtures of at most kSmallMix components on wave tiles (the good side: K_b
// = n_below + 1 <= 26) -- a log-sum-exp straight from the block's LDS copy
// of the coefficients, in one pass against the mixture's peak bound mtop (the
// same fp64 t = alpha + y'(beta + gamma y') as lse_terms); a wave with a
// candidate far below every peak takes the two-pass form: the lane's largest
// term m, then the terms 2^(t - ceil m) summed in fp32 over runs of 8 and in
// fp64 across them (round 5's form, ~40% more work).  No envelope
// round, window, scalar coefficient loads or per-group lift: the envelope /
// fp64 lift loop these mixtures took (their blocks are wide in sigma units,
// so never in the fp32 form) spent ~7 us per config-5 wave waiting on loads.
// Output as lse_chunks': NaN for a NaN candidate, (-inf, 0) when every term
// is -inf, a NaN term makes the sum NaN.
constexpr int kSmallMix = 32;
template <int KR>
__device__ __forceinline__ void lse_small(const double (*__restrict__ cf)[kSmallMix], int K,
                                          const double (&y)[KR], LseAcc (&out)[KR], double mtop) {
  double y2[KR];
#pragma unroll
  for (int r = 0; r < KR; ++r) y2[r] = y[r] * y[r];
  // one pass against the mixture's bound mtop (staged with the coefficients:
  // row 3 = alpha - mtop), the terms 2^(t - mtop) <= 1 summed in fp32 over
  // runs of 8 and in fp64 across them.  A lane whose sum comes out below
  // 2^-60 (a candidate far below every component's peak: its terms may have
  // flushed in fp32) sends the wave to the two-pass form below
  if (mtop > -INFINITY && mtop < INFINITY) {
    double sd[KR];
    float sf[KR];
#pragma unroll
    for (int r = 0; r < KR; ++r) { sd[r] = 0.0; sf[r] = 0.0f; }
    for (int k = 0; k < K; ++k) {
      const double cx = cf[3][k], cy = cf[1][k], cz = cf[2][k];
#pragma unroll
      for (int r = 0; r < KR; ++r)
        sf[r] += __builtin_amdgcn_exp2f((float)fma(cz, y2[r], fma(cy, y[r], cx)));
      if ((k & 7) == 7) {
#pragma unroll
        for (int r = 0; r < KR; ++r) { sd[r] += (double)sf[r]; sf[r] = 0.0f; }
      }
    }
    bool ok = true;
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      sd[r] += (double)sf[r];
      ok &= !(sd[r] < 0x1p-60);  // (NaN: the lpdf is NaN either way)
    }
    if (__all(ok)) {
#pragma unroll
      for (int r = 0; r < KR; ++r)
        out[r] = (y[r] != y[r]) ? LseAcc{NAN, NAN} : LseAcc{mtop, sd[r]};
      return;
    }
  }
  double m[KR];
#pragma unroll
  for (int r = 0; r < KR; ++r) m[r] = -INFINITY;
  for (int k = 0; k < K; ++k) {
    const double cx = cf[0][k], cy = cf[1][k], cz = cf[2][k];
#pragma unroll
    for (int r = 0; r < KR; ++r) m[r] = fmax(m[r], fma(cz, y2[r], fma(cy, y[r], cx)));
  }
  double ms[KR], sd[KR];
  float sf[KR];
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    m[r] = ceil(m[r]);
    ms[r] = m[r] == -INFINITY ? 0.0 : m[r];
    sd[r] = 0.0;
    sf[r] = 0.0f;
  }
  for (int k = 0; k < K; ++k) {
    const double cx = cf[0][k], cy = cf[1][k], cz = cf[2][k];
#pragma unroll
    for (int r = 0; r < KR; ++r)
      sf[r] += __builtin_amdgcn_exp2f((float)(fma(cz, y2[r], fma(cy, y[r], cx)) - ms[r]));
    if ((k & 7) == 7) {
#pragma unroll
      for (int r = 0; r < KR; ++r) { sd[r] += (double)sf[r]; sf[r] = 0.0f; }
    }
  }
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    sd[r] += (double)sf[r];
    if (y[r] != y[r]) out[r] = LseAcc{NAN, NAN};
    else if (m[r] == -INFINITY) out[r] = sd[r] == 0.0 ? LseAcc{-INFINITY, 0.0} : LseAcc{NAN, NAN};
    else out[r] = LseAcc{m[r], sd[r]};
  }
}

// PRUNE setup, part 1 (once per wave, shared by both mixtures): the wave's
// candidate range [lo, hi] (y' units, fp32 rounded outward) and whether
// every valid candidate is finite.
struct LseRange {
  float lo, hi;
  bool ok, any;
};
template <int KR>
__device__ __forceinline__ LseRange lse_range(const double (&y)[KR], const bool (&valid)[KR]) {
  // (each lane rounds its own values outward to fp32 and the wave reduces
  // those: rounding is monotone, so this is the fp32-outward rounding of the
  // fp64 extremes -- the same floats as reducing in fp64, half the shuffles)
  float wl = INFINITY, wh = -INFINITY;
  bool ok = true;
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    if (!valid[r]) continue;
    ok &= fabs(y[r]) < INFINITY;
    const float f = (float)y[r];
    const float fl = ((double)f > y[r]) ? nextafterf(f, -INFINITY) : f;
    const float fh = ((double)f < y[r]) ? nextafterf(f, INFINITY) : f;
    wl = fminf(wl, fl);
    wh = fmaxf(wh, fh);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    wl = fminf(wl, __shfl_xor(wl, o, 64));
    wh = fmaxf(wh, __shfl_xor(wh, o, 64));
  }
  auto sf = [](float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
  };
  return LseRange{sf(wl), sf(wh), __all(ok) != 0, wl <= wh};
}

// PRUNE setup, part 2 (per mixture): from the mixture's probe component (its
// widest, the Parzen prior), a lower bound on every lane's final exponent m
// (m >= max_k t_k >= t_probe) and with it the skip threshold.  Non-finite
// candidates or a missing probe disable the skip (thr = -inf).
template <int KR>
__device__ __forceinline__ LseWindow lse_window(KDbl *__restrict__ cs, int probe, int K,
                                                const double (&y)[KR], const bool (&valid)[KR],
                                                const LseRange &rg) {
  double tmin = INFINITY;
  bool ok = rg.ok && probe >= 0 && probe < K;
  const int p = ok ? probe : 0;
  const double px = cs[coef_off(p, 0)], py = cs[coef_off(p, 1)], pz = cs[coef_off(p, 2)];
#pragma unroll
  for (int r = 0; r < KR; ++r)
    if (valid[r]) tmin = fmin(tmin, fma(fma(pz, y[r], py), y[r], px));
  // threshold one unit conservative; the (wave-uniform) values travel in SGPRs.
  // Each lane maps its own minimum through the (monotone) fp32 threshold and
  // the wave takes the smallest: the threshold of the wave's minimum, with
  // one fp32 reduction instead of an fp64 one (fmin never yields NaN here:
  // it starts at +inf and skips NaN terms); the validity test by ballot
  const float dead = kLseDeadBase + (float)(32 - __builtin_clz((unsigned)max(K - 1, 1)));
  float thl = (float)(tmin - (double)dead) - 1.0f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) thl = fminf(thl, __shfl_xor(thl, o, 64));
  ok = ok && __all(tmin > -1.0e30);
  float th = ok ? thl : -INFINITY;
  if (!rg.any) th = -INFINITY;  // no valid candidate in the wave
  th = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, th)));
  return LseWindow{rg.lo, rg.hi, th};
}

// CENSUS counts, per lane, the valid pairs, the live ones and the ones
// evaluated (live for some candidate of the wave) -- roofline accounting only.
struct Census {
  uint32_t total, live, exec;
};

// Candidate-side bounds of the quantized lpdf, tpe.py:146-152 (GMM) and
// 284-293 (LGMM: on log scale, lb clipped at 0, both floored at EPS).
template <bool LOGN>
__device__ __forceinline__ void quant_bounds(const tpe_hp &H, double x, double &ub, double &lb) {
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

// one quantized term w (Phi(ub) - Phi(lb)) in the reference's operation
// order (GMM: 0.5 * (1 + erf), LGMM: .5 + .5 * erf; two-stage difference)
template <bool LOGN>
__device__ __forceinline__ double erf_term(double zu, double zl, double w) {
#pragma clang fp contract(off)
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
  return inc;
}

// a term whose two erf arguments are beyond 6.5 on one side is an exact 0
// (erf saturates to +-1 from 5.93)
__device__ __forceinline__ bool erf_dead(double zu, double zl) {
  return (zu >= 6.5 && zl >= 6.5) || (zu <= -6.5 && zl <= -6.5);
}

// the same chunks, quantized: sum_k w (Phi(ub) - Phi(lb)),
// tpe.py:146-160 (GMM: 0.5 * (1 + erf)) / 284-299 (LGMM: .5 + .5 * erf).
// Canonical order (k_lattice reproduces it): each chunk is summed in
// component order from 0, the chunk sums are added to the wave's total.
// A chunk is skipped when every candidate of the wave is provably beyond
// 6.6 sigma-units of every one of its components on one side (Coef.w holds
// 6.6 * max(sqrt(2) sigma, EPS)): all its terms are then exact zeros.
// wlo / whi: the wave's min lb / max ub; `exact` false (a NaN bound)
// disables the chunk test.  Inside a chunk, a component is skipped when all
// its terms in the wave are exact zeros.
template <int KR, bool LOGN, bool CENSUS>
__device__ __forceinline__ void erf_chunks(KDbl *__restrict__ cs, int c0, int nb,
                                           const double (&ub)[KR], const double (&lb)[KR],
                                           const bool (&valid)[KR], double wlo, double whi,
                                           bool exact, double (&prob)[KR], Census &cen) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < KR; ++r) prob[r] = 0.0;
  for (int c = c0; c * kChunk < nb; c += kWaves) {
    const int k0 = c * kChunk, k1 = min(nb, k0 + kChunk);
    if (exact) {  // the chunk's envelope, one component per lane of the first kChunk
      double lo = INFINITY, hi = -INFINITY;
      if (lane < k1 - k0) {
        const double qx = cs[coef_off(k0 + lane, 0)], qw = cs[coef_off(k0 + lane, 3)];
        lo = qx - qw;
        hi = qx + qw;
      }
#pragma unroll
      for (int o = kChunk / 2; o > 0; o >>= 1) {
        lo = fmin(lo, __shfl_xor(lo, o, 64));
        hi = fmax(hi, __shfl_xor(hi, o, 64));
      }
      lo = __shfl(lo, 0, 64);
      hi = __shfl(hi, 0, 64);
      if (wlo >= hi || whi <= lo) {
        if constexpr (CENSUS) {
#pragma unroll
          for (int r = 0; r < KR; ++r) cen.total += valid[r] ? (uint32_t)(k1 - k0) : 0u;
        }
        continue;
      }
    }
    double pc[KR];
#pragma unroll
    for (int r = 0; r < KR; ++r) pc[r] = 0.0;
    for (int k = k0; k < k1; ++k) {
      const double cx = cs[coef_off(k, 0)], cy = cs[coef_off(k, 1)];
      double zu[KR], zl[KR];
      bool dead_all = true;
#pragma unroll
      for (int r = 0; r < KR; ++r) {
        zu[r] = (ub[r] - cx) * cy;
        zl[r] = (lb[r] - cx) * cy;
        const bool dead = !valid[r] || erf_dead(zu[r], zl[r]);
        dead_all &= dead;
        if constexpr (CENSUS) {
          cen.total += valid[r] ? 1u : 0u;
          cen.live += dead ? 0u : 1u;
        }
      }
      const bool skip = __all(dead_all);
      if constexpr (CENSUS) {
#pragma unroll
        for (int r = 0; r < KR; ++r) cen.exec += (valid[r] && !skip) ? 1u : 0u;
      }
      if (skip) continue;  // exact zeros for every candidate of the wave
      const double w = cs[coef_off(k, 2)];
#pragma unroll
      for (int r = 0; r < KR; ++r) pc[r] += erf_term<LOGN>(zu[r], zl[r], w);
    }
#pragma unroll
    for (int r = 0; r < KR; ++r) prob[r] += pc[r];
  }
}

#ifdef TPE_STAMPS
// diagnostic build only (make dbg; tools/score_stamps.py): per-block wall
// clock (100 MHz) at entry, after the component loop and at the end, plus the
// (slot, tile) and hardware ids of the block, for the blocks of suggestion 0
__device__ unsigned long long g_score_stamps[8192][4];
// (TPE_STAMPS_WAVE_LSE: only the wave-tile log-sum-exp launches stamp -- a
// mixed level's lookup launch runs beside it and would overwrite its rows)
#ifdef TPE_STAMPS_WAVE_LSE
#define STAMP_KIND_OK kind_wave_lse(KIND)
#else
#define STAMP_KIND_OK true
#endif
#define SSTAMP(i)                                                                        \
  do {                                                                                   \
    if (STAMP_KIND_OK && threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.x < 8192) {     \
      const unsigned b = blockIdx.x;                                                     \
      g_score_stamps[b][i] = wall_clock64();                                             \
      if (i == 0)                                                                        \
        g_score_stamps[b][3] =                                                           \
            ((unsigned long long)(slot & 0xffff) << 48) |                                \
            ((unsigned long long)(tile & 0xffff) << 32) |                                \
            ((unsigned long long)(__builtin_amdgcn_s_getreg(63488 | 20) & 0xf) << 16) |  \
            (__builtin_amdgcn_s_getreg(63488 | 4) & 0xffff);                             \
    }                                                                                    \
  } while (0)
#else
#define SSTAMP(i) do {} while (0)
#endif

template <int R>
struct ScoreSmemT {
  double2 wpart[2][kWaves][R][64];      // per-wave partials (below, above)
  double2 merged[2][R][64];             // merged per (mixture, candidate row)
  double xs[R > 1 ? kWaves : 1][R][64];  // two-row wave tiles: each wave's candidates
                                        //   (kept here, not in registers, till finalize)
  double best_s[kWaves], best_v[kWaves];  // wave tiles: each wave's argmax
  int64_t best_i[kWaves];
#ifdef TPE_REREAD
  int64_t best_li[kWaves];
#endif
  uint32_t arrive;                      // wave tiles: waves done with the tile
  double small[2][4][kSmallMix];        // wave tiles: mixtures of <= kSmallMix components
                                        //   (alpha, beta, gamma, alpha - mtop rows; below,
                                        //   above), lse_small
  double small_m[2];                    //   mtop = ceil(max_k peak_k), the terms' bound
  DrawTableT<kFuseTab> dt;              // lookup tiles drawing their candidates (lookup_inline)
  double top_s;                         // lookup scans: the best score any value can get
  int top_nan;                          //   (a NaN score: top is NaN)
  double red_s[kWaves];                 //   its per-wave partial maxima
  int red_n[kWaves];
};
typedef ScoreSmemT<kRMax> ScoreSmem;
// k_score_wave1: one candidate row, and the staged tables beside it
struct ScoreSmem1 : ScoreSmemT<1> {
  StageSmem stg;
};

#ifdef TPE_REREAD
// diagnostic build only (make dbg3; tools/reread_diag.py): per hp of
// suggestion 0, the winner's value and index and what a finalize-time re-read
// of its candidate finds at the addresses it could have taken
__device__ double g_reread[512][20];
__device__ int64_t g_tile_li[1 << 20][2];
#endif

#ifdef TPE_REREAD2
// diagnostic build only (make dbg4; tools/reread_shard.py): at finalize,
// every valid wave-tile row compares the candidate it scored (registers) with
// a plain and a volatile re-read of the same slot; [0] rows, [1] plain
// differs, [2] volatile differs, [3] examples taken; then up to 64 examples
// of (li, cpos[li], x, plain, volatile, chunk begin, n_cand, hp)
__device__ unsigned long long g_rr2_cnt[4];
__device__ double g_rr2_ex[64][8];
#endif

// A final record of a tile_draw launch that ends its call (ScoreArgs::pub_*),
// called by a whole wave after its lane 0 stored the record write-through
// (store_record_sc1, drained): lane 0 takes an arrival ticket; the wave whose
// ticket is the launch's last copies every record of the call (agent-scope
// loads) into the pinned host buffer, then a system-scope release and the
// sequence word the host spins on -- what k_publish does, one launch less.
// (The tile records' protocol above: sc1 stores, ticket, sc1 loads, no L2
// write-back; the diagnostic TPE_REREAD build stores plainly and releases.)
// Every store is a vector store.
__device__ __forceinline__ void store_record_sc1(Partial *rr, const Partial &v) {
  gu64 *w = (gu64 *)(uintptr_t)rr;
  __hip_atomic_store(w + 0, dbits(v.score), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(w + 1, dbits(v.value), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(w + 2, (uint64_t)v.index, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(w + 3, (uint64_t)(uint32_t)v.active | ((uint64_t)(uint32_t)v.pad << 32),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void publish_arrive(const ScoreArgs &A) {
  const int lane = threadIdx.x & 63;
  int last = 0;
  if (lane == 0) {
#ifdef TPE_REREAD
    constexpr int kOrd = __ATOMIC_RELEASE;
#else
    constexpr int kOrd = __ATOMIC_RELAXED;
#endif
    const uint32_t t = __hip_atomic_fetch_add(A.pub_ticket, 1u, kOrd, __HIP_MEMORY_SCOPE_AGENT);
    last = t == (uint32_t)A.pub_events - 1 ? 1 : 0;
    if (last) __hip_atomic_store(A.pub_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!__shfl(last, 0, 64)) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the ticket
  gu64 *src = (gu64 *)(uintptr_t)A.results;
  for (int i = lane; i < A.pub_words; i += 64)
    A.pub_dst[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (lane == 0) __hip_atomic_store(A.pub_flag, A.pub_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// (SM: ScoreSmem, or ScoreSmem1 for the one-row wave tiles, whose
// workgroup stages both mixtures' tables in LDS when they fit kStageBlocks)
template <int KIND, bool CENSUS, typename SM, bool LDRAW = false, bool TDRAW = false, int MW = 16>
__device__ __forceinline__ void score_tile(const ScoreArgs &A, SM &sm, int slot, int tile,
                                           int ntiles, bool known_active) {
  constexpr bool STAGE = std::is_same<SM, ScoreSmem1>::value;
  constexpr int KR = tile_rows(KIND);
  constexpr bool LSE = kind_lse(KIND);
  constexpr bool WT = tile_waves(KIND) > 1;  // wave tiles: own candidates, all components
  constexpr bool ERF = KIND == KIND_ERF_G || KIND == KIND_ERF_L;
  constexpr bool LAT = KIND == KIND_LAT;  // quantized, looked up on its value lattice
  constexpr bool LOGN = kind_logn(KIND);
  const int s = blockIdx.y;
  const int hp = A.level_hps[slot];
  const tpe_hp H = A.hps[hp];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  SSTAMP(0);
  const bool act = A.force_active || known_active ||
                   hp_active(H, A.results + (int64_t)s * A.n_hp, A.cond_parent, A.cond_branch);
  if (!act) {  // one record says "inactive"; no tickets are taken
    if constexpr (TDRAW) {  // (its final record: one arrival)
      if (A.pub_flag) {
        if (tile == 0 && threadIdx.x < 64) {
          if (threadIdx.x == 0)
            store_record_sc1(A.results + (int64_t)s * A.n_hp + hp, Partial{NAN, NAN, -1, 0, 0});
          publish_arrive(A);
        }
        return;
      }
    }
    if (tile == 0 && threadIdx.x == 0)
      A.results[(int64_t)s * A.n_hp + hp] = Partial{NAN, NAN, -1, 0, 0};
    return;
  }
  const int64_t sb = 2 * (int64_t)hp, sa = sb + 1;
  const MixInfo ib = A.info[sb], ia = A.info[sa];
  // staged tables (one-row wave tiles): below blocks [0, nbb), above after
  const int nbb = (ib.K + kCoefBlock - 1) / kCoefBlock, nba = (ia.K + kCoefBlock - 1) / kCoefBlock;
  bool staged = false;
  if constexpr (WT) {  // the block's arrival counter (finalize), before any wave can arrive
    if (threadIdx.x == 0) sm.arrive = 0u;
    // small mixtures' coefficients (lse_small) into LDS: thread t of the first
    // 2 x kSmallMix copies component t % kSmallMix of mixture t / kSmallMix
    if constexpr (LSE) {
      // (wave 0, every lane: lanes 32q .. 32q + 31 hold mixture q.  The
      // bound mtop: every term t_k(y) is at most its peak alpha - beta^2 /
      // (4 gamma), so 2^(t - mtop) <= 1 for any candidate -- lse_small's one
      // pass needs no per-lane maximum)
      if (threadIdx.x < 2 * kSmallMix) {
        const int q = threadIdx.x / kSmallMix, k = threadIdx.x % kSmallMix;
        const int Kq = q ? ia.K : ib.K;
        const bool cp = Kq <= kSmallMix && k < Kq && A.lse_prune != 0;
        double ca = 0.0, cb = 0.0, cg = 0.0, pk = -INFINITY;
        if (cp) {
          const double *t = reinterpret_cast<const double *>(A.coef + (q ? sa : sb) * A.kcap);
          ca = t[coef_off(k, 0)];
          cb = t[coef_off(k, 1)];
          cg = t[coef_off(k, 2)];
          pk = ca - cb * cb / (4.0 * cg);
        }
#pragma unroll
        for (int o = kSmallMix / 2; o > 0; o >>= 1) pk = fmax(pk, __shfl_xor(pk, o, 64));
        const double mt = ceil(pk);
        if (cp) {
          sm.small[q][0][k] = ca;
          sm.small[q][1][k] = cb;
          sm.small[q][2][k] = cg;
          sm.small[q][3][k] = ca - mt;
        }
        if (k == 0) sm.small_m[q] = mt;
      }
    }
    if constexpr (STAGE) {
      staged = nbb + nba <= kStageBlocks && A.lse_prune > 2;  // block-uniform
      if (staged) {
        // 16-B units: per block its envelope, then its Coef32 (8 units)
        const float4 *gb = reinterpret_cast<const float4 *>(A.coef + sb * A.kcap);
        const float4 *ga = reinterpret_cast<const float4 *>(A.coef + sa * A.kcap);
        const float4 *cb32 = reinterpret_cast<const float4 *>(A.coef32 + sb * (A.kcap / kCoefBlock));
        const float4 *ca32 = reinterpret_cast<const float4 *>(A.coef32 + sa * (A.kcap / kCoefBlock));
        float4 *env = sm.stg.env;
        float4 *c32 = reinterpret_cast<float4 *>(sm.stg.c32);
        for (int u = threadIdx.x; u < 9 * (nbb + nba); u += blockDim.x) {
          const int b = u / 9, part = u - 9 * b;
          const bool above = b >= nbb;
          const int bl = above ? b - nbb : b;
          if (part == 0)  // the w-row of block bl: 16 float4 per block, the envelope at 12
            env[b] = (above ? ga : gb)[(int64_t)bl * 16 + 12];
          else
            c32[(int64_t)b * 8 + part - 1] = (above ? ca32 : cb32)[(int64_t)bl * 8 + part - 1];
        }
      }
    }
    __syncthreads();
    WSTAMP(0);
  }
  const Coef *__restrict__ cb = A.coef + sb * A.kcap;
  const Coef *__restrict__ ca = A.coef + sa * A.kcap;
  const int64_t coff = (int64_t)s * A.cand_sstride + (int64_t)(A.cand_slot0 + slot) * A.n_cand;
  const double *__restrict__ cand = A.cand + coff;
  // value-bucketed candidates (k_bucket, or the sorted draw) carry their
  // chunk positions: the quantized kinds always, log-sum-exp when lse_pos
  const int32_t *__restrict__ cpos =
      ((ERF || (LSE && A.lse_pos)) && A.cand_pos) ? A.cand_pos + coff : nullptr;

  // lookup slots drawn here (ScoreArgs::lookup_draw): the below mixture's
  // draw table in LDS (block-wide, before any wave can arrive), then each
  // candidate is the draw of its global index, as k_draw_sorted would have
  // written it
  bool ldraw = false;
  if constexpr (LDRAW && (LAT || KIND == KIND_CAT)) {
    ldraw = lookup_inline(A, ib.K);  // block-uniform
    if (ldraw) build_table(H, ib.K, A.mw + sb * A.kcap, A.mmu + sb * A.kcap, A.msig + sb * A.kcap, sm.dt);
    // the scan's early exit (lookup_scan below): the largest score any value
    // of the slot can take -- over every category (CAT) or lattice point
    // (LAT), NaN on top as in numpy's argmax
    double ms = -INFINITY;
    int mn = 0;
    if constexpr (LAT) {
      // (the points a draw can reach: the lattice's two margin points on
      // each side absorb host/device rounding -- none is reachable for GMM,
      // whose clamped x / q rounds inside [rint(low / q), rint(high / q)];
      // for LGMM the device exp may reach one more point on each side)
      const LatInfo L = A.lat_info[hp];
      const int64_t m0 = H.family == TPE_LGMM ? 1 : 2;
      for (int64_t j = m0 + threadIdx.x; j < (int64_t)L.R - m0; j += blockDim.x) {
        const double2 v = A.lat[L.off + j];
        const double sc = v.x - v.y;
        mn |= sc != sc;
        ms = fmax(ms, sc);
      }
    } else {
      for (int c = threadIdx.x; c < ib.K; c += blockDim.x) {
        const double sc = reinterpret_cast<const double *>(cb)[coef_off(c, 0)] -
                          reinterpret_cast<const double *>(ca)[coef_off(c, 0)];
        mn |= sc != sc;
        ms = fmax(ms, sc);
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      ms = fmax(ms, __shfl_xor(ms, o, 64));
      mn |= __shfl_xor(mn, o, 64);
    }
    if (lane == 0) { sm.red_s[wave] = ms; sm.red_n[wave] = mn; }
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = -INFINITY;
      int n = 0;
      for (int w = 0; w < kWaves; ++w) { t = fmax(t, sm.red_s[w]); n |= sm.red_n[w]; }
      sm.top_s = t;
      sm.top_nan = n;
    }
    __syncthreads();
  }
  // tiny unsorted draws (ScoreArgs::tile_draw): the tile draws its own
  // candidates from the below mixture's LDS table -- the table and values of
  // k_draw<true> (K <= kFuseTab: the host only takes this path then)
  if constexpr (TDRAW) {
    if (ib.K >= 1 && ib.K <= kFuseTab)
      build_table(H, ib.K, A.mw + sb * A.kcap, A.mmu + sb * A.kcap, A.msig + sb * A.kcap, sm.dt);
  }
  int64_t li[KR];
  bool valid[KR];
  double x[KR], y[KR], ub[KR], lb[KR];
  // the wave's 64 * KR candidates.  Log-sum-exp wave tiles: the block's 8
  // waves take wave tiles spread over their 4096-candidate sort block (wave
  // w of the q-th of the sort block's nbs blocks: wave tile q + nbs w), not 8
  // consecutive ones -- a sort block spans the whole value range bucket by
  // bucket, so its dense value windows (the waves with the most live
  // component blocks) are shared out over blocks, CUs and SIMDs instead of
  // landing on one CU together.  A wave's sums depend only on its own
  // candidates: the mapping changes no result.
  // (wave-uniform: a scalar, so the finalize can recompute li from it)
  const int wvs = __builtin_amdgcn_readfirstlane(wave);
  int64_t wt0 = (int64_t)tile * tile_cands(KIND) + (WT ? wvs * 64 * KR : 0);
  if constexpr (kind_wave_lse(KIND)) {
    static_assert((kSortedBlock >> kSortLog2Large) == 1 &&
                      (1 << kSortLog2Small) % tile_cands(KIND) == 0,
                  "blocks tile the sort block");
    const int SBB = (1 << A.sort_log2) / tile_cands(KIND);  // blocks per sort block
    const int sb = tile / SBB, q = tile % SBB;
    const int nbs = min(SBB, ntiles - sb * SBB);
    wt0 = ((int64_t)sb * SBB * kWaves + q + (int64_t)nbs * wvs) * 64 * KR;
  }
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    li[r] = wt0 + r * 64 + lane;
    valid[r] = li[r] < A.n_cand;
    if constexpr (LDRAW && (LAT || KIND == KIND_CAT)) {
      // (self-drawing lookups: the scan in the finalize below, lookup_scan,
      // draws and scores its own candidates; nothing is read here)
      x[r] = 0.0;
      continue;
    } else if constexpr (TDRAW) {
      const uint64_t gi = (uint64_t)(A.cand_begin + li[r]);
      const uint64_t seed = suggestion_seed(A, s);
      const bool tab = ib.K >= 1 && ib.K <= kFuseTab;
      x[r] = !valid[r] ? (LOGN ? 1.0 : 0.0)
             : tab ? draw_table_ool<kFuseTab>(A.hps + hp, ib.K, A.mmu + sb * A.kcap,
                                              A.msig + sb * A.kcap, &sm.dt,
                                              draw_block0(seed, gi, (uint32_t)hp), seed, gi,
                                              (uint32_t)hp)
                   : draw_one_ool(A.hps + hp, A.info + sb, A.mw + sb * A.kcap, A.mmu + sb * A.kcap,
                                  A.msig + sb * A.kcap, seed, gi, (uint32_t)hp);
    } else {
      x[r] = valid[r] ? cand[li[r]] : (LOGN ? 1.0 : 0.0);
      if constexpr (LSE && WT && KR > 1) sm.xs[wave][r][lane] = x[r];
    }
    y[r] = ub[r] = lb[r] = 0.0;
    // candidate-side transforms, once per candidate
    if constexpr (LSE) {
      y[r] = (LOGN ? fast_log(x[r]) : x[r]) - H.prior_mu;
    } else if constexpr (ERF) {
      quant_bounds<LOGN>(H, x[r], ub[r], lb[r]);
    }
  }

  if constexpr (LSE || ERF) {
    // warm this XCD's L2 with both mixtures' coefficient lines: one dword per
    // 128-B line, issued before the component loop, so the loop's scalar loads
    // hit L2 instead of each group paying a far (MALL / HBM) round trip
    float sink = 0.f;
    if (A.l2_warm) {
      const int nlb = (ib.K + 3) >> 2, nla = (ia.K + 3) >> 2;
      for (int i = threadIdx.x; i < nlb + nla; i += blockDim.x) {
        const Coef *c = i < nlb ? cb + 4 * i : ca + 4 * (i - nlb);
        sink += *(const volatile float *)c;
      }
    }
    // wave w owns the chunks c = w (mod kWaves) of each mixture (the live
    // erf components of the tile spread over the waves)
    LseAcc lacc[2][KR];
    double pacc[2][KR];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < KR; ++r) { lacc[q][r] = LseAcc{-INFINITY, 0.0}; pacc[q][r] = 0.0; }
    Census cen{0u, 0u, 0u};
    // quantized: the wave's candidate envelope for the chunk skip test
    double wlo = INFINITY, whi = -INFINITY;
    bool exact = true;
    if constexpr (ERF) {
#pragma unroll
      for (int r = 0; r < KR; ++r) {
        if (!valid[r]) continue;
        exact &= lb[r] == lb[r] && ub[r] == ub[r];
        // both bounds: a clipped bound pair may come out with ub < lb
        wlo = fmin(wlo, fmin(lb[r], ub[r]));
        whi = fmax(whi, fmax(lb[r], ub[r]));
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        wlo = fmin(wlo, __shfl_xor(wlo, o, 64));
        whi = fmax(whi, __shfl_xor(whi, o, 64));
      }
      exact = __all(exact);
    }
    // wave index as a scalar: the component addresses below are wave-uniform,
    // so the coefficients come in through scalar loads (SGPR operands)
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    LseCensus lcen{0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    int nvalid = 0;
#pragma unroll
    for (int r = 0; r < KR; ++r) nvalid += valid[r] ? 1 : 0;
    LseRange rg{0.0f, 0.0f, false, false};
    if constexpr (LSE) {
      if (A.lse_prune != 0) rg = lse_range<KR>(y, valid);
    }
    if constexpr (WT) WSTAMP(2);
#pragma unroll
    for (int mix = 0; mix < 2; ++mix) {
      const Coef *__restrict__ cm = mix ? ca : cb;
      const int K = mix ? ia.K : ib.K;
      if constexpr (LSE) {
        const bool prune = A.lse_prune != 0;
        // a wave without a valid candidate (the tail of a partial sort block:
        // li >= n_cand on every lane) has nothing to sum; its rows are never
        // read, so it keeps the empty sum instead of running an unpruned
        // loop over every block (lse_window: no range, no threshold)
        if (prune && !rg.any) {
          if constexpr (WT) {
#pragma unroll
            for (int r = 0; r < KR; ++r)
              sm.wpart[mix][wave][r][lane] = make_double2(lacc[mix][r].m, lacc[mix][r].s);
          }
          continue;
        }
        if (WT && prune && K <= kSmallMix) {
          // a small mixture (the good side): the direct exact two-pass sum
          lse_small<KR>(sm.small[mix], K, y, lacc[mix], sm.small_m[mix]);
          if constexpr (CENSUS) {
            lcen.total += (uint32_t)(K * nvalid);
            lcen.exec += (uint32_t)(K * nvalid);
          }
#pragma unroll
          for (int r = 0; r < KR; ++r)
            sm.wpart[mix][wave][r][lane] = make_double2(lacc[mix][r].m, lacc[mix][r].s);
          if (mix == 0) WSTAMP(3);
          continue;
        }
        LseWindow win{0.0f, 0.0f, -INFINITY};
        if (prune) win = lse_window<KR>(uniform_ptr(cm), mix ? ia.probe : ib.probe, K, y, valid, rg);
        if (WT && mix == 1) WSTAMP(4);
        // shifted single-exponent loop when the wave's window allows it
        // (lse_chunks_shifted's guard), else the exact per-group-lift loop
        // (mixtures of >= lse_shift_min components: fewer leave too few
        // terms near a wave-wide exponent for most waves to pass its guard)
        // (wave tiles: the shifted form over every chunk in one pass -- within
        // 3e-7 of the exact sum, large mixtures only, as for 8-wave tiles;
        // smaller ones keep the exact per-group lift below)
        constexpr int ST = WT ? 1 : kWaves;
        const int cw0 = WT ? 0 : wv;
        bool shifted = false;
        Stage stv{};
        stv.genv = A.coefe ? A.coefe + (mix ? sa : sb) * (A.kcap / kCoefBlock) : nullptr;
        // (the tightening pays where the pass-2 rounds are many: mixtures of
        // the range-search size -- config 4 78.7 against 79.5 ms without it;
        // at K ~ 1e3 it costs more than it prunes, config 5 474.7 vs 471.2)
        stv.tight = A.lse_tight && K >= kRangeMinK;
        if constexpr (STAGE) {
          stv.env = (LF4 *)(sm.stg.env + (mix ? nbb : 0));
          stv.c32 = (LC32 *)(sm.stg.c32 + (mix ? nbb : 0));
        }
        if (prune && A.lse_prune > 1 && K >= A.lse_shift_min && win.thr > -INFINITY) {
          // (the moment table of the launch's width: CoefM chunks or CoefM8 blocks)
          const int64_t ms = mix ? sa : sb;
          const MixInfo &mi = mix ? ia : ib;
          // (two-row wave tiles only: the one-row tiles of <= 2^18 candidates
          // -- config 3 -- are bound by per-wave latency, 0.5 live blocks per
          // wave, and the form's eligibility loads only add to it: 33 -> 71 us
          // per config-3 level-2 launch with it.  Never reading it there also
          // keeps fit_suggest, which writes the table only for two-row
          // steps, equal to fit + suggest)
          const CoefM *mt16 = (KR == 2 && MW == 16 && A.lse_mom == 16)
                                  ? A.coefm + ms * mom_stride(A.kcap) : nullptr;
          const CoefM8 *mt8 = (KR == 2 && MW == 8 && A.lse_mom == 8)
                                  ? A.coefm8 + ms * (A.kcap / kCoefBlock) : nullptr;
          const CoefM8 *mth = (KR == 2 && MW == 16 && A.lse_mom == 16 && A.lse_momh)
                                  ? A.coefmh + ms * mom_stride(A.kcap) : nullptr;
          if (STAGE && staged)  // (prune mode 3 only: the staged blocks are Coef32)
            shifted = lse_chunks_shifted<KR, CENSUS, ST, true, STAGE, MW>(
                uniform_ptr(cm), cm, cw0, K, y, valid, lacc[mix], win, nvalid, lcen,
                uniform_ptr32(A.coef32 + ms * (A.kcap / kCoefBlock)), mt16, mt8, stv,
                mi.env_cmax, mi.env_amin, mi.probe, mth);
          else if (A.lse_prune > 2)  // block-local fp32 pairs (Coef32), moment chunks (CoefM / 8)
            shifted = lse_chunks_shifted<KR, CENSUS, ST, true, false, MW>(
                uniform_ptr(cm), cm, cw0, K, y, valid, lacc[mix], win, nvalid, lcen,
                uniform_ptr32(A.coef32 + ms * (A.kcap / kCoefBlock)), mt16, mt8, stv,
                mi.env_cmax, mi.env_amin, mi.probe, mth);
          else
            shifted = lse_chunks_shifted<KR, CENSUS, ST>(uniform_ptr(cm), cm, cw0, K, y, valid,
                                                         lacc[mix], win, nvalid, lcen);
        }
        if (!shifted) {
          if (WT && prune && A.lse_prune > 1 && K >= A.lse_shift_min && win.thr > -INFINITY) WINFO(2, 1);
          if constexpr (WT) {
            // the exact per-group-lift loop over every chunk in order, one
            // pass (64 consecutive chunks per envelope round).  (Round 2 ran
            // it as 8 owner passes c = v (mod 8) merged in v order, the 8-wave
            // tile's association: bit-identical to that tile, but 8 envelope
            // rounds and lift states per mixture where a config-5 wave has
            // ~3 live blocks per pass.  Nothing compares the two tile shapes
            // bit for bit: batched, sharded and chunked runs of one draw take
            // the same tile shape.)
            if (STAGE && staged)
              lse_chunks<KR, CENSUS, 1, true, STAGE>(
                  uniform_ptr(cm), cm, 0, K, y, lacc[mix], prune, win, nvalid, lcen,
                  uniform_ptr32(A.coef32 + (mix ? sa : sb) * (A.kcap / kCoefBlock)), stv);
            else if (A.lse_prune > 2 || A.lse_f32)  // block-local fp32 (Coef32) where the block allows it
              lse_chunks<KR, CENSUS, 1, true>(
                  uniform_ptr(cm), cm, 0, K, y, lacc[mix], prune, win, nvalid, lcen,
                  uniform_ptr32(A.coef32 + (mix ? sa : sb) * (A.kcap / kCoefBlock)), stv);
            else
              lse_chunks<KR, CENSUS, 1>(uniform_ptr(cm), cm, 0, K, y, lacc[mix], prune, win,
                                        nvalid, lcen, nullptr, stv);
          } else if (A.lse_prune > 2 || A.lse_f32) {
            lse_chunks<KR, CENSUS, kWaves, true>(
                uniform_ptr(cm), cm, wv, K, y, lacc[mix], prune, win, nvalid, lcen,
                uniform_ptr32(A.coef32 + (mix ? sa : sb) * (A.kcap / kCoefBlock)));
          } else {
            lse_chunks<KR, CENSUS, kWaves>(uniform_ptr(cm), cm, wv, K, y, lacc[mix], prune, win,
                                           nvalid, lcen);
          }
        }
        if constexpr (WT) {
          // the wave's final sums of this mixture wait in its own LDS rows
          // (registers stay free for the next mixture's loop: no spills)
#pragma unroll
          for (int r = 0; r < KR; ++r)
            sm.wpart[mix][wave][r][lane] = make_double2(lacc[mix][r].m, lacc[mix][r].s);
          if (mix == 0) WSTAMP(3);
        }
      } else {
        erf_chunks<KR, LOGN, CENSUS>(uniform_ptr(cm), wv, K, ub, lb, valid, wlo, whi, exact, pacc[mix], cen);
      }
    }
    if (sink == 1.5e-30f) sm.merged[0][0][lane].y = sink;  // keeps the warm-up loads
    if constexpr (CENSUS && ERF) {
      unsigned long long c3[3] = {cen.total, cen.live, cen.exec};
#pragma unroll
      for (int q = 0; q < 3; ++q) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c3[q] += __shfl_xor(c3[q], o, 64);
        if (lane == 0) atomicAdd(A.census + q, c3[q]);
      }
    }
    if constexpr (CENSUS && LSE) {
      // nvalid is per lane: the per-lane sums add up to the wave's pairs
      unsigned long long c2[9] = {lcen.total, lcen.exec, lcen.shift, lcen.f32, lcen.retry,
                                  lcen.wide, lcen.mom, lcen.mom8, lcen.momh};
#pragma unroll
      for (int q = 0; q < 9; ++q) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c2[q] += __shfl_xor(c2[q], o, 64);
      }
      if (lane == 0) {
        atomicAdd(A.census + 3, c2[0]);
        atomicAdd(A.census + 4, c2[2]);
        atomicAdd(A.census + 5, c2[1]);
        atomicAdd(A.census + 6, c2[3]);
        atomicAdd(A.census + 7, c2[4]);
        atomicAdd(A.census + 8, c2[5]);
        atomicAdd(A.census + 9, c2[6]);
        atomicAdd(A.census + 10, c2[7]);
        atomicAdd(A.census + 11, c2[8]);
      }
    }
    if constexpr (!WT) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < KR; ++r)
        sm.wpart[q][wave][r][lane] = LSE ? make_double2(lacc[q][r].m, lacc[q][r].s)
                                         : make_double2(pacc[q][r], 0.0);
    __syncthreads();
    // wave 2r + q merges mixture q of candidate row r, in wave order
    if (wave < 2 * KR) {
      const int q = wave & 1, r = wave >> 1;
      double2 v0 = sm.wpart[q][0][r][lane];
      for (int w = 1; w < kWaves; ++w) {
        const double2 v = sm.wpart[q][w][r][lane];
        if constexpr (LSE) {
          LseAcc t{v0.x, v0.y};
          lse_merge(t, LseAcc{v.x, v.y});
          v0 = make_double2(t.m, t.s);
        } else {
          v0.x += v.x;
        }
      }
      sm.merged[q][r][lane] = v0;
    }
    __syncthreads();
    }
  }
  SSTAMP(1);
  if constexpr (WT) WSTAMP(1);
  if (!WT && wave != 0) return;

  // ---- finalize (every wave of a wave tile, wave 0 of an 8-wave tile):
  // lpdfs, EI, argmax (numpy semantics)
  double best_s = NAN, best_v = NAN;
  int64_t best_i = -1;
#ifdef TPE_REREAD
  int64_t best_li = -1;  // the bucketed slot of the lane's best (diagnostic build)
#endif
  if constexpr (LDRAW && (LAT || KIND == KIND_CAT)) {
    // Lookup scan (self-drawing lookups): the block owns a segment of
    // lookup_seg candidates; wave w walks its 256-candidate pieces w, w + 8,
    // ... in index order, drawing and scoring each candidate, and stops after
    // the first piece holding a candidate whose score is the slot's top
    // (top_s / NaN): no later candidate can beat it (numpy's argmax: the
    // largest score, the first index among equals, NaN first), and the
    // globally first top candidate lies in some piece t*, which wave t* mod 8
    // reaches before any piece of its own after it.  The records that result
    // are the ones the full scan gives.
    const double top = sm.top_s;
    const bool tnan = sm.top_nan != 0;
    const uint64_t seed = suggestion_seed(A, s);
    const double *mu_b = A.mmu + sb * A.kcap, *sg_b = A.msig + sb * A.kcap;
    const int64_t seg0 = (int64_t)tile * A.lookup_seg;
    const int64_t seg1 = min<int64_t>(seg0 + A.lookup_seg, A.n_cand);
    LatInfo L{};
    if constexpr (LAT) L = A.lat_info[hp];
    for (int64_t p0 = seg0 + (int64_t)wave * 64 * KR; p0 < seg1; p0 += (int64_t)kWaves * 64 * KR) {
      bool hit = false;
#pragma unroll
      for (int r = 0; r < KR; ++r) {
        const int64_t l = p0 + r * 64 + lane;
        if (l >= seg1) continue;
        const uint64_t gi = (uint64_t)(A.cand_begin + l);
        const double xv = draw_table_ool<kFuseTab>(A.hps + hp, ib.K, mu_b, sg_b, &sm.dt,
                                                   draw_block0(seed, gi, (uint32_t)hp), seed, gi,
                                                   (uint32_t)hp);
        double lpb, lpa;
        if constexpr (LAT) {
          const double J = rint(xv / H.q);
          const int64_t idx = fabs(J) < 4.0e15 ? (int64_t)J - L.j0 : -1;
          const bool in = idx >= 0 && idx < (int64_t)L.R;
          const double2 v = in ? A.lat[L.off + idx] : make_double2(NAN, NAN);
          lpb = v.x;
          lpa = v.y;
        } else {
          const int64_t c = (int64_t)xv;
          const bool in = (xv >= 0.0) && (c < ib.K) && ((double)c == xv);
          lpb = in ? reinterpret_cast<const double *>(cb)[coef_off(c, 0)] : NAN;
          lpa = in ? reinterpret_cast<const double *>(ca)[coef_off(c, 0)] : NAN;
        }
        const double sc = lpb - lpa;
        if (A.out_lb) A.out_lb[l] = lpb;
        if (A.out_la) A.out_la[l] = lpa;
        hit |= tnan ? (sc != sc) : (sc == top);
        take_better(best_s, best_v, best_i, sc, xv, (int64_t)gi);
      }
      if (__ballot(hit) && !A.out_lb && !A.out_la) break;
    }
  } else
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    // two-row log-sum-exp wave tiles recompute their slots from the scalar
    // wt0 and take their candidates back from LDS rather than keeping either
    // in registers through the component loops
    if constexpr (LSE && WT && KR > 1 && !TDRAW) {
      const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
      li[r] = wt0 + r * 64 + ln;
      valid[r] = li[r] < A.n_cand;
      asm volatile("" ::: "memory");  // (a reload, not the stored register)
      x[r] = sm.xs[wave][r][ln];
    }
    if (!valid[r]) continue;
    double lpb = NAN, lpa = NAN, sc;
#ifdef TPE_REREAD3
    // (diagnostic build dbg5: the winner's value taken from a plain re-read)
    if constexpr (LSE && WT) x[r] = cand[li[r]];
#endif
#ifdef TPE_REREAD2
    if constexpr (LSE && WT) {
      const double xp = cand[li[r]];
      const double xv = *(const volatile double *)&cand[li[r]];
      const bool dp = xp != x[r] && !(xp != xp && x[r] != x[r]);
      const bool dv = xv != x[r] && !(xv != xv && x[r] != x[r]);
      atomicAdd(&g_rr2_cnt[0], 1ull);
      if (dp) atomicAdd(&g_rr2_cnt[1], 1ull);
      if (dv) atomicAdd(&g_rr2_cnt[2], 1ull);
      if (dp || dv) {
        const unsigned long long e = atomicAdd(&g_rr2_cnt[3], 1ull);
        if (e < 64) {
          double *o = g_rr2_ex[e];
          o[0] = (double)li[r];
          o[1] = cpos ? (double)cpos[li[r]] : -1.0;
          o[2] = x[r];
          o[3] = xp;
          o[4] = xv;
          o[5] = (double)A.cand_begin;
          o[6] = (double)A.n_cand;
          o[7] = (double)hp;
        }
      }
    }
#endif
    if constexpr (LSE) {
      const double LN2 = 0.6931471805599453;
      const double2 b = WT ? sm.wpart[0][wave][r][lane] : sm.merged[0][r][lane];
      const double2 a = WT ? sm.wpart[1][wave][r][lane] : sm.merged[1][r][lane];
      if (A.out_lb || A.out_la) {  // the lpdfs themselves (operator / parity paths)
        lpb = (b.x == -INFINITY) ? NAN : (b.x + log2(b.y)) * LN2;
        lpa = (a.x == -INFINITY) ? NAN : (a.x + log2(a.y)) * LN2;
        if constexpr (LOGN) { const double lx = log(x[r]); lpb -= lx; lpa -= lx; }
        sc = lpb - lpa;
      } else {
        // EI only (the suggest): ((m_b - m_a) + log2(s_b / s_a)) ln 2 -- one
        // log2 instead of two, and LGMM's log x cancels; the exponents are
        // integers (exact difference), a NaN / -inf lpdf gives a NaN score
        sc = (b.x == -INFINITY || a.x == -INFINITY) ? NAN
                                                    : ((b.x - a.x) + fast_log2(b.y / a.y)) * LN2;
      }
    } else if constexpr (ERF) {
      lpb = log(sm.merged[0][r][lane].x) - ib.log_pacc;
      lpa = log(sm.merged[1][r][lane].x) - ia.log_pacc;
    } else if constexpr (LAT) {
      const LatInfo L = A.lat_info[hp];
      const double J = rint(x[r] / H.q);  // x == J * q for every drawn candidate
      const int64_t idx = fabs(J) < 4.0e15 ? (int64_t)J - L.j0 : -1;
      const bool in = idx >= 0 && idx < (int64_t)L.R;
      const double2 v = in ? A.lat[L.off + idx] : make_double2(NAN, NAN);
      lpb = v.x;
      lpa = v.y;
    } else {
      const int64_t c = (int64_t)x[r];
      const bool in = (x[r] >= 0.0) && (c < ib.K) && ((double)c == x[r]);
      lpb = in ? reinterpret_cast<const double *>(cb)[coef_off(c, 0)] : NAN;
      lpa = in ? reinterpret_cast<const double *>(ca)[coef_off(c, 0)] : NAN;
    }
    const int64_t lo = cpos ? (int64_t)cpos[li[r]] : li[r];  // original position
    if (A.out_lb) A.out_lb[lo] = lpb;
    if (A.out_la) A.out_la[lo] = lpa;
    if constexpr (!LSE) sc = lpb - lpa;
    const int64_t gi = A.cand_begin + lo;
#ifdef TPE_REREAD
    if (better(sc, gi, best_s, best_i)) {
      best_s = sc; best_v = x[r]; best_i = gi;
      best_li = li[r];
    }
#else
    take_better(best_s, best_v, best_i, sc, x[r], gi);
#endif
  }
#ifdef TPE_REREAD
  // the same reduction carrying the winner's bucketed slot, plus the slot a
  // re-read that does not carry it would take: lane 0's own best
  const int64_t dbg_own0 = __shfl(best_li, 0, 64);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double os = __shfl_xor(best_s, o, 64), ov = __shfl_xor(best_v, o, 64);
    const int64_t oi = __shfl_xor(best_i, o, 64), ol = __shfl_xor(best_li, o, 64);
    if (better(os, oi, best_s, best_i)) { best_s = os; best_v = ov; best_i = oi; best_li = ol; }
  }
#else
  wave_best(best_s, best_v, best_i);
#endif
  if constexpr (WT) WSTAMP(8);
  if constexpr (WT) {
    // the block's argmax over its wave tiles without a block barrier: each
    // wave leaves its record in LDS and arrives on the block's LDS counter;
    // the last to arrive merges the 8 records (better() orders ties by index,
    // so arrival order does not matter) and publishes the tile -- the other
    // waves exit at once instead of waiting for the block's slowest wave
    if (lane == 0) {
      sm.best_s[wave] = best_s;
      sm.best_v[wave] = best_v;
      sm.best_i[wave] = best_i;
#ifdef TPE_REREAD
      sm.best_li[wave] = best_li;
#endif
    }
    int last = 0;
    if (lane == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      last = __hip_atomic_fetch_add(&sm.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) ==
             (uint32_t)kWaves - 1;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    if (!__shfl(last, 0, 64)) return;
    const int w = lane < kWaves ? lane : 0;
    best_s = sm.best_s[w];
    best_v = sm.best_v[w];
    best_i = lane < kWaves ? sm.best_i[w] : -1;
#ifdef TPE_REREAD
    best_li = sm.best_li[w];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double os = __shfl_xor(best_s, o, 64), ov = __shfl_xor(best_v, o, 64);
      const int64_t oi = __shfl_xor(best_i, o, 64), ol = __shfl_xor(best_li, o, 64);
      if (better(os, oi, best_s, best_i)) { best_s = os; best_v = ov; best_i = oi; best_li = ol; }
    }
#else
    wave_best(best_s, best_v, best_i);
#endif
  }
  const int rix = tile, nrec = ntiles;
#ifdef TPE_REREAD
  if (lane == 0 && s == 0 && (int64_t)hp * A.pstride + rix < (1 << 20))
    g_tile_li[(int64_t)hp * A.pstride + rix][1] = dbg_own0;
#endif
  Partial *pbase = A.partial + ((int64_t)s * A.n_hp + hp) * A.pstride;
  int is_last = 0;
  if (lane == 0) {
    // publish the tile record write-through (8-B agent-scope stores = sc1),
    // drain, then take an arrival ticket; the last arriver reads every record
    // with sc1 loads.  No L2 write-back / L1 invalidate fences (the
    // MI355X_MICROARCH.md "valid forms" row: one lane stores and signals, the
    // workgroup whose add returned last loads, all stores and loads sc1).
    gu64 *rec = (gu64 *)(uintptr_t)(pbase + rix);
    __hip_atomic_store(rec + 0, dbits(best_s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(rec + 1, dbits(best_v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(rec + 2, (uint64_t)best_i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef TPE_REREAD
    __hip_atomic_store(rec + 3, (uint64_t)best_li, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    gu32 *tk = (gu32 *)(uintptr_t)(A.ticket + (int64_t)s * A.n_hp + hp);
    const uint32_t t = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = (t == (uint32_t)nrec - 1) ? 1 : 0;
    if (is_last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  is_last = __shfl(is_last, 0, 64);
  SSTAMP(2);
  if (!is_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the ticket
  double fs = NAN, fv = NAN;
  int64_t fi = -1;
#ifdef TPE_REREAD
  int64_t ft = -1;
#endif
  for (int i = lane; i < nrec; i += 64) {
    gu64 *rec = (gu64 *)(uintptr_t)(pbase + i);
    const double qs = bitsd(__hip_atomic_load(rec + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const double qv = bitsd(__hip_atomic_load(rec + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const int64_t qi = (int64_t)__hip_atomic_load(rec + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef TPE_REREAD
    if (better(qs, qi, fs, fi)) { fs = qs; fv = qv; fi = qi; ft = i; }
#else
    take_better(fs, fv, fi, qs, qv, qi);
#endif
  }
#ifdef TPE_REREAD
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double os = __shfl_xor(fs, o, 64), ov = __shfl_xor(fv, o, 64);
    const int64_t oi = __shfl_xor(fi, o, 64), ot = __shfl_xor(ft, o, 64);
    if (better(os, oi, fs, fi)) { fs = os; fv = ov; fi = oi; ft = ot; }
  }
  if (lane == 0) {
    Partial *rr = A.results + (int64_t)s * A.n_hp + hp;
    if (!(A.accumulate && better(rr->score, rr->index, fs, fi))) {
      *rr = Partial{fs, fv, fi, 1, 0};
      if (s == 0 && ft >= 0 && hp < 512) {
        // the winner's slot as carried through every reduction, and the
        // values a finalize-time re-read finds at each candidate address
        gu64 *rec = (gu64 *)(uintptr_t)(pbase + ft);
        const int64_t lt = (int64_t)__hip_atomic_load(rec + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int64_t tix = (int64_t)hp * A.pstride + ft;
        const int64_t lw0 = -1;  // (no block argmax since round 4: per-wave records)
        const int64_t lown = tix < (1 << 20) ? g_tile_li[tix][1] : -1;
        const volatile double *vc = cand;
        const int64_t pos = fi - A.cand_begin;
        double *d = g_reread[hp];
        d[0] = fv;
        d[1] = (double)fi;
        d[2] = (double)lt;
        d[3] = (lt >= 0 && lt < A.n_cand) ? vc[lt] : NAN;
        d[4] = (lt >= 0 && lt < A.n_cand && cpos) ? (double)cpos[lt] : NAN;
        d[5] = (pos >= 0 && pos < A.n_cand) ? vc[pos] : NAN;
        d[6] = (lw0 >= 0 && lw0 < A.n_cand) ? vc[lw0] : NAN;
        d[7] = (lown >= 0 && lown < A.n_cand) ? vc[lown] : NAN;
        d[8] = (double)A.cand_begin;
        d[9] = (double)ft;
        d[10] = (double)lw0;
        d[11] = (double)lown;
        d[12] = (double)(uintptr_t)cand;
        d[13] = (double)(uintptr_t)A.partial;
        d[14] = (double)A.n_cand;
        d[15] = (double)(uintptr_t)cpos;
        // the same lane's other candidate row (slot bit 64 of a two-row wave tile)
        const int64_t lr = lt ^ 64;
        d[16] = (lt >= 0 && lr < A.n_cand) ? vc[lr] : NAN;
      }
    }
  }
#else
  wave_best(fs, fv, fi);
  if (lane == 0) {
    Partial *rr = A.results + (int64_t)s * A.n_hp + hp;
    if (TDRAW && A.pub_flag) store_record_sc1(rr, Partial{fs, fv, fi, 1, 0});  // (never accumulating)
    else if (!(A.accumulate && better(rr->score, rr->index, fs, fi))) *rr = Partial{fs, fv, fi, 1, 0};
  }
#endif
  if constexpr (TDRAW) {  // (this slot's final record: one arrival)
    if (A.pub_flag) publish_arrive(A);
  }
}

#ifdef TPE_REREAD
}  // namespace tpe
extern "C" int tpe_debug_reread(double *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(tpe::g_reread), sizeof(tpe::g_reread)) == hipSuccess
             ? 0 : -5;
}
namespace tpe {
#endif

#ifdef TPE_REREAD2
}  // namespace tpe
extern "C" int tpe_debug_reread2(unsigned long long *cnt, double *ex, int reset) {
  if (reset) {
    unsigned long long z[4] = {0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(tpe::g_rr2_cnt), z, sizeof(z)) == hipSuccess ? 0 : -5;
  }
  if (hipMemcpyFromSymbol(cnt, HIP_SYMBOL(tpe::g_rr2_cnt), sizeof(tpe::g_rr2_cnt)) != hipSuccess) return -5;
  return hipMemcpyFromSymbol(ex, HIP_SYMBOL(tpe::g_rr2_ex), sizeof(tpe::g_rr2_ex)) == hipSuccess ? 0 : -5;
}
namespace tpe {
#endif

#ifdef TPE_STAMPS
}  // namespace tpe
extern "C" int tpe_debug_score_stamps(unsigned long long *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(tpe::g_score_stamps), sizeof(tpe::g_score_stamps)) ==
                 hipSuccess ? 0 : -5;
}
extern "C" int tpe_debug_wave_info(unsigned *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(tpe::g_wave_info), sizeof(tpe::g_wave_info)) ==
                 hipSuccess
             ? 0
             : -1;
}
extern "C" int tpe_debug_wave_info_clear() {
  static const unsigned zero[8192 * 8 * 4] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(tpe::g_wave_info), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
extern "C" int tpe_debug_wave_stamps(unsigned long long *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(tpe::g_wave_stamps), sizeof(tpe::g_wave_stamps)) ==
                 hipSuccess ? 0 : -5;
}
namespace tpe {
#endif

// One launch scores every hp of a level: a 1-D grid of blocks over the
// level's kind groups (ScoreArgs::grp_*), heaviest kind first, each group's
// slots cut into tiles of 64 * tile_rows(kind) candidates (1 row for the
// quantized kinds, whose per-pair cost is highest: smaller blocks spread their
// work over more CUs; 2 for log-sum-exp; 4 for categorical lookups).
// XCD-aware tile order inside a kind group.  Workgroups are dispatched to the
// 8 XCDs round-robin by flat id, each XCD with its own L2: local block l of a
// group of n (the first of which sits on XCD p) runs on XCD (p + l) % 8.
// Renumber so that every XCD takes one contiguous run of the group's tiles
// -- a slot's tiles then share one or two L2s (its coefficient tables are
// fetched by those only, not by all 8), and every XCD still gets the same
// share of the group's work.
__device__ __forceinline__ int xcd_local(int l, int n, int p) {
  const int q = (p + l) & 7;               // this block's XCD
  const int fq = (q - p + 8) & 7;          // the group's first local on XCD q
  int off = 0;
  for (int x = 0; x < q; ++x) {            // locals on the XCDs before q
    const int fx = (x - p + 8) & 7;
    off += fx < n ? (n - fx + 7) >> 3 : 0;
  }
  return off + ((l - fq) >> 3);
}

// Compact grids: the group's rows are its active slots in slot order; the
// first row's first tile also writes the "inactive" record of every slot of
// the group that has no rows (the record score_tile writes for an inactive
// slot of a full grid).
__device__ __forceinline__ void mark_inactive(const ScoreArgs &A, int s, int s0, int n) {
  if (threadIdx.x >= 64) return;
  Partial *res = A.results + (int64_t)s * A.n_hp;
  for (int i = (int)threadIdx.x; i < n; i += 64) {
    const int hp = A.level_hps[s0 + i];
    if (!hp_active(A.hps[hp], res, A.cond_parent, A.cond_branch)) res[hp] = Partial{NAN, NAN, -1, 0, 0};
  }
}

// The kinds a scoring kernel instantiates: every kind but the per-candidate
// erf ones, every kind, or only the wave-tile log-sum-exp kinds (levels of
// large draws whose every slot is one: a kernel with only their register
// allocation -- the combined one keeps the most any kind needs).
enum { kSetNoErf = 0, kSetAll = 1, kSetWave = 2, kSetWave1 = 3, kSetLookup = 4, kSetTiny = 5 };

template <int SET, bool CENSUS, typename SM, int MW = 16>
__device__ __forceinline__ void score_block(const ScoreArgs &A, SM &sm) {
  const int b = blockIdx.x;
  int g = 0;
  while (g + 1 < A.n_groups && b >= A.grp_block0[g + 1]) ++g;
  const int nt = A.grp_tiles[g];
  const int local = xcd_local(b - A.grp_block0[g], A.grp_block0[g + 1] - A.grp_block0[g],
                              (int)(((int64_t)blockIdx.y * gridDim.x + A.grp_block0[g]) & 7));
  int slot = A.grp_slot0[g] + local / nt;
  const int tile = local % nt;
  if (A.compact) {
    const int row = local / nt;
    if (row == 0 && tile == 0) mark_inactive(A, blockIdx.y, A.grp_slot0[g], A.grp_slots[g]);
    slot = active_slot(A, blockIdx.y, A.grp_slot0[g], A.grp_slots[g], row);
    if (slot < 0) return;
  }
  const bool known = A.compact != 0;
  if constexpr (SET == kSetWave) {
    if (A.grp_kind[g] == KIND_LSE_LW)
      score_tile<KIND_LSE_LW, CENSUS, SM, false, false, MW>(A, sm, slot, tile, nt, known);
    else score_tile<KIND_LSE_GW, CENSUS, SM, false, false, MW>(A, sm, slot, tile, nt, known);
    return;
  } else if constexpr (SET == kSetLookup) {
    if (A.grp_kind[g] == KIND_LAT) score_tile<KIND_LAT, CENSUS, SM, true>(A, sm, slot, tile, nt, known);
    else score_tile<KIND_CAT, CENSUS, SM, true>(A, sm, slot, tile, nt, known);
    return;
  } else if constexpr (SET == kSetTiny) {
    // (tiny unsorted draws of levels without lattice or per-candidate erf
    // slots: the log-sum-exp kinds and categoricals, each tile drawing)
    switch (A.grp_kind[g]) {
      case KIND_LSE_G: score_tile<KIND_LSE_G, CENSUS, SM, false, true>(A, sm, slot, tile, nt, known); break;
      case KIND_LSE_L: score_tile<KIND_LSE_L, CENSUS, SM, false, true>(A, sm, slot, tile, nt, known); break;
      case KIND_LSE_G1: score_tile<KIND_LSE_G1, CENSUS, SM, false, true>(A, sm, slot, tile, nt, known); break;
      case KIND_LSE_L1: score_tile<KIND_LSE_L1, CENSUS, SM, false, true>(A, sm, slot, tile, nt, known); break;
      default: score_tile<KIND_CAT, CENSUS, SM, false, true>(A, sm, slot, tile, nt, known); break;
    }
    return;
  } else if constexpr (SET == kSetWave1) {
    if (A.grp_kind[g] == KIND_LSE_LW1)
      score_tile<KIND_LSE_LW1, CENSUS, SM, false, false, MW>(A, sm, slot, tile, nt, known);
    else score_tile<KIND_LSE_GW1, CENSUS, SM, false, false, MW>(A, sm, slot, tile, nt, known);
    return;
  } else {
    switch (A.grp_kind[g]) {
      case KIND_LSE_G: score_tile<KIND_LSE_G, CENSUS, SM>(A, sm, slot, tile, nt, known); break;
      case KIND_LSE_L: score_tile<KIND_LSE_L, CENSUS, SM>(A, sm, slot, tile, nt, known); break;
      case KIND_LSE_G1: score_tile<KIND_LSE_G1, CENSUS, SM>(A, sm, slot, tile, nt, known); break;
      case KIND_LSE_L1: score_tile<KIND_LSE_L1, CENSUS, SM>(A, sm, slot, tile, nt, known); break;
      case KIND_LSE_GW: score_tile<KIND_LSE_GW, CENSUS, SM>(A, sm, slot, tile, nt, known); break;
      case KIND_LSE_LW: score_tile<KIND_LSE_LW, CENSUS, SM>(A, sm, slot, tile, nt, known); break;
      case KIND_ERF_G:
        if constexpr (SET == kSetAll) score_tile<KIND_ERF_G, CENSUS, SM>(A, sm, slot, tile, nt, known);
        break;
      case KIND_ERF_L:
        if constexpr (SET == kSetAll) score_tile<KIND_ERF_L, CENSUS, SM>(A, sm, slot, tile, nt, known);
        break;
      case KIND_LAT: score_tile<KIND_LAT, CENSUS, SM>(A, sm, slot, tile, nt, known); break;
      default: score_tile<KIND_CAT, CENSUS, SM>(A, sm, slot, tile, nt, known); break;
    }
  }
}

template <bool ERFK, bool CENSUS>
__global__ __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(6)))
void k_score(ScoreArgs A) {
  __shared__ ScoreSmem sm;
  score_block<ERFK ? kSetAll : kSetNoErf, CENSUS>(A, sm);
}

#ifndef TPE_WAVE_EU
#define TPE_WAVE_EU 6
#endif
// MW: the moment width (16: CoefM chunks, the config-4 regime; 8: CoefM8
// blocks, mixtures of ~1e3 components) -- one instantiation per width, so
// each keeps its own register allocation
template <bool CENSUS, int MW>
__global__ __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(TPE_WAVE_EU)))
void k_score_wave(ScoreArgs A) {
  __shared__ ScoreSmem sm;
  score_block<kSetWave, CENSUS, ScoreSmem, MW>(A, sm);
}
// the one-row wave tiles (KIND_LSE_GW1 / LW1) in a kernel of their own: the
// two-row kernel's register allocation is left as it is
template <bool CENSUS, int MW>
__global__ __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(TPE_WAVE_EU)))
void k_score_wave1(ScoreArgs A) {
  __shared__ ScoreSmem1 sm;
  score_block<kSetWave1, CENSUS, ScoreSmem1, MW>(A, sm);
}

// tiny unsorted draws whose tiles draw their own candidates (tile_draw), in a
// kernel of their own (the draw's call out of k_score's register allocation)
template <bool CENSUS>
__global__ __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(4)))
void k_score_tdraw(ScoreArgs A) {
  __shared__ ScoreSmem sm;
  score_block<kSetTiny, CENSUS>(A, sm);
}

// the lookup tiles (categorical, value lattice) that draw their own
// candidates (ScoreArgs::lookup_draw) in a kernel of their own: the table
// draw's call is kept out of the combined kernel's register allocation
template <bool CENSUS>
__global__ __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(4)))
void k_score_lookup(ScoreArgs A) {
  __shared__ ScoreSmemT<1> sm;
  score_block<kSetLookup, CENSUS>(A, sm);
}

// Value-lattice scoring of the bounded quantized hps (KIND_LAT).  A drawn
// candidate of such an hp is one of R lattice values j * q, and its lpdf
// depends on that value only, so both lpdfs are evaluated once per lattice
// point and shared by every candidate and every suggestion of the call.
// One block per (point, hp): lane t takes component 16 * c + (t & 15) of
// chunk c = t / 16 of the below mixture, then of the above mixture; a chunk is
// summed in component order by its 16 lanes, and thread 0 / 1 adds the chunk
// sums of the below / above mixture in erf_chunks' canonical order (chunk c
// to the total of "wave" c mod kWaves, totals in wave order), so a lattice
// lpdf is bit-identical to the per-candidate kernel's for that value.
// pc + v[lane + 1] + v[lane + 2] + ... + v[lane + I] in that order, the
// neighbours read with DPP row_shl (within the lane's 16-lane row; no LDS
// round trip per term)
template <int I>
struct RowShlSum {
  static __device__ __forceinline__ double run(double pc, double v) {
    static_assert(I < 16, "row_shl reaches 15 lanes");
    return RowShlSum<I - 1>::run(pc, v) + dppd<0x100 + I>(v);
  }
};
template <>
struct RowShlSum<0> {
  static __device__ __forceinline__ double run(double pc, double) { return pc; }
};

template <bool LOGN>
__device__ __forceinline__ void lattice_point(const ScoreArgs &A, const tpe_hp &H, int hp,
                                              const LatInfo &L, int64_t pt, double *csum,
                                              double2 *__restrict__ out) {
#pragma clang fp contract(off)
  const double x = (double)(L.j0 + pt) * H.q;
  double ub, lb;
  quant_bounds<LOGN>(H, x, ub, lb);
  const int64_t sb = 2 * (int64_t)hp;
  const MixInfo ib = A.info[sb], ia = A.info[sb + 1];
  const int ncb = (ib.K + kChunk - 1) / kChunk, nca = (ia.K + kChunk - 1) / kChunk;
  const int nch = ncb + nca;
  const double *cb = reinterpret_cast<const double *>(A.coef + sb * A.kcap);
  const double *ca = reinterpret_cast<const double *>(A.coef + (sb + 1) * A.kcap);
  const int j = threadIdx.x & (kChunk - 1);
  // kLatU rounds of the block at a time: every coefficient load of the batch
  // is issued before the first erf, so one memory latency covers kLatU rounds
  constexpr int kLatU = 4;
  for (int t0 = 0; t0 < kChunk * nch; t0 += kLatU * (int)blockDim.x) {
    double cx[kLatU], cy[kLatU], cw[kLatU];
    bool ok[kLatU];
#pragma unroll
    for (int u = 0; u < kLatU; ++u) {
      const int c = (t0 + u * (int)blockDim.x + (int)threadIdx.x) / kChunk;
      const bool above = c >= ncb;
      const int k = (above ? c - ncb : c) * kChunk + j;
      ok[u] = c < nch && k < (above ? ia.K : ib.K);
      const double *cs = above ? ca : cb;
      cx[u] = ok[u] ? cs[coef_off(k, 0)] : 0.0;
      cy[u] = ok[u] ? cs[coef_off(k, 1)] : 0.0;
      cw[u] = ok[u] ? cs[coef_off(k, 2)] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kLatU; ++u) {
      const int c = (t0 + u * (int)blockDim.x + (int)threadIdx.x) / kChunk;
      double inc = 0.0;
      if (ok[u]) {
        const double zu = (ub - cx[u]) * cy[u], zl = (lb - cx[u]) * cy[u];
        if (!erf_dead(zu, zl)) inc = erf_term<LOGN>(zu, zl, cw[u]);
      }
      // the chunk in component order, summed in its first lane: lane seg
      // reads lane seg + i of its 16-lane DPP row (row_shl:i)
      const double pc = RowShlSum<kChunk - 1>::run(0.0 + inc, inc);
      if (j == 0 && c < nch) csum[c] = pc;
    }
  }
  __syncthreads();
  // the "wave" totals: lane w (mod kWaves) of the first 2 * kWaves threads sums
  // the chunks c = w, w + kWaves, ... of one mixture in order; lanes 0 / kWaves
  // add the totals in wave order (erf_chunks / score_tile's merge)
  const int t = threadIdx.x;
  double sw = 0.0;
  if (t < 2 * kWaves) {
    const int above = t / kWaves, w = t % kWaves;
    const int c0 = above ? ncb : 0, n = above ? nca : ncb;
    for (int c = w; c < n; c += kWaves) sw += csum[c0 + c];
  }
  static_assert(kWaves == 8, "the wave totals of a mixture sit in 8 lanes of one DPP row");
  const double tot = RowShlSum<kWaves - 1>::run(sw, sw);
  if (t == 0 || t == kWaves) {
    const int above = t / kWaves;
    const double lp = log(tot) - (above ? ia.log_pacc : ib.log_pacc);
    double *o = reinterpret_cast<double *>(out + L.off + pt);
    o[above] = lp;
  }
}

// grid (lattice point, job): the jobs (hp descriptor + lattice) travel in the
// kernel arguments, so a block's first memory accesses are its coefficients
// DRAW: rows y >= J.n_jobs draw the level's candidates instead (k_draw<true>'s
// blocks, table of <= kFuseTab components in the same dynamic LDS)
template <bool DRAW>
__global__ __launch_bounds__(kLatThreads) void k_lattice(ScoreArgs A, LatJobs J,
                                                          double2 *__restrict__ out) {
  extern __shared__ double csum[];  // [chunks of both mixtures]
  if constexpr (DRAW) {
    if ((int)blockIdx.y >= J.n_jobs) {
      const int d = ((int)blockIdx.y - J.n_jobs) * (int)gridDim.x + (int)blockIdx.x;
      if (d >= J.draw_blocks) return;
      const int per_s = J.draw_gx * A.slot_rows;
      draw_block<kFuseTab>(A, d % J.draw_gx, (d % per_s) / J.draw_gx, d / per_s,
                           *reinterpret_cast<DrawTableT<kFuseTab> *>(csum),
                           (int64_t)J.draw_gx * blockDim.x);
      return;
    }
  }
  const int64_t pt = blockIdx.x;
  if (J.compact) {
    const int slot = active_slot_any(A, A.n_suggest, 0, J.n_lat, blockIdx.y);
    if (slot < 0) return;
    const int hp = A.level_hps[slot];
    const LatInfo L = A.lat_info[hp];
    if (pt >= L.R) return;
    const tpe_hp H = A.hps[hp];
    if (H.family == TPE_LGMM) lattice_point<true>(A, H, hp, L, pt, csum, out);
    else lattice_point<false>(A, H, hp, L, pt, csum, out);
    return;
  }
  const LatJob &jb = J.job[blockIdx.y];
  if (pt >= jb.L.R) return;
  if (jb.H.family == TPE_LGMM) lattice_point<true>(A, jb.H, jb.hp, jb.L, pt, csum, out);
  else lattice_point<false>(A, jb.H, jb.hp, jb.L, pt, csum, out);
}

hipError_t launch_lattice(const ScoreArgs &a, const int32_t *hps_of_level, const tpe_hp *hps,
                          const LatInfo *lat, int32_t n_lat, double2 *lat_out, hipStream_t st,
                          int32_t lat_rows) {
  const int64_t nch = 2 * ((a.kcap + kChunk - 1) / kChunk);
  if (nch > kLatChunks) return hipErrorInvalidValue;
  if (lat_rows > 0 && lat_rows < n_lat) {
    // compact: one launch, rows = the most lattice hps active in some suggestion
    LatJobs J{};
    int64_t rmax = 0;
    for (int32_t i = 0; i < n_lat; ++i) rmax = std::max<int64_t>(rmax, lat[hps_of_level[i]].R);
    if (rmax > kLatMaxR) return hipErrorInvalidValue;
    if (rmax <= 0) return hipSuccess;
    J.n_jobs = lat_rows;
    J.compact = 1;
    J.n_lat = n_lat;
    k_lattice<false><<<dim3((unsigned)rmax, (unsigned)lat_rows), kLatThreads,
                       (size_t)nch * sizeof(double), st>>>(a, J, lat_out);
    return hipGetLastError();
  }
  for (int32_t i0 = 0; i0 < n_lat; i0 += kLatJobs) {
    LatJobs J{};
    int64_t rmax = 0;
    const int32_t n = std::min<int32_t>(kLatJobs, n_lat - i0);
    for (int32_t i = 0; i < n; ++i) {
      const int32_t hp = hps_of_level[i0 + i];
      J.job[i].H = hps[hp];
      J.job[i].L = lat[hp];
      J.job[i].hp = hp;
      rmax = std::max<int64_t>(rmax, lat[hp].R);
    }
    if (rmax > kLatMaxR) return hipErrorInvalidValue;
    if (rmax <= 0) continue;
    J.n_jobs = n;
    k_lattice<false><<<dim3((unsigned)rmax, (unsigned)n), kLatThreads,
                       (size_t)nch * sizeof(double), st>>>(a, J, lat_out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

const void *lattice_draw_kernel_fn() { return reinterpret_cast<const void *>(&k_lattice<true>); }

hipError_t launch_lattice_draw(const ScoreArgs &a, const int32_t *hps_of_level, const tpe_hp *hps,
                               const LatInfo *lat, int32_t n_lat, double2 *lat_out,
                               hipStream_t st, int32_t lat_rows) {
  static_assert(kLatThreads == 256, "draw rows run k_draw's 256-thread blocks");
  const int64_t nch = 2 * ((a.kcap + kChunk - 1) / kChunk);
  if (nch > kLatChunks || n_lat < 1 || n_lat > kLatJobs || a.n_cand <= 0) return hipErrorInvalidValue;
  LatJobs J{};
  int64_t rmax = 0;
  for (int32_t i = 0; i < n_lat; ++i) {
    const int32_t hp = hps_of_level[i];
    J.job[i].H = hps[hp];
    J.job[i].L = lat[hp];
    J.job[i].hp = hp;
    rmax = std::max<int64_t>(rmax, lat[hp].R);
  }
  if (rmax > kLatMaxR || rmax <= 0) return hipErrorInvalidValue;
  const int64_t gx = (a.n_cand + kLatThreads - 1) / kLatThreads;
  const int64_t draws = gx * a.slot_rows * a.n_suggest;
  if (draws > ((int64_t)1 << 30)) return hipErrorInvalidValue;
  J.n_jobs = n_lat;
  if (lat_rows > 0 && lat_rows < n_lat) {  // compact lattice rows (launch_lattice)
    J.n_jobs = lat_rows;
    J.compact = 1;
    J.n_lat = n_lat;
  }
  J.draw_gx = (int32_t)gx;
  J.draw_blocks = (int32_t)draws;
  const int64_t rows = (draws + rmax - 1) / rmax;
  const size_t lds = std::max<size_t>((size_t)nch * sizeof(double), sizeof(DrawTableT<kFuseTab>));
  k_lattice<true><<<dim3((unsigned)rmax, (unsigned)(J.n_jobs + rows)), kLatThreads, lds, st>>>(
      a, J, lat_out);
  return hipGetLastError();
}

// the groups of a (kind) subset of a launch's grid, renumbered
// the launch class of a kind group: 0 wave-tile log-sum-exp (k_score_wave /
// k_score_wave1), 1 lookups drawing their own candidates (k_score_lookup),
// 2 the rest (k_score)
static int group_class(const ScoreArgs &a, int kind) {
  if (kind_wave_lse(kind)) return 0;
  if (a.lookup_draw && (kind == KIND_CAT || kind == KIND_LAT)) return 1;
  return 2;
}
static ScoreArgs select_groups(const ScoreArgs &a, int cls) {
  ScoreArgs b = a;
  b.n_groups = 0;
  int32_t blocks = 0;
  for (int i = 0; i < a.n_groups; ++i) {
    if (group_class(a, a.grp_kind[i]) != cls) continue;
    const int j = b.n_groups++;
    b.grp_kind[j] = a.grp_kind[i];
    b.grp_slot0[j] = a.grp_slot0[i];
    b.grp_tiles[j] = a.grp_tiles[i];
    b.grp_slots[j] = a.grp_slots[i];
    b.grp_block0[j] = blocks;
    blocks += a.grp_block0[i + 1] - a.grp_block0[i];
  }
  b.grp_block0[b.n_groups] = blocks;
  return b;
}

// one launch of a single class's groups
static hipError_t launch_class(const ScoreArgs &a, int cls, bool has_erf, hipStream_t st) {
  if (a.n_groups <= 0) return hipSuccess;
  const int blocks = a.grp_block0[a.n_groups];
  if (blocks <= 0) return hipSuccess;
  const dim3 g((unsigned)blocks, a.n_suggest);
  bool one_row = false;
  for (int i = 0; i < a.n_groups; ++i)
    one_row |= a.grp_kind[i] == KIND_LSE_GW1 || a.grp_kind[i] == KIND_LSE_LW1;
  const bool m8 = a.lse_mom == 8;
  if (cls == 0 && one_row) {
    if (m8) {
      if (a.census) k_score_wave1<true, 8><<<g, kWaves * 64, 0, st>>>(a);
      else k_score_wave1<false, 8><<<g, kWaves * 64, 0, st>>>(a);
    } else {
      if (a.census) k_score_wave1<true, 16><<<g, kWaves * 64, 0, st>>>(a);
      else k_score_wave1<false, 16><<<g, kWaves * 64, 0, st>>>(a);
    }
  } else if (cls == 0) {
    if (m8) {
      if (a.census) k_score_wave<true, 8><<<g, kWaves * 64, 0, st>>>(a);
      else k_score_wave<false, 8><<<g, kWaves * 64, 0, st>>>(a);
    } else {
      if (a.census) k_score_wave<true, 16><<<g, kWaves * 64, 0, st>>>(a);
      else k_score_wave<false, 16><<<g, kWaves * 64, 0, st>>>(a);
    }
  } else if (cls == 1) {
    // one block per segment of a slot (the scan's early exit works within a
    // segment) instead of one per 2048-candidate tile: segments of whole
    // 2048-candidate pieces, as many as keep ~4 blocks per CU busy (a launch
    // of few rows keeps the tiles' parallelism; config 5's 80 rows per launch
    // get ~13 segments of ~8e4 candidates per slot)
    ScoreArgs b = a;
    int64_t rows_all = 0;
    for (int i = 0; i < a.n_groups; ++i)
      rows_all += (a.grp_block0[i + 1] - a.grp_block0[i]) / a.grp_tiles[i];
    const int64_t pieces = (a.n_cand + 2047) / 2048;
    const int64_t want = std::max<int64_t>(1, (4 * kNumCUs) / std::max<int64_t>(1, rows_all * a.n_suggest));
    const int64_t nseg0 = std::min<int64_t>(pieces, want);
    b.lookup_seg = (pieces + nseg0 - 1) / nseg0 * 2048;
    const int32_t nseg = (int32_t)((a.n_cand + b.lookup_seg - 1) / b.lookup_seg);
    int32_t blk = 0;
    for (int i = 0; i < b.n_groups; ++i) {
      const int32_t rows = (a.grp_block0[i + 1] - a.grp_block0[i]) / a.grp_tiles[i];
      b.grp_block0[i] = blk;
      b.grp_tiles[i] = nseg;
      blk += rows * nseg;
    }
    b.grp_block0[b.n_groups] = blk;
    const dim3 gl((unsigned)blk, a.n_suggest);
    if (b.census) k_score_lookup<true><<<gl, kWaves * 64, 0, st>>>(b);
    else k_score_lookup<false><<<gl, kWaves * 64, 0, st>>>(b);
  } else if (has_erf) {
    if (a.census) k_score<true, true><<<g, kWaves * 64, 0, st>>>(a);
    else k_score<true, false><<<g, kWaves * 64, 0, st>>>(a);
  } else {
    if (a.census) k_score<false, true><<<g, kWaves * 64, 0, st>>>(a);
    else k_score<false, false><<<g, kWaves * 64, 0, st>>>(a);
  }
  return hipGetLastError();
}

int score_classes(const ScoreArgs &a) {
  int m = 0;
  for (int i = 0; i < a.n_groups; ++i) m |= 1 << group_class(a, a.grp_kind[i]);
  return m;
}

hipError_t launch_score(const ScoreArgs &a, bool has_erf, hipStream_t st, hipStream_t side,
                        hipEvent_t ev_fork, hipEvent_t ev_join, int classes) {
  if (a.n_groups <= 0 || a.n_suggest <= 0) return hipSuccess;
  if (a.grp_block0[a.n_groups] <= 0) return hipSuccess;
  if (a.tile_draw) {  // (every group: the host takes this path for such levels only)
    const dim3 g((unsigned)a.grp_block0[a.n_groups], a.n_suggest);
    if (a.census) k_score_tdraw<true><<<g, kWaves * 64, 0, st>>>(a);
    else k_score_tdraw<false><<<g, kWaves * 64, 0, st>>>(a);
    return hipGetLastError();
  }
  bool has[3] = {false, false, false};
  for (int i = 0; i < a.n_groups; ++i) has[group_class(a, a.grp_kind[i])] = true;
  for (int c = 0; c < 3; ++c) has[c] = has[c] && ((classes >> c) & 1);
  const int ncls = (int)has[0] + (int)has[1] + (int)has[2];
  if (ncls == 0) return hipSuccess;
  if (ncls == 1) {
    const int c = has[0] ? 0 : has[1] ? 1 : 2;
    return launch_class(score_classes(a) == (1 << c) ? a : select_groups(a, c), c, has_erf, st);
  }
  // a level of several classes: one launch per class.  The wave-tile
  // log-sum-exp launch on st; the others in order on st, or beside it on the
  // side stream when one is given (TPE_SIDE_STREAMS)
  hipError_t e;
  const bool fork = side && has[0];
  if (fork) {
    if ((e = hipEventRecord(ev_fork, st)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(side, ev_fork, 0)) != hipSuccess) return e;
  }
  hipStream_t so = fork ? side : st;
  hipError_t eo = hipSuccess;
  for (int c = 1; c <= 2 && eo == hipSuccess; ++c)
    if (has[c]) eo = launch_class(select_groups(a, c), c, has_erf, so);
  // (once forked, the side stream is joined back on every path)
  const hipError_t ej = fork ? hipEventRecord(ev_join, side) : hipSuccess;
  const hipError_t ew = has[0] ? launch_class(select_groups(a, 0), 0, false, st) : hipSuccess;
  if (fork && ej == hipSuccess && (e = hipStreamWaitEvent(st, ev_join, 0)) != hipSuccess) return e;
  return eo != hipSuccess ? eo : ej != hipSuccess ? ej : ew;
}

}  // namespace tpe
