// tpe_fit.hip -- good/bad split, adaptive Parzen fit / categorical posterior
// and per-component lpdf constants of every (hp, side) slot, gfx950.
//
// Reference (pminervini/hyperopt, hyperopt/tpe.py):
//   ap_filter_trials            tpe.py:613-641   split_threshold / gather
//   linear_forgetting_weights   tpe.py:381-394   lf_weight
//   adaptive_parzen_normal      tpe.py:398-475   fit_continuous
//   ap_categorical_sampler      tpe.py:573-607   fit_categorical
//   GMM1_lpdf / LGMM1_lpdf      tpe.py:104-166, 259-301: per-component
//                               constants + p_accept (prep_slot)
//
// One 1024-thread block per (hp, side).  Everything a block touches more than
// once lives in LDS (160 KB on gfx950): the sort keys and permutations, and
// for K <= kMixLds the whole mixture until the final copy-out.  The sort is a
// stable LSD radix sort of the permutation over 8-bit digits of a 64-bit key
// (digits that are equal for every key are skipped), with wave-level ballot
// ranking, so its cost is a few passes of ~2 barriers each instead of the
// O(log^2 n) barrier stages of a bitonic network.  Every floating-point
// operation that reaches the outputs is the reference's own, in its order
// (numpy pairwise summation included), so the fit is bit-identical to the
// reference whenever the reference's argsort has no ties to reorder.
#include <math.h>

#include "tpe_device.hpp"

#pragma clang fp contract(off)

namespace tpe {

// k_fit runs once per CU per suggest, so its cost is dominated by first-time
// instruction fetch: helpers called several times per block are kept out of
// line (NOINLINE) so later calls run from a warm instruction cache.
#define NOINLINE __attribute__((noinline))

#ifdef TPE_STAMPS
// diagnostic build only (make dbg; tools/fit_stamps.py): per-slot phase
// timestamps of k_fit, wall clock (100 MHz)
__device__ unsigned long long g_stamps[512][48];  // [0, 16) phases, [16, 48) sub-phases
#define STAMP(ph)                                                             \
  do {                                                                        \
    if (threadIdx.x == 0 && blockIdx.z == 0)                                  \
      g_stamps[(2 * blockIdx.x + blockIdx.y) & 511][ph] = wall_clock64();     \
  } while (0)
#else
#define STAMP(ph) do {} while (0)
#endif

constexpr int kFitWaves = kFitThreads / 64;  // 16
constexpr int kSortCap = 10000;              // elements sorted in LDS (u16 positions)
constexpr int kMixLds = 4097;                // K kept in LDS until copy-out (m <= 4096)
constexpr int kMixStride = 4104;             // doubles per LDS mixture array
constexpr int kDigits = 256;
constexpr int kPreN = 12 * kFitThreads;      // histories whose values k_fit prefetches

// dynamic LDS map (bytes)
constexpr int kOffKeys = 0;                               // u64 [kSortCap]
constexpr int kOffPosA = kOffKeys + 8 * kSortCap;         // u16 [kSortCap]
constexpr int kOffPosB = kOffPosA + 2 * kSortCap;         // u16 [kSortCap]
constexpr int kOffCnt = kOffPosB + 2 * kSortCap;          // u32 [256][16]
constexpr int kOffRun = kOffCnt + 4 * kDigits * kFitWaves;  // u32 [16][256]
constexpr int kFitLds = kOffRun + 4 * kDigits * kFitWaves;  // 155,648 B
static_assert(4 * 8 * kMixStride <= kFitLds, "LDS mixture arrays");

// numpy pairwise_sum tree of one chunk (n <= 8192): a node of length m > 128
// splits into m2 = floor(m/2) rounded down to a multiple of 8 and m - m2, a
// node of <= 128 is a leaf.  A child is at most half its parent + 8, so the
// tree is at most 7 levels deep and its nodes fit a 1-based heap of 256 ids
// (children of id: 2 id, 2 id + 1).  Any thread finds a node's range from its
// id by descending from the root, so no tree has to be built first.
constexpr int kNpHeap = 256;

struct NpNode {
  int lo, n;  // n = 0: no such node (an ancestor is a leaf)
};
__device__ __forceinline__ NpNode np_node(int len, int id) {
  const int depth = 31 - __builtin_clz((unsigned)id);
  int lo = 0, n = len;
  for (int b = depth - 1; b >= 0; --b) {
    if (n <= 128) return NpNode{0, 0};
    int n2 = n / 2;
    n2 -= n2 % 8;
    if ((id >> b) & 1) { lo += n2; n -= n2; }
    else n = n2;
  }
  return NpNode{lo, n};
}

constexpr int kGatherRows = 12;  // trials per thread in one gather chunk (12288 per block)
struct GatherEx {  // one wave's share of a gather chunk
  int nlt, pad;
  uint64_t kand, kor;
};

struct FitShared {
  GatherEx gx[1][kFitWaves];
  int gcnt[kGatherRows][kFitWaves];  // selected trials per (row, wave) of a gather chunk
  int gbase[kGatherRows][kFitWaves]; // their exclusive prefix in (row, wave) order
  double val[2][kNpHeap];    // pairwise-sum node values by heap id (two arrays at once)
  uint64_t rk[2][kFitWaves];
  uint32_t rp[2][kFitWaves];
  uint64_t vand[kFitWaves], vor[kFitWaves];
  int wsum[kFitWaves + 1];
  int isum[kFitWaves];
  float envc[kFitWaves], enva[kFitWaves];  // envelope extremes (envelope_extremes)
  int m, nlt;
};

// ------------------------------------------------------------------------
// wave / block primitives
// ------------------------------------------------------------------------
__device__ __forceinline__ void wave_min_kp(uint64_t &k, uint32_t &p) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t ok = __shfl_xor(k, o, 64);
    const uint32_t op = __shfl_xor(p, o, 64);
    if (kp_less(ok, op, k, p)) { k = ok; p = op; }
  }
}

__device__ __forceinline__ uint32_t wave_excl_scan_u32(uint32_t v) {
  return (uint32_t)wave_incl_scan((int)v) - v;
}

// block-wide exclusive scan of small ints: (exclusive prefix, total) -- by
// value, in registers (an out-reference of a call lives on the scratch stack)
__device__ __forceinline__ int2 block_excl_scan(int v, int *wsum) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int x = wave_incl_scan(v);
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int before = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kFitWaves; ++i) {
    const int s = wsum[i];
    before += (i < w) ? s : 0;
    tot += s;
  }
  __syncthreads();
  return make_int2(before + x - v, tot);
}

// lanes of this wave whose 8-bit digit equals mine (among lanes with v set)
__device__ __forceinline__ uint64_t match8(uint32_t d, bool v) {
  uint64_t m = __ballot(v);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const bool s = (d >> b) & 1u;
    const uint64_t bb = __ballot(s);
    m &= s ? bb : ~bb;
  }
  return m;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// ------------------------------------------------------------------------
// stable LSD radix sort of a permutation (ascending key, ties keep the
// initial order = position).  keys[] indexed by element id; a/b: LDS (u16)
// or global (u32) permutations; cnt/run: 16 KB each in LDS.  Returns the
// buffer holding the sorted permutation.
// ------------------------------------------------------------------------
template <typename PosT>
__device__ NOINLINE void radix_pass(const uint64_t *keys, const PosT *a, PosT *b, int n, int shift,
                           uint32_t *cnt, uint32_t *run) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int per = ((n + kFitWaves * 64 - 1) / (kFitWaves * 64)) * 64;  // slots per wave
  const int r0 = w * per, r1 = min(n, r0 + per);
  uint32_t *mycnt = cnt + w * kDigits;  // wave-private row while counting
  for (int d = lane; d < kDigits; d += 64) mycnt[d] = 0;
  for (int base = r0; base < r1; base += 64) {
    const int r = base + lane;
    const bool v = r < r1;
    const uint32_t d = v ? (uint32_t)(keys[a[r]] >> shift) & 255u : 0u;
    const uint64_t mt = match8(d, v);
    if (v && lane == __ffsll((long long)mt) - 1) mycnt[d] += __popcll(mt);
  }
  __syncthreads();
  // this wave's base for every digit: exclusive prefix over (digit, wave).
  // Lane l owns digits 4l..4l+3: one conflict-free 16-byte read per wave row.
  uint32_t tot[4] = {0u, 0u, 0u, 0u}, mine[4] = {0u, 0u, 0u, 0u};
#pragma unroll 2
  for (int i = 0; i < kFitWaves; ++i) {
    const uint4 c = *reinterpret_cast<const uint4 *>(cnt + i * kDigits + 4 * lane);
    const uint32_t below = (i < w) ? 1u : 0u;
    tot[0] += c.x; tot[1] += c.y; tot[2] += c.z; tot[3] += c.w;
    mine[0] += below * c.x; mine[1] += below * c.y; mine[2] += below * c.z; mine[3] += below * c.w;
  }
  const uint32_t ls = tot[0] + tot[1] + tot[2] + tot[3];
  uint32_t acc = wave_excl_scan_u32(ls);
  uint32_t *myrun = run + w * kDigits;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    myrun[4 * lane + q] = acc + mine[q];
    acc += tot[q];
  }
  // stable scatter (wave-private running bases, LDS ops in program order)
  for (int base = r0; base < r1; base += 64) {
    const int r = base + lane;
    const bool v = r < r1;
    const PosT e = v ? a[r] : (PosT)0;
    const uint32_t d = v ? (uint32_t)(keys[e] >> shift) & 255u : 0u;
    const uint64_t mt = match8(d, v);
    const uint32_t rank = __popcll(mt & lanemask_lt());
    const uint32_t bs = v ? myrun[d] : 0u;
    if (v) b[bs + rank] = e;
    if (v && lane == __ffsll((long long)mt) - 1) myrun[d] = bs + __popcll(mt);
  }
  __syncthreads();
}

// ------------------------------------------------------------------------
// 64 < n <= 1024 (keys in LDS): each wave sorts a run of 64 (key, position)
// pairs in registers (bitonic network over shuffles), then runs are merged
// pairwise in LDS (4 levels): an element's index in the merged run is its
// index in its own run plus its lower bound in the partner run.
// ------------------------------------------------------------------------
constexpr int kMergeMax = 1024;

__device__ void wave_bitonic64(uint64_t &k, uint32_t &p) {
  const int lane = threadIdx.x & 63;
  // loops kept rolled: k_fit runs once per CU, so code size is latency
  for (int kk = 2; kk <= 64; kk <<= 1) {
    for (int j = kk >> 1; j > 0; j >>= 1) {
      const bool asc = (lane & kk) == 0 || kk == 64;
      const uint64_t ok = __shfl_xor(k, j, 64);
      const uint32_t op = __shfl_xor(p, j, 64);
      const bool lower = (lane & j) == 0;
      const bool other_less = kp_less(ok, op, k, p);
      // the lower slot keeps the min when ascending, the max when descending
      if ((lower == asc) ? other_less : !other_less) { k = ok; p = op; }
    }
  }
}

__device__ void merge_sort_1024(const uint64_t *keys, int n, uint16_t *out, uint64_t *bk0,
                                uint16_t *bp0, uint64_t *bk1, uint16_t *bp1) {
  const int t = threadIdx.x;
  uint64_t k = t < n ? keys[t] : ~0ull;
  uint32_t p = (uint32_t)t;  // padding (~0, t >= n): distinct, after every real key
  STAMP(21);
  wave_bitonic64(k, p);
  STAMP(22);
  bk0[t] = k;
  bp0[t] = (uint16_t)p;
  __syncthreads();
  STAMP(23);
  uint64_t *sk = bk0, *dk = bk1;
  uint16_t *sp = bp0, *dp = bp1;
  for (int len = 64; len < kFitThreads; len <<= 1) {
    const int run = t / len, idx = t % len;
    const int other = (run ^ 1) * len;
    int lo = 0, hi = len;  // lower bound of (k, p) in the partner run
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (kp_less(sk[other + mid], sp[other + mid], k, p)) lo = mid + 1;
      else hi = mid;
    }
    const int dst = (run & ~1) * len + idx + lo;
    dk[dst] = k;
    dp[dst] = (uint16_t)p;
    __syncthreads();
    uint64_t *tk = sk; sk = dk; dk = tk;
    uint16_t *tp = sp; sp = dp; dp = tp;
    k = sk[t];  // this thread now owns merged position t
    p = sp[t];
    STAMP(24 + (__builtin_ctz((unsigned)len) - 6));
  }
  if (t < n) out[t] = sp[t];
  __syncthreads();
}

// The same sort on one packed word per element: 32 key bits (from the lowest
// bit that varies over the keys, or up to the highest one: the bits outside
// are equal for all) above the position, so a step is one 64-bit compare and
// one exchange instead of a (key, position) pair.  Exact when no varying bit
// is dropped (!lossy); otherwise a run of equal truncated keys is ordered by
// position, so each such run (rare, short) is re-ranked by its full keys;
// false (the caller then sorts the full keys) for a run of more than kRunMax.
// the word of lane ^ J: DPP for J < 16 (row_shl / row_shr pairs for 4 and 8),
// ds_bpermute across rows
template <int J>
__device__ __forceinline__ uint64_t xor_lane64(uint64_t v) {
  if constexpr (J == 1) return dpp64<kDppXor1>(v);
  else if constexpr (J == 2) return dpp64<kDppXor2>(v);
  else if constexpr (J == 4 || J == 8) {
    const uint64_t up = dpp64<0x100 + J>(v);  // row_shl:J  (lane + J)
    const uint64_t dn = dpp64<0x110 + J>(v);  // row_shr:J  (lane - J)
    return (threadIdx.x & J) ? dn : up;
  } else {
    return __shfl_xor(v, J, 64);
  }
}
template <int KK, int J>
__device__ __forceinline__ void bitonic_stage(uint64_t &k) {
  const int lane = threadIdx.x & 63;
  const bool asc = (lane & KK) == 0 || KK == 64;
  const uint64_t ok = xor_lane64<J>(k);
  const bool lower = (lane & J) == 0;
  const bool other_less = ok < k;
  if ((lower == asc) ? other_less : !other_less) k = ok;
}
__device__ __forceinline__ void wave_bitonic64_packed(uint64_t &k) {
  bitonic_stage<2, 1>(k);
  bitonic_stage<4, 2>(k); bitonic_stage<4, 1>(k);
  bitonic_stage<8, 4>(k); bitonic_stage<8, 2>(k); bitonic_stage<8, 1>(k);
  bitonic_stage<16, 8>(k); bitonic_stage<16, 4>(k); bitonic_stage<16, 2>(k);
  bitonic_stage<16, 1>(k);
  bitonic_stage<32, 16>(k); bitonic_stage<32, 8>(k); bitonic_stage<32, 4>(k);
  bitonic_stage<32, 2>(k); bitonic_stage<32, 1>(k);
  bitonic_stage<64, 32>(k); bitonic_stage<64, 16>(k); bitonic_stage<64, 8>(k);
  bitonic_stage<64, 4>(k); bitonic_stage<64, 2>(k); bitonic_stage<64, 1>(k);
}

// PER elements per thread (element e = u * 1024 + t for register u): PER = 1
// sorts up to 1024 elements in two 4-way merge levels, PER = 4 up to 4096 in
// three (the large-history fit's observation sides of 1k-4k trials, which the
// 8-bit LSD radix sort took 8 passes of ~4 us over).  After the in-register
// 64-runs the merge levels keep the 32 key bits (kb) and the positions (pb)
// in separate LDS arrays and search only kb: every run of a quad holds a
// contiguous position range, ascending with the run index, so an equal key of
// an earlier run precedes the element and one of a later run follows it --
// the searches read 4-byte words, half the LDS traffic of the packed words.
template <int PER>
__device__ __forceinline__ bool merge_sort_packed(const uint64_t *keys, int n, int shift, bool lossy,
                                                  uint16_t *out, uint32_t *kb0, uint32_t *kb1,
                                                  uint16_t *pb0, uint16_t *pb1) {
  const int t = threadIdx.x;
  constexpr int kN = PER * kFitThreads;
  uint32_t k[PER], p[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    k[u] = ~0u;
    p[u] = 0u;
    if (u * kFitThreads >= n) continue;  // all padding: never read (below)
    const int e = u * kFitThreads + t;
    // padding (e >= n): all-ones key bits, position e > every real position
    uint64_t w = (e < n ? ((keys[e] >> shift) << 32) : 0xFFFFFFFF00000000ull) | (uint64_t)e;
    // (a wave-row of padding only is in order already: no network)
    if (u * kFitThreads + (t & ~63) < n) wave_bitonic64_packed(w);
    k[u] = (uint32_t)(w >> 32);
    p[u] = (uint32_t)w;
    kb0[e] = k[u];
    pb0[e] = (uint16_t)p[u];
  }
  STAMP(21);
  __syncthreads();
  STAMP(22);
  // 4-way merge levels (64 -> 256 -> 1024 [-> 4096]): an element's position in
  // its quad of runs is its index in its own run plus its rank in each of the
  // three others, three branch-free binary searches side by side -- half the
  // dependent LDS reads of pairwise levels
  static_assert(kFitThreads == 1024, "64 * 4 * 4");
  uint32_t *sk = kb0, *dk = kb1;
  uint16_t *sp = pb0, *dp = pb1;
#pragma unroll
  for (int len = 64; len < kN; len <<= 2) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      if (u * kFitThreads >= n) continue;  // (block-uniform)
      const int e = u * kFitThreads + t;
      const int qb = e & ~(4 * len - 1), r = (e / len) & 3;  // (r: wave-uniform)
      const int j1 = (r + 1) & 3, j2 = (r + 2) & 3, j3 = (r + 3) & 3;
      const uint32_t *o1 = sk + qb + j1 * len, *o2 = sk + qb + j2 * len, *o3 = sk + qb + j3 * len;
      // count o[i] < key, plus o[i] == key in an earlier run: o[i] < key + (j < r)
      const uint64_t x1 = (uint64_t)k[u] + (j1 < r ? 1u : 0u), x2 = (uint64_t)k[u] + (j2 < r ? 1u : 0u),
                     x3 = (uint64_t)k[u] + (j3 < r ? 1u : 0u);
      // a run that is all padding (first position >= n, all keys all-ones)
      // is not searched: an element of a later run (padding too) ranks after
      // all of it, any other after none of it (runs of a skipped u hold no
      // data, and are only ever such runs)
      // padding (position >= n) sorts after every real element and in position
      // order among itself: it keeps its place, e, in every level (no search)
      const bool pad = p[u] >= (uint32_t)n;
      const bool s1 = !pad && qb + j1 * len < n, s2 = !pad && qb + j2 * len < n,
                 s3 = !pad && qb + j3 * len < n;
      int i1 = 0, i2 = 0, i3 = 0;
#pragma unroll
      for (int step = len / 2; step > 0; step >>= 1) {
        if (s1) i1 += ((uint64_t)o1[i1 + step - 1] < x1) ? step : 0;
        if (s2) i2 += ((uint64_t)o2[i2 + step - 1] < x2) ? step : 0;
        if (s3) i3 += ((uint64_t)o3[i3 + step - 1] < x3) ? step : 0;
      }
      i1 = s1 ? i1 + (((uint64_t)o1[i1] < x1) ? 1 : 0) : (j1 < r ? len : 0);
      i2 = s2 ? i2 + (((uint64_t)o2[i2] < x2) ? 1 : 0) : (j2 < r ? len : 0);
      i3 = s3 ? i3 + (((uint64_t)o3[i3] < x3) ? 1 : 0) : (j3 < r ? len : 0);
      const int dst = pad ? e : qb + (e & (len - 1)) + i1 + i2 + i3;
      dk[dst] = k[u];
      dp[dst] = (uint16_t)p[u];
    }
    __syncthreads();
    uint32_t *tk = sk; sk = dk; dk = tk;
    uint16_t *tp = sp; sp = dp; dp = tp;
#pragma unroll
    for (int u = 0; u < PER; ++u) {  // merged position e
      if (u * kFitThreads >= n) continue;
      k[u] = sk[u * kFitThreads + t];
      p[u] = sp[u * kFitThreads + t];
    }
    STAMP(23 + (__builtin_ctz((unsigned)len) - 6) / 2);
  }
  // runs of equal truncated keys (sorted by position so far) are ranked by
  // their full keys; a run longer than kRunMax sends the block to the full sort
  constexpr int kRunMax = 16;
  bool bad = false;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int e = u * kFitThreads + t;
    if (e < n) {
      int s0 = e, s1 = e + 1;
      if (lossy) {
        while (s0 > 0 && e - s0 < kRunMax && sk[s0 - 1] == k[u]) --s0;
        while (s1 < n && s1 - e <= kRunMax && sk[s1] == k[u]) ++s1;
      }
      if (s1 - s0 > kRunMax) {
        // a long run is in order when all its full keys are equal (ties of a
        // quantized hp: ordered by position already), i.e. when no adjacent
        // pair of it differs; else the block takes the full sort
        const bool mixed = e > s0 && keys[p[u]] != keys[sp[e - 1]];
        if (mixed) bad = true;
        else out[e] = (uint16_t)p[u];
      } else if (s1 - s0 == 1) {
        out[e] = (uint16_t)p[u];
      } else {
        const uint64_t kf = keys[p[u]];
        int r = 0;
        for (int v = s0; v < s1; ++v) {
          const uint32_t pv = sp[v];
          r += kp_less(keys[pv], pv, kf, p[u]) ? 1 : 0;
        }
        out[s0 + r] = (uint16_t)p[u];
      }
    }
  }
  STAMP(26);
  const bool ok = !__syncthreads_or(bad);
  STAMP(27);
  return ok;
}

template <typename PosT, bool SMALL = false>
__device__ __forceinline__ PosT *block_sort_perm(const uint64_t *keys, PosT *a, PosT *b, int n, uint64_t vary,
                                 uint32_t *cnt, uint32_t *run, FitShared &sm) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (n > 64 && n <= kMergeMax && sizeof(PosT) == 2) {
    // cnt + run regions (32 KB) hold the merge buffers (12 KB; the full-key
    // fallback: its two key buffers, b the positions)
    uint64_t *bk = reinterpret_cast<uint64_t *>(cnt);
    // the 32-bit window: from the lowest varying bit, or up to the highest
    const int hb = 63 - __builtin_clzll(vary | 1ull), lb = vary ? __builtin_ctzll(vary) : 0;
    const int shift = max(lb, hb - 31);
    uint32_t *kb = reinterpret_cast<uint32_t *>(cnt);
    uint16_t *pb = reinterpret_cast<uint16_t *>(kb + 2 * kFitThreads);
    if (merge_sort_packed<1>(keys, n, shift, shift > lb, reinterpret_cast<uint16_t *>(a), kb,
                             kb + kFitThreads, pb, pb + kFitThreads))
      return a;
    uint16_t *bp = reinterpret_cast<uint16_t *>(b);
    merge_sort_1024(keys, n, reinterpret_cast<uint16_t *>(a), bk, bp, bk + kFitThreads,
                    bp + kFitThreads);
    return a;
  }
  if (n <= 64) {  // one wave: rank by counting, no barriers inside
    if (w == 0 && lane < n) {
      const uint64_t k = keys[lane];
      int rank = 0;
      for (int j = 0; j < n; ++j) rank += kp_less(keys[j], j, k, lane) ? 1 : 0;
      a[rank] = (PosT)lane;
    }
    __syncthreads();
    return a;
  }
  if (SMALL) return a;  // n <= kMergeMax: unreachable
  int passes = 0;
  for (int shift = 0; shift < 64; shift += 8) passes += ((vary >> shift) & 255u) ? 1 : 0;
  if (sizeof(PosT) == 2 && n <= 4 * kMergeMax && passes > 2) {
    // keys in LDS (n <= 4096: bytes [0, 32 KB) of the key region), the merge
    // buffers (2 x 16 KB keys, 2 x 8 KB positions) above them (the last
    // overlaps a, which the radix fallback re-initialises), the result in b
    static_assert(8 * 4 * kMergeMax + 12 * 4 * kMergeMax <= kOffPosB, "merge buffers below b");
    uint32_t *kb = reinterpret_cast<uint32_t *>(const_cast<uint64_t *>(keys) + 4 * kMergeMax);
    uint16_t *pb = reinterpret_cast<uint16_t *>(kb + 8 * kMergeMax);
    const int hb = 63 - __builtin_clzll(vary | 1ull), lb = vary ? __builtin_ctzll(vary) : 0;
    const int shift = max(lb, hb - 31);
    if (merge_sort_packed<4>(keys, n, shift, shift > lb, reinterpret_cast<uint16_t *>(b), kb,
                             kb + 4 * kMergeMax, pb, pb + 4 * kMergeMax))
      return b;
  }
  for (int i = threadIdx.x; i < n; i += blockDim.x) a[i] = (PosT)i;
  __syncthreads();
  STAMP(38);
  for (int shift = 0; shift < 64; shift += 8) {
    if (((vary >> shift) & 255u) == 0) continue;
    radix_pass<PosT>(keys, a, b, n, shift, cnt, run);
    STAMP(39);
    PosT *t = a; a = b; b = t;
  }
  return a;
}

// ------------------------------------------------------------------------
// numpy float64 sum (ndarray.sum) of NA arrays: buffers of 8192 elements,
// each reduced by the pairwise tree above, buffer results added in order.
// Leaves run in parallel on 8-lane groups, lane s owning numpy's accumulator
// r[s]; wave 0 then adds the internal nodes level by level (a wave's LDS ops
// complete in order, so the levels need no barrier).
template <int NA>
__device__ __forceinline__ void block_np_sums(const double *const (&arr)[NA], int64_t n,
                                              FitShared &sm, double (&out)[NA]) {
  const int s = threadIdx.x & 7, groups = blockDim.x >> 3;
  for (int64_t c0 = 0; c0 < n; c0 += 8192) {
    const int cn = (int)min<int64_t>(8192, n - c0);
    // a node at depth d holds at most cn / 2^d + 16 elements (a right child
    // is at most 7 above half its parent), so internal nodes (> 128) live at
    // depth <= dtop and leaves below heap id 2^(dtop + 2)
    int dtop = 0;
    while (dtop < 6 && cn > (112 << (dtop + 1))) ++dtop;
    const int idend = 1 << (dtop + 2);
    __syncthreads();  // previous chunk's root consumed, the arrays written
    STAMP(28);
    for (int id0 = 1; id0 < idend; id0 += groups) {  // uniform trip count
      const int id = id0 + (threadIdx.x >> 3);
      const NpNode nd = id < kNpHeap ? np_node(cn, id) : NpNode{0, 0};
      const bool leaf = nd.n > 0 && nd.n <= 128;
      const int ln = leaf ? nd.n : 0;
      const int body = ln - ln % 8;
#pragma unroll
      for (int q = 0; q < NA; ++q) {
        const double *p = arr[q] + c0 + nd.lo;
        double r = 0.0;
        if (ln >= 8) {
          r = p[s];
          // unrolled: the loads of a group are issued before its in-order adds
#pragma unroll 4
          for (int i = 8 + s; i < body; i += 8) r += p[i];
        }
        // ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) in lane s = 0
        // (fp addition commutes exactly; half_mirror brings lane 7's
        // (r6 + r7) + (r4 + r5) to lane 0)
        r = r + dppd<kDppXor1>(r);
        r = r + dppd<kDppXor2>(r);
        r = r + dppd<kDppHalfMirror>(r);
        if (leaf && s == 0) {
          // the (< 8) trailing elements in order: loads first, then the adds
          const int t0 = ln < 8 ? 0 : body;
          double res = ln < 8 ? 0.0 : r, tl[7];
#pragma unroll
          for (int j = 0; j < 7; ++j) tl[j] = (t0 + j < ln) ? p[t0 + j] : 0.0;
#pragma unroll
          for (int j = 0; j < 7; ++j)
            if (t0 + j < ln) res += tl[j];
          sm.val[q][id] = res;
        }
      }
    }
    __syncthreads();
    STAMP(29);
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      for (int d = dtop; d >= 0; --d) {
        const int id = (1 << d) + lane;
        if (lane < (1 << d) && np_node(cn, id).n > 128) {
#pragma unroll
          for (int q = 0; q < NA; ++q) sm.val[q][id] = sm.val[q][2 * id] + sm.val[q][2 * id + 1];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      }
      // running total of the buffers in the unused heap slot 0
      if (lane == 0) {
#pragma unroll
        for (int q = 0; q < NA; ++q)
          sm.val[q][0] = (c0 == 0) ? (0.0 + sm.val[q][1]) : (sm.val[q][0] + sm.val[q][1]);
      }
    }
  }
  __syncthreads();
  STAMP(30);
#pragma unroll
  for (int q = 0; q < NA; ++q) out[q] = n > 0 ? sm.val[q][0] : 0.0;
}

__device__ double block_np_sum(const double *a, int64_t n, FitShared &sm) {
  const double *const arr[1] = {a};
  double out[1];
  block_np_sums<1>(arr, n, sm, out);
  return out[0];
}

// ------------------------------------------------------------------------
// scalar helpers of the reference
// ------------------------------------------------------------------------
// linear_forgetting_weights(n, lf)[i] (tpe.py:381-394) with numpy linspace
// rounding (i*step + start, last ramp element == stop).  The two divisions
// are hoisted: LfRamp is built once per slot.
struct LfRamp {
  int64_t ramp;  // ramp length n - lf (<= 0: all ones)
  double start, step;
};
__device__ __forceinline__ LfRamp lf_ramp(int64_t n, int32_t lf) {
  LfRamp r;
  r.ramp = n < lf ? 0 : n - lf;
  r.start = 1.0 / (double)(n > 0 ? n : 1);
  r.step = r.ramp > 1 ? (1.0 - r.start) / (double)(r.ramp - 1) : 0.0;
  return r;
}
__device__ __forceinline__ double lf_weight(const LfRamp &r, int64_t i) {
  if (i >= r.ramp) return 1.0;
  if (r.ramp == 1) return r.start;
  if (i == r.ramp - 1) return 1.0;
  return (double)i * r.step + r.start;
}

// the observation transform of an hp (tpe.py:510-560 posteriors): one log
// at most per value; `floor` = the clip's lower bound (max(EPS, exp(low)) or
// EPS), computed once per slot by ObsFloor
__device__ __forceinline__ double obs_floor(int32_t tf, double low) {
  if (tf == TPE_OBS_LOG_CLIP_EXPLOW) return np_maximum(kEPS, exp(low));
  return kEPS;
}
__device__ __forceinline__ double obs_transform(double v, int32_t tf, double floor) {
  if (tf == TPE_OBS_IDENT) return v;
  const bool clip = tf == TPE_OBS_LOG_CLIP_EXPLOW || tf == TPE_OBS_LOG_CLIP_EPS;
  return log(clip ? np_maximum(v, floor) : v);
}

// ------------------------------------------------------------------------
// (a2) split: the n_below-th smallest (loss key, position).  below(j) <=>
// (key_j, j) <= threshold.  mode 0: nothing below, 1: everything below.
// ------------------------------------------------------------------------
struct Split {
  uint64_t k;
  uint32_t p;
  int mode;  // 0 none, 1 all, 2 threshold
};

__device__ __forceinline__ bool is_below(const Split &t, uint64_t k, uint32_t j) {
  return t.mode == 1 || (t.mode == 2 && !kp_less(t.k, t.p, k, j));
}

struct FitCtx {
  unsigned char *lds;
  uint64_t *gkeys;      // global sort keys   [scap]
  uint32_t *gpa, *gpb;  // global permutations [scap]
};

struct Digit {
  uint32_t d;     // selected digit
  uint32_t cnt;   // values with that digit (under the prefix)
  uint32_t need;  // the rank sought, inside that digit
};

// select_digit's value functions, passed by value (in registers: a lambda
// capturing by reference would put its captures on the scratch stack and
// make every value a scratch load)
struct KeyAt {
  const uint64_t *keys;
  __device__ uint64_t operator()(int j) const { return keys[j]; }
};
struct TiedPosAt {  // positions of the trials whose key equals T
  const uint64_t *keys;
  uint64_t T;
  __device__ uint64_t operator()(int j) const { return keys[j] == T ? (uint64_t)j : ~0ull; }
};

// One radix-select step: histogram of the 8-bit digit at `shift` of the
// values v(j) whose bits under `mask` equal `prefix` -- each wave counts into
// its own 256 bins (cnt[wave][256]) with one LDS atomic per value (an 8-ballot
// match per 64 values to elect one adder per distinct digit cost ~20
// instructions per value: 3-8 us of a 1e4-trial split), the bins summed per
// digit into tot[256] -- then the digit holding the need-th (1-based)
// smallest; `need` becomes the rank inside it.
template <typename ValFn>
__device__ __forceinline__ Digit select_digit(ValFn val, int n, uint64_t mask, uint64_t prefix, int shift,
                                       uint32_t need, uint32_t *cnt, uint32_t *tot, FitShared &sm,
                                       int par) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t *mine = cnt + w * kDigits;
  for (int d = lane; d < kDigits; d += 64) mine[d] = 0;
  STAMP(16);
  // (a wave's LDS operations complete in order: its zeroing precedes its adds)
  for (int j0 = 0; j0 < n; j0 += blockDim.x) {
    const int j = j0 + threadIdx.x;
    const uint64_t x = j < n ? val(j) : 0ull;
    const bool v = j < n && (x & mask) == prefix;
    if (v) __hip_atomic_fetch_add(&mine[(uint32_t)(x >> shift) & 255u], 1u, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  STAMP(17);
  __syncthreads();
  STAMP(18);
  if (threadIdx.x < kDigits) {
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < kFitWaves; ++q) c += cnt[q * kDigits + threadIdx.x];
    tot[threadIdx.x] = c;
  }
  __syncthreads();
  if (w == 0) {
    const uint4 c = *reinterpret_cast<const uint4 *>(tot + 4 * lane);
    const uint32_t ls = c.x + c.y + c.z + c.w;
    const uint32_t before = wave_excl_scan_u32(ls);
    if (before < need && need <= before + ls) {  // the digit reaching `need`
      uint32_t acc = before, dd = 4 * lane, cn = c.x;
      if (acc + c.x < need) {
        acc += c.x; dd += 1; cn = c.y;
        if (acc + c.y < need) {
          acc += c.y; dd += 1; cn = c.z;
          if (acc + c.z < need) { acc += c.z; dd += 1; cn = c.w; }
        }
      }
      sm.rp[par][0] = dd;
      sm.rp[par][1] = need - acc;
      sm.rp[par][2] = cn;
    }
  }
  STAMP(19);
  __syncthreads();
  STAMP(20);
  return Digit{sm.rp[par][0], sm.rp[par][2], sm.rp[par][1]};
}

// (a2) the n_below-th smallest (loss key, position) by radix select over the
// 64-bit keys (digits constant over all losses skipped), then -- only when
// several trials tie on that loss -- over the positions of the tied ones.
// The losses are read here (four loads in flight per thread); their keys
// stay in LDS (up to kSortCap trials, else the global copy) for the gather.
template <bool SMALL = false>
__device__ __forceinline__ Split compute_split(const FitArgs &A, const FitCtx &C, FitShared &sm) {
  const int n = (int)A.n;
  const int nb = A.n_below;
  if (nb <= 0 || n == 0) return Split{0, 0, 0};
  if (nb >= n) return Split{0, 0, 1};
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t *lk = reinterpret_cast<uint64_t *>(C.lds + kOffKeys);
  uint32_t *cnt = reinterpret_cast<uint32_t *>(C.lds + kOffCnt);  // [16 waves][256]
  uint32_t *tot = reinterpret_cast<uint32_t *>(C.lds + kOffRun);  // [256]
  uint64_t *keys = (SMALL || n <= kSortCap) ? lk : C.gkeys;
  STAMP(31);
  uint64_t an = ~0ull, on = 0ull;
  {
    // four loads in flight per thread before their keys are stored
    for (int j0 = threadIdx.x; j0 < n; j0 += 4 * (int)blockDim.x) {
      double l[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) l[u] = A.losses[min(j0 + u * (int)blockDim.x, n - 1)];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int j = j0 + u * (int)blockDim.x;
        if (j < n) {
          const uint64_t k = sort_key(l[u]);
          keys[j] = k;
          an &= k;
          on |= k;
        }
      }
    }
  }
  STAMP(32);
  an = wave_and(an);
  on = wave_or(on);
  if (lane == 0) { sm.vand[w] = an; sm.vor[w] = on; }
  STAMP(33);
  __syncthreads();
  STAMP(34);
  an = ~0ull;
  on = 0ull;
#pragma unroll
  for (int i = 0; i < kFitWaves; ++i) { an &= sm.vand[i]; on |= sm.vor[i]; }
  const uint64_t vary = an ^ on;
  STAMP(11);
  uint64_t mask = ~vary, prefix = an & ~vary;  // constant digits are known
  uint32_t need = (uint32_t)nb, eq = (uint32_t)n;
  int step = 0;
  const KeyAt kv{keys};
  for (int shift = 56; shift >= 0; shift -= 8) {
    const uint64_t dm = 255ull << shift;
    if ((vary & dm) == 0) continue;
    const Digit g = select_digit(kv, n, mask, prefix, shift, need, cnt, tot, sm, step & 1);
    ++step;
    need = g.need;
    prefix |= (uint64_t)g.d << shift;
    mask |= dm;
    eq = g.cnt;
    if (step <= 4) STAMP(11 + step);
    // every key under this prefix is below: the largest key with the prefix
    // is an exact threshold (usually after 2-3 digits)
    if (need == eq) return Split{prefix | ~mask, ~0u, 2};
  }
  // prefix = threshold key T; `need` of the `eq` trials with key T are below
  if (need == eq) return Split{prefix, ~0u, 2};
  const uint64_t T = prefix;
  uint64_t pmask = 0, pprefix = 0;
  const TiedPosAt pv{keys, T};
  for (int shift = 24; shift >= 0; shift -= 8) {
    const Digit g = select_digit(pv, n, pmask | 0xFFFFFFFF00000000ull, pprefix, shift, need,
                                 cnt, tot, sm, step & 1);
    ++step;
    need = g.need;
    pprefix |= (uint64_t)g.d << shift;
    pmask |= 255ull << shift;
  }
  return Split{T, (uint32_t)pprefix, 2};
}

// ------------------------------------------------------------------------
// the scoring table of a continuous slot (block-wide): coefficients of the K
// components, and for log-sum-exp kinds the block envelopes (one xor-shuffle
// reduction per 8 components, computed with the coefficients) and the
// padding components of the last block (alpha = -inf: terms exactly 0).
// ------------------------------------------------------------------------
__device__ __forceinline__ void store_table(const tpe_hp &H, Coef *cf, Coef32 *cf32, CoefM *cfm,
                                            CoefM8 *cfm8, CoefM8 *cfmh, float4 *cfe, int K,
                                            const double *w,
                                            const double *mu, const double *sg, double pacc,
                                            bool quant) {
  const int kp = (K + kCoefBlock - 1) / kCoefBlock * kCoefBlock;
  const int kp16 = (K + kMomChunk - 1) / kMomChunk * kMomChunk;
  // kp and the block size are multiples of 8: the 8 lanes of a block's
  // components are active together for the shuffles; kp16 (log-sum-exp):
  // the 16 lanes of a moment chunk likewise (lanes past kp are padding of
  // the chunk only, with no coefficient entry)
  // (cfm null: the moment table is not wanted by this fit's suggest)
  for (int k = threadIdx.x; k < (quant ? K : (cfm || cfmh) ? kp16 : kp); k += blockDim.x) {
    EnvTerm e{0.0, 0.0, 0.0};
    const bool real = k < K;
    const Coef c = real ? make_coef(H, w[k], mu[k], sg[k], pacc, &e)
                        : Coef{-INFINITY, 0.0, 0.0, 0.0};
    if (k < kp) {
      store_coef(cf, k, c, quant);
      if (!quant) store_lse_envelope(cf, k, e, real, c, cf32, cfe);
      if (!quant && cfm8) store_lse_moments8(cfm8, k, e, real);
    }
    if (!quant && cfm) store_lse_moments(cfm, k, e, real);
    if (!quant && cfmh) store_lse_moments16h(cfmh, k, e, real);
  }
}

// The extremes of a log-sum-exp table's block envelopes outside the probe's
// block (MixInfo::env_cmax / env_amin, for the scoring waves' live-range
// search): max c (e.z) and min a^2 (|e.w|, the sign flags a wide block), as
// stored.  Block-wide (after the table's stores: one barrier first); every
// thread returns them.
__device__ __forceinline__ float2 envelope_extremes(const Coef *cf, int K, int probe,
                                                    FitShared &sm) {
  __syncthreads();
  const int nb = (K + kCoefBlock - 1) / kCoefBlock, pb = probe >= 0 ? probe / kCoefBlock : -1;
  const double *t = reinterpret_cast<const double *>(cf);
  float cmax = -INFINITY, amin = INFINITY;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    if (b == pb) continue;
    const float *e = reinterpret_cast<const float *>(t + coef_off((int64_t)b * kCoefBlock, 3));
    cmax = fmaxf(cmax, e[2] == e[2] ? e[2] : INFINITY);
    amin = fminf(amin, fabsf(e[3]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cmax = fmaxf(cmax, __shfl_xor(cmax, o, 64));
    amin = fminf(amin, __shfl_xor(amin, o, 64));
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) { sm.envc[wv] = cmax; sm.enva[wv] = amin; }
  __syncthreads();
  cmax = -INFINITY;
  amin = INFINITY;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
    cmax = fmaxf(cmax, sm.envc[w]);
    amin = fminf(amin, sm.enva[w]);
  }
  return make_float2(cmax, amin);
}

// ------------------------------------------------------------------------
// per-component lpdf constants + truncation mass of one slot (block-wide);
// w/mu/sg may be LDS or global; tmp: K doubles of scratch
// ------------------------------------------------------------------------
// (the descriptor comes by global pointer: a reference to a by-value copy
// would put that copy on the scratch stack when the call is not inlined)
__device__ __forceinline__ void prep_slot(const tpe_hp *Hg, int64_t slot, int K, const double *w, const double *mu,
                          const double *sg, MixInfo *info, Coef *coef, Coef32 *coef32,
                          CoefM *coefm, CoefM8 *coefm8, float4 *coefe, int64_t kcap,
                          double *tmp, FitShared &sm) {
  const tpe_hp H = *Hg;
  Coef *cf = coef + slot * kcap;
  Coef32 *cf32 = coef32 + slot * (kcap / kCoefBlock);
  CoefM *cfm = coefm ? coefm + slot * mom_stride(kcap) : nullptr;
  CoefM8 *cfm8 = coefm8 ? coefm8 + slot * (kcap / kCoefBlock) : nullptr;
  float4 *cfe = coefe ? coefe + slot * (kcap / kCoefBlock) : nullptr;
  const double wsum = block_np_sum(w, K, sm);
  STAMP(7);
  if (H.family == TPE_CAT) {
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
      Coef c;
      c.x = log(w[k]); c.y = 0.0; c.z = 0.0; c.w = 0.0;
      store_coef(cf, k, c);
    }
    if (threadIdx.x == 0) {
      MixInfo mi;
      mi.K = K; mi.kind = 2; mi.p_accept = 1.0; mi.log_pacc = 0.0; mi.wsum = wsum;
      mi.probe = -1; mi.env_cmax = 0.0f; mi.env_amin = 0.0f; mi.pad2 = 0;
      info[slot] = mi;
    }
    return;
  }
  const bool bounded = (H.flags & (TPE_HAS_LOW | TPE_HAS_HIGH)) != 0;
  double pacc = 1.0;
  if (bounded) {  // tpe.py:130-136 / 273-276 (log-space bounds for LGMM)
    for (int k = threadIdx.x; k < K; k += blockDim.x)
      tmp[k] = w[k] * (normal_cdf(H.high, mu[k], sg[k]) - normal_cdf(H.low, mu[k], sg[k]));
    __syncthreads();
    pacc = block_np_sum(tmp, K, sm);
  }
  STAMP(8);
  const bool quant = (H.flags & TPE_HAS_Q) != 0;
  store_table(H, cf, cf32, cfm, cfm8, nullptr, cfe, K, w, mu, sg, pacc, quant);
  if (threadIdx.x == 0) {
    MixInfo mi;
    mi.K = K; mi.kind = quant ? 1 : 0; mi.p_accept = pacc; mi.log_pacc = log(pacc);
    mi.wsum = wsum; mi.probe = -1; mi.env_cmax = 0.0f; mi.env_amin = 0.0f; mi.pad2 = 0;
    info[slot] = mi;
  }
}

// ------------------------------------------------------------------------
// (a4) adaptive_parzen_normal on the m observations ob[] (tid order) after
// the sort; nlt = #{obs < prior_mu} = searchsorted(sorted, prior_mu, 'left')
// ------------------------------------------------------------------------
template <bool MIXLDS, typename PosT, int QN = 4>  // QN: observations per thread (m <= QN * 1024)
__device__ __forceinline__ void fit_continuous(const FitArgs &A, const FitCtx &C, FitShared &sm, const tpe_hp &H,
                               int64_t slot, const double *ob, const PosT *perm, int m, int nlt) {
  const double pm = H.prior_mu, ps = H.prior_sigma;
  const int K = m + 1;
  double *lm = reinterpret_cast<double *>(C.lds);
  double *gw = A.mw + slot * A.kcap, *gm = A.mmu + slot * A.kcap, *gs = A.msig + slot * A.kcap;
  double *mu = MIXLDS ? lm : gm;
  double *w = MIXLDS ? lm + kMixStride : gw;
  double *sg = MIXLDS ? lm + 2 * kMixStride : gs;
  double *tmp = MIXLDS ? lm + 3 * kMixStride : A.tmp + slot * A.kcap;
  int pos;
  if (m == 0) pos = 0;                          // tpe.py:410-413
  else if (m == 1) pos = (pm < ob[0]) ? 0 : 1;  // tpe.py:414-422
  else pos = nlt;                               // tpe.py:427-428
  const bool lfw = A.lf && A.lf < m;            // tpe.py:440
  const LfRamp lr = lf_ramp(m, A.lf);
  // place the sorted observations around the prior (tpe.py:429-432, 441-445)
  if (MIXLDS) {
    double v[4], wt[4];
#pragma unroll
    for (int q = 0; q < QN; ++q) {
      const int r = threadIdx.x + q * kFitThreads;
      if (r < m) {
        const int e = (int)perm[r];
        v[q] = ob[e];
        wt[q] = lfw ? lf_weight(lr, e) : 1.0;
      }
    }
    __syncthreads();  // perm (LDS) is overwritten by the mixture arrays below
#pragma unroll
    for (int q = 0; q < QN; ++q) {
      const int r = threadIdx.x + q * kFitThreads;
      if (r < m) {
        const int o = r + (r >= pos ? 1 : 0);
        mu[o] = v[q];
        w[o] = wt[q];
      }
    }
  } else {
    for (int r = threadIdx.x; r < m; r += blockDim.x) {
      const int e = (int)perm[r];
      const int o = r + (r >= pos ? 1 : 0);
      mu[o] = ob[e];
      w[o] = lfw ? lf_weight(lr, e) : 1.0;
    }
  }
  if (threadIdx.x == 0) { mu[pos] = pm; w[pos] = A.prior_weight; }
  __syncthreads();
  STAMP(4);
  // neighbour sigma (tpe.py:433-439), clip (456-460), prior sigma (461)
  const double hi = ps / 1.0;
  const double lo = ps / fmin(100.0, 1.0 + (double)K);
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    double s;
    if (m == 0) s = ps;
    else if (m == 1) s = (k == pos) ? ps : ps * .5;
    else if (k == 0) s = mu[1] - mu[0];
    else if (k == K - 1) s = mu[K - 1] - mu[K - 2];
    else s = np_maximum(mu[k] - mu[k - 1], mu[k + 1] - mu[k]);
    s = np_minimum(np_maximum(s, lo), hi);
    if (k == pos) s = ps;
    sg[k] = s;
  }
  STAMP(5);
  const double tot = block_np_sum(w, K, sm);  // tpe.py:468 (its barriers cover sg too)
  // normalise, and the truncation-mass terms of the same component
  // (tpe.py:130-136 / 273-276; LGMM bounds are log-space) -- no barrier between
  const bool bounded = (H.flags & (TPE_HAS_LOW | TPE_HAS_HIGH)) != 0;
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const double wk = w[k] / tot;
    w[k] = wk;
    if (bounded)
      tmp[k] = wk * (normal_cdf(H.high, mu[k], sg[k]) - normal_cdf(H.low, mu[k], sg[k]));
  }
  STAMP(6);
  double sums[2];
  {
    const double *const arr[2] = {w, tmp};
    if (bounded) block_np_sums<2>(arr, K, sm, sums);
    else { const double *const a1[1] = {w}; double s1[1]; block_np_sums<1>(a1, K, sm, s1); sums[0] = s1[0]; sums[1] = 1.0; }
  }
  STAMP(8);
  const double wsum = sums[0], pacc = sums[1];
  // per-component lpdf constants (tpe.py:138-160, 277-299) + copy-out
  const bool quant = (H.flags & TPE_HAS_Q) != 0;
  Coef *cf = A.coef + slot * A.kcap;
  Coef32 *cf32 = A.coef32 + slot * (A.kcap / kCoefBlock);
  CoefM *cfm = A.coefm ? A.coefm + slot * mom_stride(A.kcap) : nullptr;
  CoefM8 *cfm8 = A.coefm8 ? A.coefm8 + slot * (A.kcap / kCoefBlock) : nullptr;
  CoefM8 *cfmh = A.coefmh ? A.coefmh + slot * mom_stride(A.kcap) : nullptr;
  float4 *cfe = A.coefe ? A.coefe + slot * (A.kcap / kCoefBlock) : nullptr;
  if (MIXLDS)
    for (int k = threadIdx.x; k < K; k += blockDim.x) { gw[k] = w[k]; gm[k] = mu[k]; gs[k] = sg[k]; }
  store_table(H, cf, cf32, cfm, cfm8, cfmh, cfe, K, w, mu, sg, pacc, quant);
  // (block-uniform: K, quant)
  const float2 ex = (!quant && K >= kRangeMinK) ? envelope_extremes(cf, K, pos, sm)
                                                : make_float2(0.0f, 0.0f);
  if (threadIdx.x == 0) {
    MixInfo mi;
    mi.K = K; mi.kind = quant ? 1 : 0; mi.p_accept = pacc; mi.log_pacc = log(pacc);
    mi.wsum = wsum;
    mi.probe = pos;  // the prior: sigma = prior_sigma, the widest after the clip
    mi.env_cmax = ex.x;
    mi.env_amin = ex.y > 0.0f && ex.y < INFINITY && ex.x < INFINITY ? ex.y : 0.0f;
    mi.pad2 = 0;
    A.info[slot] = mi;
  }
}

// ------------------------------------------------------------------------
// (a8) categorical posterior: LF-weighted bincount in observation order
// (np.bincount adds sequentially per bin), + pseudocounts, normalised.
// perm: observations stably sorted by category -> one segment per bin whose
// serial sum keeps the reference's rounding.
// ------------------------------------------------------------------------
// the per-bin sums, pseudocounts and normalisation once ws holds the LF
// weights grouped by bin (bin c: ws[seg[2c], seg[2c+1]) in observation order)
__device__ __forceinline__ void categorical_tail(const FitArgs &A, FitShared &sm, const tpe_hp &H,
                                                 int64_t slot, const int *seg, const double *ws);

template <typename PosT>
__device__ __forceinline__ void fit_categorical(const FitArgs &A, const FitCtx &C, FitShared &sm,
                                const tpe_hp &H, int64_t slot, const uint64_t *keys,
                                const PosT *perm, int m) {
  const int upper = H.upper;
  double *mu = A.mmu + slot * A.kcap;
  // segment bounds per bin: LDS (cnt/run region) when they fit, else the
  // (not yet written) global mu array of the slot
  int *seg = upper <= 4096 ? reinterpret_cast<int *>(C.lds + kOffCnt) : reinterpret_cast<int *>(mu);
  for (int c = threadIdx.x; c < 2 * upper; c += blockDim.x) seg[c] = 0;
  __syncthreads();
  for (int r = threadIdx.x; r < m; r += blockDim.x) {
    const uint64_t b = keys[perm[r]];
    if (b >= (uint64_t)upper) continue;
    if (r == 0 || keys[perm[r - 1]] != b) seg[2 * b] = r;
    if (r == m - 1 || keys[perm[r + 1]] != b) seg[2 * b + 1] = r + 1;
  }
  __syncthreads();  // keys are dead from here on
  STAMP(40);
  // LF weights in sorted order, in parallel (LDS over the keys, or HBM scratch)
  double *ws = m <= kSortCap ? reinterpret_cast<double *>(C.lds + kOffKeys) : A.ob + slot * A.kcap;
  const LfRamp lr = lf_ramp(m, A.lf);
  for (int r = threadIdx.x; r < m; r += blockDim.x) ws[r] = lf_weight(lr, (int64_t)perm[r]);
  __syncthreads();
  STAMP(41);
  categorical_tail(A, sm, H, slot, seg, ws);
}

// Categorical fit of a large history (m <= kSortCap observations, keys in
// LDS) over few bins (upper <= 64): no sort.  A stable counting pass puts each
// observation's LF weight straight at its place in the bin-grouped order:
// every wave takes a contiguous run of the observations, counts its bins by
// one ballot per bin and 64 observations, and scatters with the bin's base
// (bins in order, waves in order within a bin) plus the rank among the equal
// keys of its 64 -- the order the stable sort gives, so the sums are the same.
constexpr int kCatFastBins = 64;
constexpr int kCatFastChunks = (kSortCap + kFitThreads - 1) / kFitThreads;  // 64-runs per wave
__device__ __forceinline__ void fit_categorical_counting(const FitArgs &A, const FitCtx &C,
                                                         FitShared &sm, const tpe_hp &H,
                                                         int64_t slot, int m) {
  const int upper = H.upper;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t *keys = reinterpret_cast<const uint64_t *>(C.lds + kOffKeys);
  int *seg = reinterpret_cast<int *>(C.lds + kOffCnt);                 // [2 * upper]
  uint32_t *wc = reinterpret_cast<uint32_t *>(C.lds + kOffRun);        // [16 waves][64 bins]
  const int per = (m + kFitWaves * 64 - 1) / (kFitWaves * 64) * 64;    // <= 64 * kCatFastChunks
  const int r0 = wv * per;
  // this wave's keys into registers (bin, or -1), then its per-bin counts
  int kr[kCatFastChunks];
  uint32_t cnt = 0;
#pragma unroll
  for (int q = 0; q < kCatFastChunks; ++q) {
    const int i = r0 + q * 64 + lane;
    const bool v = q * 64 < per && i < m;
    const uint64_t k = v ? keys[i] : ~0ull;
    kr[q] = k < (uint64_t)upper ? (int)k : -1;
    if (q * 64 < per) {
      for (int b = 0; b < upper; ++b) {
        const uint64_t bal = __ballot(kr[q] == b);
        if (lane == b) cnt += (uint32_t)__popcll(bal);
      }
    }
  }
  wc[wv * kCatFastBins + lane] = lane < upper ? cnt : 0u;
  __syncthreads();  // every key is in registers: the key region is free for ws
  // lane b: bin b's start (bins before it, all waves) + its count in waves before this one
  uint32_t tot = 0, mine = 0;
#pragma unroll
  for (int w = 0; w < kFitWaves; ++w) {
    const uint32_t c = wc[w * kCatFastBins + lane];
    tot += c;
    mine += w < wv ? c : 0u;
  }
  const uint32_t start = wave_excl_scan_u32(tot);
  if (wv == 0 && lane < upper) {
    seg[2 * lane] = (int)start;
    seg[2 * lane + 1] = (int)(start + tot);
  }
  uint32_t run = start + mine;
  double *ws = reinterpret_cast<double *>(C.lds + kOffKeys);
  const LfRamp lr = lf_ramp(m, A.lf);
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
#pragma unroll
  for (int q = 0; q < kCatFastChunks; ++q) {
    if (q * 64 >= per) break;
    uint32_t rank = 0, inc = 0;
    for (int b = 0; b < upper; ++b) {
      const uint64_t bal = __ballot(kr[q] == b);
      if (kr[q] == b) rank = (uint32_t)__popcll(bal & lt);
      if (lane == b) inc = (uint32_t)__popcll(bal);
    }
    const uint32_t base = (uint32_t)__shfl((int)run, kr[q] < 0 ? 0 : kr[q], 64);
    if (kr[q] >= 0) ws[base + rank] = lf_weight(lr, (int64_t)(r0 + q * 64 + lane));
    run += inc;
  }
  __syncthreads();
  STAMP(41);
  categorical_tail(A, sm, H, slot, seg, ws);
}

__device__ __forceinline__ void categorical_tail(const FitArgs &A, FitShared &sm, const tpe_hp &H,
                                                 int64_t slot, const int *seg, const double *ws) {
  const int upper = H.upper;
  double *w = A.mw + slot * A.kcap, *mu = A.mmu + slot * A.kcap, *sg = A.msig + slot * A.kcap;
  for (int c = threadIdx.x; c < upper; c += blockDim.x) {
    // serial per bin (np.bincount order); loads run 8 ahead of the adds
    double cnt = 0.0;
    const int r1 = seg[2 * c + 1];
    int r = seg[2 * c];
    for (; r + 8 <= r1; r += 8) {
      double wv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) wv[u] = ws[r + u];
#pragma unroll
      for (int u = 0; u < 8; ++u) cnt += wv[u];
    }
    for (; r < r1; ++r) cnt += ws[r];
    double pc;
    if (H.flags & TPE_PCHOICE)
      pc = cnt + (double)upper * (A.prior_weight * A.pprior[H.pprior_begin + c]);
    else
      pc = cnt + A.prior_weight;
    w[c] = pc;
  }
  __syncthreads();
  STAMP(5);
  const double tot = block_np_sum(w, upper, sm);
  for (int c = threadIdx.x; c < upper; c += blockDim.x) {
    w[c] = w[c] / tot;
    mu[c] = 0.0;
    sg[c] = 0.0;
  }
  __syncthreads();
  prep_slot(A.hps + slot / 2, slot, upper, w, mu, sg, A.info, A.coef, A.coef32, A.coefm, A.coefm8,
            A.coefe, A.kcap, A.tmp + slot * A.kcap, sm);
}

// ------------------------------------------------------------------------
// k_fit: split + fit + lpdf constants, one block per (hp, side)
// ------------------------------------------------------------------------
#ifndef TPE_FIT_REPS
#define TPE_FIT_REPS 1  // diagnostic builds: > 1 repeats the fit (warm caches)
#endif
template <bool SMALL>
__device__ __forceinline__ void fit_slot(const FitArgs &A, unsigned char *dyn_lds,
                                         FitShared &sm);

// SMALL: histories of <= kMergeMax trials, the whole fit in LDS; a separate
// instantiation without the large-history paths keeps the code a CU pair
// runs (and shares one instruction cache for) small
template <bool SMALL>
__global__ __launch_bounds__(kFitThreads) void k_fit(FitArgs A, HistPatch P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_lds[];
  __shared__ FitShared sm;
  if (P.n_rows > 0 || P.n_loss > 0) {
    // the history update that came with this call (tpe_plan_update_history,
    // deferred into the fit): each block writes its hp's new rows and every
    // new loss -- the blocks of other hps write the same loss values -- and
    // reads them back after its own barrier
    const int hp = blockIdx.x;
    double *vals = const_cast<double *>(A.vals);
    uint8_t *act = const_cast<uint8_t *>(A.active);
    double *losses = const_cast<double *>(A.losses);
    for (int r = threadIdx.x; r < (int)P.n_rows; r += blockDim.x) {
      vals[(int64_t)hp * P.ld + P.row0 + r] = P.vals[hp * (int)P.n_rows + r];
      act[(int64_t)hp * P.ld + P.row0 + r] = P.active[hp * (int)P.n_rows + r];
    }
    for (int i = threadIdx.x; i < (int)P.n_loss; i += blockDim.x) losses[P.loss0 + i] = P.losses[i];
    __threadfence_block();
    __syncthreads();
  }
  for (int rep = 0; rep < TPE_FIT_REPS; ++rep) {
    fit_slot<SMALL>(A, dyn_lds, sm);
    __syncthreads();
  }
}

template <bool SMALL>
__device__ __forceinline__ void fit_slot(const FitArgs &A, unsigned char *dyn_lds,
                                         FitShared &sm) {
  const int hp = blockIdx.x, side = blockIdx.y;  // side 0 = below ("good")
  const int64_t slot = 2 * (int64_t)hp + side;
  const tpe_hp H = A.hps[hp];
  FitCtx C;
  C.lds = dyn_lds;
  unsigned char *gsb = A.sortbuf + slot * 16 * A.scap;
  C.gkeys = reinterpret_cast<uint64_t *>(gsb);
  C.gpa = reinterpret_cast<uint32_t *>(gsb + 8 * A.scap);
  C.gpb = C.gpa + A.scap;
  STAMP(0);
#ifdef TPE_STAMPS
  const unsigned long long clk0 = clock64();  // shader clock: SCLK = cycles / wall time
#endif
  // histories of <= kPreN trials: every trial's value and activity is loaded
  // into registers up front (in flight during the split), so the gather
  // below needs no memory round trip; the losses' sort keys come from the
  // split's copy
  const bool pre = SMALL || A.n <= kPreN;
  constexpr int PER = SMALL ? 1 : kGatherRows;  // rows: trial c0 + u * 1024 + t
  const double *row = A.vals + (int64_t)hp * A.ld;
  const uint8_t *arow = A.active + (int64_t)hp * A.ld;
  double prv[PER];
  uint8_t pac[PER];
  if (pre) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int64_t j = min<int64_t>((int64_t)u * kFitThreads + threadIdx.x, A.n - 1);
      pac[u] = j >= 0 ? arow[j] : 0;
      prv[u] = j >= 0 ? row[j] : 0.0;
    }
  }
  const Split t = compute_split<SMALL>(A, C, sm);
  __syncthreads();
  STAMP(1);

  // ---- gather this side's observations in tid order (tpe.py:629-636):
  // chunks of PER * 1024 trials, trial c0 + u * 1024 + t in thread t's row u
  // (coalesced loads); the order inside a chunk is u-major, so a selected
  // trial's slot is the chunk base + the trials selected in earlier (row,
  // wave) pairs + its rank in its wave's ballot of row u.  The chunks move
  // raw values only; the transform (a float64 log for the log families) and
  // the sort keys run afterwards over the m gathered values, densely (a
  // conditional hp's side is a sparse subset of the rows: transformed in
  // place, every row with one selected lane would cost the whole wave a log)
  const bool cat = H.family == TPE_CAT;
  // observations: LDS above the keys when the history is small (no global
  // stores in flight at the barriers that follow), else slot scratch
  double *ob = (SMALL || A.n <= kMergeMax)
                   ? reinterpret_cast<double *>(dyn_lds + kOffKeys + 8 * kMergeMax)
                   : A.ob + slot * A.kcap;
  uint64_t *lk = reinterpret_cast<uint64_t *>(dyn_lds + kOffKeys);
  // the split's loss keys (compute_split: LDS up to kSortCap trials)
  const uint64_t *lkey = (SMALL || A.n <= kSortCap) ? lk : C.gkeys;
  int m = 0;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int64_t c0 = 0; c0 < A.n; c0 += PER * kFitThreads) {
    if (!pre) {  // all loads issued before any use: one memory round trip per chunk
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int64_t j = min<int64_t>(c0 + (int64_t)u * kFitThreads + threadIdx.x, A.n - 1);
        pac[u] = arow[j];
        prv[u] = row[j];
      }
    }
    uint32_t fm = 0u;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int64_t j = c0 + (int64_t)u * kFitThreads + threadIdx.x;
      const bool f = j < A.n && pac[u] && (is_below(t, lkey[j], (uint32_t)j) == (side == 0));
      fm |= f ? 1u << u : 0u;
      const uint64_t b = __ballot(f);
      if (lane == 0) sm.gcnt[u][wv] = (int)__popcll(b);
    }
    STAMP(35);
    __syncthreads();
    // (row, wave) exclusive prefix of the counts, by wave 0: lane l takes the
    // consecutive entries [l * E, l * E + E) of the row-major table
    if (wv == 0) {
      constexpr int NE = PER * kFitWaves, E = (NE + 63) / 64;
      const int *gc = &sm.gcnt[0][0];
      int *gb = &sm.gbase[0][0];
      int c[E], loc = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int q = lane * E + e;
        c[e] = q < NE ? gc[q] : 0;
        loc += c[e];
      }
      int acc = wave_incl_scan(loc) - loc;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int q = lane * E + e;
        if (q < NE) gb[q] = acc;
        acc += c[e];
      }
    }
    __syncthreads();
    STAMP(36);
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const bool f = (fm >> u) & 1u;
      const uint64_t b = __ballot(f);
      if (f) ob[m + sm.gbase[u][wv] + (int)__popcll(b & lanemask_lt())] = prv[u];
    }
    m += sm.gbase[PER - 1][kFitWaves - 1] + sm.gcnt[PER - 1][kFitWaves - 1];
    __syncthreads();  // (the next chunk's counts reuse gcnt / gbase; ob complete)
  }
  // transform in place, sort keys, and the block's count below the prior mean
  // and key-bit reductions (bits equal over all keys: kand == kor there)
  const double ofloor = obs_floor(H.obs_transform, H.low);
  int nlt = 0;
  uint64_t kand = ~0ull, kor = 0ull;
  for (int i = threadIdx.x; i < m; i += kFitThreads) {
    const double v = obs_transform(ob[i], H.obs_transform, ofloor);
    ob[i] = v;
    nlt += (v < H.prior_mu) ? 1 : 0;
    const uint64_t k = cat ? (uint64_t)(int64_t)v : sort_key(v);
    kand &= k;
    kor |= k;
    if (i < kSortCap) lk[i] = k;
    else C.gkeys[i] = k;
  }
  {
    const int nw = wave_sum(nlt);
    const uint64_t aw = wave_and(kand), ow = wave_or(kor);
    if (lane == 0) { sm.gx[0][wv].nlt = nw; sm.gx[0][wv].kand = aw; sm.gx[0][wv].kor = ow; }
    __syncthreads();
    nlt = 0;
#pragma unroll
    for (int i = 0; i < kFitWaves; ++i) {
      const GatherEx &e = sm.gx[0][i];
      nlt += e.nlt;
      kand &= e.kand;
      kor |= e.kor;
    }
  }
  STAMP(37);
  const uint64_t vary = kand ^ kor;
  const bool lds_sort = SMALL || m <= kSortCap;
  if (!lds_sort) {  // the sort runs on the global key copy
    __syncthreads();
    for (int i = threadIdx.x; i < kSortCap; i += blockDim.x) C.gkeys[i] = lk[i];
  }
  __syncthreads();
  STAMP(2);

  uint32_t *cnt = reinterpret_cast<uint32_t *>(dyn_lds + kOffCnt);
  uint32_t *run = reinterpret_cast<uint32_t *>(dyn_lds + kOffRun);
  bool done = false;
  if constexpr (!SMALL) {
    // categorical over few bins, more observations than the merge sort's:
    // no sort (fit_categorical_counting)
    if (lds_sort && cat && H.upper <= kCatFastBins && m > kMergeMax) {
      STAMP(3);
      fit_categorical_counting(A, C, sm, H, slot, m);
      done = true;
    }
  }
  if (done) {
  } else if (lds_sort) {
    const uint16_t *perm = block_sort_perm<uint16_t, SMALL>(
        lk, reinterpret_cast<uint16_t *>(dyn_lds + kOffPosA),
        reinterpret_cast<uint16_t *>(dyn_lds + kOffPosB), m, vary, cnt, run, sm);
    STAMP(3);
    if (cat) fit_categorical<uint16_t>(A, C, sm, H, slot, lk, perm, m);
    else if (SMALL) fit_continuous<true, uint16_t, 1>(A, C, sm, H, slot, ob, perm, m, nlt);
    else if (m + 1 <= kMixLds) fit_continuous<true, uint16_t>(A, C, sm, H, slot, ob, perm, m, nlt);
    else fit_continuous<false, uint16_t>(A, C, sm, H, slot, ob, perm, m, nlt);
  } else if (!SMALL) {
    const uint32_t *perm =
        block_sort_perm<uint32_t>(C.gkeys, C.gpa, C.gpb, m, vary, cnt, run, sm);
    STAMP(3);
    if (cat) fit_categorical<uint32_t>(A, C, sm, H, slot, C.gkeys, perm, m);
    else fit_continuous<false, uint32_t>(A, C, sm, H, slot, ob, perm, m, nlt);
  }
  __syncthreads();
  STAMP(10);
#ifdef TPE_STAMPS
  if (threadIdx.x == 0 && blockIdx.z == 0)
    g_stamps[(2 * blockIdx.x + blockIdx.y) & 511][9] = clock64() - clk0;
#endif
}

// operator-level split (tpe_split): same threshold, then the mask
__global__ __launch_bounds__(kFitThreads) void k_split(FitArgs A, uint8_t *__restrict__ below) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_lds[];
  __shared__ FitShared sm;
  FitCtx C;
  C.lds = dyn_lds;
  C.gkeys = reinterpret_cast<uint64_t *>(A.sortbuf);
  C.gpa = reinterpret_cast<uint32_t *>(A.sortbuf + 8 * A.scap);
  C.gpb = C.gpa + A.scap;
  const Split t = compute_split(A, C, sm);
  for (int64_t j = threadIdx.x; j < A.n; j += blockDim.x)
    below[j] = is_below(t, sort_key(A.losses[j]), (uint32_t)j) ? 1 : 0;
}

// constants of explicitly given mixtures (operator-level tpe_score/lpdf)
__global__ __launch_bounds__(256) void k_prep(const tpe_hp *__restrict__ hps,
                                              const double *__restrict__ mw,
                                              const double *__restrict__ mmu,
                                              const double *__restrict__ msig,
                                              MixInfo *__restrict__ info, Coef *__restrict__ coef,
                                              Coef32 *__restrict__ coef32,
                                              CoefM *__restrict__ coefm,
                                              CoefM8 *__restrict__ coefm8,
                                              float4 *__restrict__ coefe, int64_t kcap,
                                              double *__restrict__ scratch) {
  __shared__ FitShared sm;
  const int hp = blockIdx.x, side = blockIdx.y;
  const int64_t slot = 2 * (int64_t)hp + side;
  const int K = info[slot].K;
  __syncthreads();
  prep_slot(hps + hp, slot, K, mw + slot * kcap, mmu + slot * kcap, msig + slot * kcap, info, coef,
            coef32, coefm, coefm8, coefe, kcap, scratch + slot * kcap, sm);
}

// ------------------------------------------------------------------------
#ifdef TPE_STAMPS
}  // namespace tpe
extern "C" int tpe_debug_stamps(unsigned long long *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(tpe::g_stamps), sizeof(tpe::g_stamps)) == hipSuccess
             ? 0 : -5;
}
namespace tpe {
#endif

bool fit_small(int64_t n) { return n <= kMergeMax; }

const void *fit_kernel_fn(bool small) {
  return small ? reinterpret_cast<const void *>(&k_fit<true>)
               : reinterpret_cast<const void *>(&k_fit<false>);
}

hipError_t launch_fit(const FitArgs &a, int32_t n_hp, hipStream_t st, const HistPatch *patch) {
  if (n_hp <= 0) return hipSuccess;
  static const HistPatch none{};
  const HistPatch &P = patch ? *patch : none;
  if (fit_small(a.n)) k_fit<true><<<dim3(n_hp, 2), kFitThreads, kFitLds, st>>>(a, P);
  else k_fit<false><<<dim3(n_hp, 2), kFitThreads, kFitLds, st>>>(a, P);
  return hipGetLastError();
}

hipError_t launch_split(const FitArgs &a, uint8_t *below, hipStream_t st) {
  k_split<<<1, kFitThreads, kFitLds, st>>>(a, below);
  return hipGetLastError();
}

hipError_t launch_prep(const tpe_hp *hps, int32_t n_hp, const double *mw, const double *mmu,
                       const double *msig, MixInfo *info, Coef *coef, Coef32 *coef32,
                       CoefM *coefm, CoefM8 *coefm8, float4 *coefe, int64_t kcap,
                       double *scratch, hipStream_t st) {
  if (n_hp <= 0) return hipSuccess;
  k_prep<<<dim3(n_hp, 2), 256, 0, st>>>(hps, mw, mmu, msig, info, coef, coef32, coefm, coefm8,
                                        coefe, kcap, scratch);
  return hipGetLastError();
}

}  // namespace tpe
