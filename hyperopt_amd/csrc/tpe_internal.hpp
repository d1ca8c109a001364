// tpe_internal.hpp -- shared host/device declarations of the TPE engine.
// Not part of the ABI (include/tpe_engine.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tpe_engine.h"

namespace tpe {

constexpr double kEPS = 1e-12;  // hyperopt/tpe.py:25
constexpr int kFitThreads = 1024;
constexpr int kScoreThreads = 256;
constexpr int kMaxLeaves = 160;  // numpy pairwise leaves per 8192 chunk (<=128)

// Per (hp, side) mixture slot, written by k_fit / k_prep.
// scoring kernel instantiations (lpdf kinds)
// KIND_LAT: a quantized hp scored on its value lattice (k_lattice) -- the
// scoring launch only looks its candidates up (run_level picks it per level)
// KIND_LSE_G1 / KIND_LSE_L1: the log-sum-exp kinds on one-row (64-candidate)
// tiles, picked by run_level when two-row tiles would give the CUs too few,
// unevenly shared blocks
// KIND_LSE_GW / KIND_LSE_LW: the log-sum-exp kinds on value-bucketed
// candidates with the block skip and the wave-wide exponent: every wave owns
// its own 128 candidates and all of both mixtures' live components (no
// cross-wave partials); a block is 8 such wave tiles
// KIND_LSE_GW1 / KIND_LSE_LW1: the same wave tiles with one candidate row
// (64 candidates per wave): for suggestions of at most kWaveRowSplitMax
// candidates, whose levels are too small to fill the GPU -- the waves of
// dense value windows (most live component blocks) then carry half the pairs
// and end the launch sooner (run_level, chosen by the per-suggestion
// candidate count, so a batch and every shard take the same tiles)
enum { KIND_LSE_G = 0, KIND_LSE_L = 1, KIND_ERF_G = 2, KIND_ERF_L = 3, KIND_CAT = 4,
       KIND_LAT = 5, KIND_LSE_G1 = 6, KIND_LSE_L1 = 7, KIND_LSE_GW = 8, KIND_LSE_LW = 9,
       KIND_LSE_GW1 = 10, KIND_LSE_LW1 = 11 };
constexpr int64_t kWaveRowSplitMax = (int64_t)1 << 18;

__host__ __device__ constexpr bool kind_lse(int k) {
  return k == KIND_LSE_G || k == KIND_LSE_L || k == KIND_LSE_G1 || k == KIND_LSE_L1 ||
         k == KIND_LSE_GW || k == KIND_LSE_LW || k == KIND_LSE_GW1 || k == KIND_LSE_LW1;
}
__host__ __device__ constexpr bool kind_logn(int k) {
  return k == KIND_LSE_L || k == KIND_LSE_L1 || k == KIND_LSE_LW || k == KIND_LSE_LW1 ||
         k == KIND_ERF_L;
}
// wave-tile log-sum-exp kinds (value-bucketed candidates, block skip)
__host__ __device__ constexpr bool kind_wave_lse(int k) {
  return k == KIND_LSE_GW || k == KIND_LSE_LW || k == KIND_LSE_GW1 || k == KIND_LSE_LW1;
}

__host__ __device__ inline int score_kind(const tpe_hp &h) {
  if (h.family == TPE_CAT) return KIND_CAT;
  const bool lg = h.family == TPE_LGMM;
  if (h.flags & TPE_HAS_Q) return lg ? KIND_ERF_L : KIND_ERF_G;
  return lg ? KIND_LSE_L : KIND_LSE_G;
}

// candidate rows (per lane) of a scoring tile of the kind: 64 * rows candidates
__host__ __device__ constexpr int tile_rows(int kind) {
  return (kind == KIND_ERF_G || kind == KIND_ERF_L || kind == KIND_LSE_G1 || kind == KIND_LSE_L1 ||
          kind == KIND_LSE_GW1 || kind == KIND_LSE_LW1)
             ? 1
         : (kind == KIND_CAT || kind == KIND_LAT) ? 4 : 2;
}
// waves of a block holding their own candidates (wave tiles), else 1 (the
// block's waves split the components of the same candidates).  The lookup
// kinds (categorical, value lattice) have no components to split: every wave
// takes its own 256 candidates (one-wave tiles left 7 of 8 waves idle, and
// a 1e6-candidate slot 3906 blocks instead of 489).
__host__ __device__ constexpr int tile_waves(int kind) {
  return (kind_wave_lse(kind) || kind == KIND_CAT || kind == KIND_LAT) ? 8 : 1;
}
// candidates of one scoring block of the kind
__host__ __device__ constexpr int tile_cands(int kind) {
  return 64 * tile_rows(kind) * tile_waves(kind);
}
constexpr int kMaxGroups = 8;  // runs of one lpdf kind per launch (a level has <= 7)
constexpr int kNumCUs = 256;   // MI355X (gfx950): 8 XCDs x 32 CUs

struct MixInfo {
  int32_t K;        // components (categorical: upper)
  int32_t kind;     // 0 LSE, 1 ERF, 2 CAT
  double p_accept;  // truncation mass (tpe.py:130-136, 273-276)
  double log_pacc;  // log(p_accept) subtracted by the quantized lpdf
  double wsum;      // sum of weights (sampler CDF total)
  int32_t probe;    // LSE: a widest component (the Parzen prior), whose term
                    // lower-bounds every candidate's log-sum-exp maximum; -1: none
  // LSE tables of >= kRangeMinK components: the largest c (e.z) and the
  // smallest a^2 (|e.w|) of the block envelopes outside the probe's block, as
  // stored (rounded outward); env_amin = 0: not computed.  A wave tile's live
  // blocks other than the probe's then lie within sqrt((cmax - thr) / amin)
  // of its candidate window (lse_chunks_shifted's range search)
  float env_cmax;
  float env_amin;
  int32_t pad2;
};
constexpr int kRangeMinK = 2048;

// Log-sum-exp block envelope (LSE kinds): in the spare w-row of every
// coefficient block, 4 floats bounding the block's terms
//   [0] min mu', [1] max mu' (rounded outward), [2] max c (log2 units,
//   rounded up), [3] min a^2 (rounded down),
// so t_k(y') <= c_max - a2_min * dist(y', [mu'_lo, mu'_hi])^2 for every
// component k of the block.  The scoring kernel skips a block whose bound,
// over the wave's candidate range, is below (lower bound of the lane maxima)
// - D - 1 with D = kLseDeadBase + ceil(log2 K): each skipped term is below
// 2^-(D+1) of the lane's largest term (>= 1/2 of the sum), so all skipped
// terms of a K-component mixture move the lpdf by at most K * 2^-D <=
// 2^-kLseDeadBase ~ 1.5e-8 relative -- 67x inside the 1e-6 parity bar.
// (Round 4: 30 -> 26, a narrower live halo: config 4 277 -> 270 ms,
// config 3 -1.6 %, config 5 -0.8 %, same box.)
constexpr float kLseDeadBase = 26.0f;
// census counters (tpe_plan_census_n): quantized total / live / evaluated,
// log-sum-exp total / one-exponent evaluated / evaluated / evaluated in the
// block-local fp32 per-group-lift form / one-exponent pairs of a wave's
// second attempt (re-centred exponent) / one-exponent pairs of wide blocks
// (the fp64 loop of mode 3) / one-exponent pairs evaluated in the moment
// form of their chunk (CoefM, 16-wide, or CoefM8, 8-wide) / of those, the
// 8-wide ones / of those, the 16-wide degree-15 ones (CoefMH)
constexpr int kCensus = 12;

// Per-component scoring coefficients (make_coef, tpe_device.hpp), 4 fields:
//   LSE: x = alpha, y = beta, z = gamma (t = alpha + y'(beta + gamma y'))
//   ERF: x = mu, y = 1/max(sqrt2*sigma, EPS), z = w, w = dead-zone half-width
//   CAT: x = log p
// A slot's table (kcap components, a multiple of kCoefBlock) is stored in
// blocks of kCoefBlock components, field-major within a block
// ([x0..x7][y0..y7][z0..z7][w0..w7], 256 B): a scoring wave fetches one
// block's three log-sum-exp fields with three 64-B scalar loads.
struct __attribute__((aligned(32))) Coef {
  double x, y, z, w;
};
constexpr int kCoefBlock = 8;
// offset (in doubles) of field f (0..3 = x, y, z, w) of component k of a table
__host__ __device__ constexpr int64_t coef_off(int64_t k, int f) {
  return (k / kCoefBlock) * (4 * kCoefBlock) + f * kCoefBlock + (k % kCoefBlock);
}
// with_w false (log-sum-exp kinds): the w-row holds the block envelope instead
__device__ __forceinline__ void store_coef(Coef *table, int64_t k, const Coef &c,
                                           bool with_w = true) {
  double *t = reinterpret_cast<double *>(table);
  t[coef_off(k, 0)] = c.x;
  t[coef_off(k, 1)] = c.y;
  t[coef_off(k, 2)] = c.z;
  if (with_w) t[coef_off(k, 3)] = c.w;
}

// The same log-sum-exp terms per block of kCoefBlock components in
// block-local fp32 form (prune mode 3, tpe_score.hip lse_chunks_shifted):
//   t_k = A + alpha_k + u (beta_k + gamma_k u),  u = y' - center,
// center = the block's mu' midpoint (fp64), A = an integer near the block's
// largest alpha (so alpha_k stays small and exact to ~2^-24 absolute).  The
// form is exact to fp32 rounding of O(1) parts only while every component
// sits within ~1 of its own scale from the centre (a_k^2 (mu'_k - centre)^2
// <= kF32Spread): blocks that straddle a gap between tight clusters (small
// sigma, wide block) are flagged -- the sign bit of their envelope's a^2
// (kLseDeadBase) -- and keep the fp64 quadratic.  One 128-B block = two 64-B
// scalar loads.
constexpr double kF32Spread = 1.0;
struct __attribute__((aligned(128))) Coef32 {
  double center;
  float base;
  float pad0;
  float a[kCoefBlock], b[kCoefBlock], c[kCoefBlock];
  float pad1[4];
};
static_assert(sizeof(Coef32) == 128, "two 64-B scalar loads");

// Moment form of a 16-component chunk (prune mode 3, one-exponent wave
// tiles).  When the chunk's components share one sigma -- every component
// whose adaptive-Parzen sigma sits at the prior_sigma / min(100, 1 + N)
// floor (tpe.py:440-456), the common case of long histories -- its terms at
// y' = centre + v factor as
//   sum_k 2^(t_k) = 2^(T* - a^2 v^2) * sum_k rho_k exp(q_k v),
//   T_k = t_k(centre), T* = max_k T_k, rho_k = 2^(T_k - T*), q_k = 2 a^2 ln2 d_k,
//   d_k = mu'_k - centre,
// and exp(q_k v) is its Taylor polynomial of degree kMomDeg: the chunk's 16
// exponentials become one exp2 and a polynomial in v with the fixed
// coefficients m_j = sum_k rho_k q_k^j / j!.  Truncation: each term's
// relative error is <= x^(kMomDeg+1) / (kMomDeg+1)! e^x with x = |v| xh,
// xh = max_k |q_k|; a wave takes the form for a chunk only while its whole
// candidate range has x <= kMomXLim (<= 7.1e-9 relative).  xh = +inf marks
// a chunk whose sigmas differ (or non-finite terms): never taken.
// (tools/moment_error.py emulates it against the oracle.)  64 B = one
// scalar load.
constexpr int kMomChunk = 16;
constexpr int kMomDeg = 9;
constexpr float kMomXLim = 0.65f;
constexpr float kMomXCap = 2.5f;          // beyond: never (the Horner sum's conditioning)
constexpr float kMomLog2Fact = 21.79106f; // log2((kMomDeg + 1)!) = log2(10!)
struct __attribute__((aligned(64))) CoefM {
  double center;   // mu' midpoint of the chunk (fp64)
  float base;      // integer near T* (A - M is exact)
  float cm;        // T* - base
  float gam;       // -a^2 (log2 units), the shared quadratic coefficient
  float m[kMomDeg + 1];
  float xh;        // max_k |q_k| (nats per unit v), rounded up; +inf: not eligible
};
static_assert(sizeof(CoefM) == 64, "one 64-B scalar load");
static_assert(kMomChunk == 2 * 8, "a moment chunk is two coefficient blocks");
// moment-table entries per slot (kcap is a multiple of kCoefBlock)
__host__ __device__ constexpr int64_t mom_stride(int64_t kcap) {
  return (kcap + kMomChunk - 1) / kMomChunk;
}

// The same moment form per coefficient block of 8 components with a
// degree-15 polynomial (CoefM8): for mixtures of ~1e3 components (configs 2,
// 3 and 5: neighbour gaps ~1e-2 against a sigma floor of 0.1) a 16-component
// chunk spans too much of sigma for the degree-9 bound (xh ~ 7.5, almost no
// chunk qualifies), while 8 components at degree 15 cover ~60-90 % of the
// live blocks (tools/moment_error.py MOM_CH=8 MOM_P=15: 1.0e-7 max relative
// lpdf error against the oracle).  The per-plan width (tpe_engine.hip
// mom_width): 16 for mixtures of >= kMom16MinK components, else 8 from the
// one-exponent size up; the scoring kernels are instantiated per width, so the
// 16-wide kernel's register allocation is the round-5 one.  A block of 8 is
// one Coef32 block: the same centre (mu' midpoint) and base.  Truncation
// tau(x) = x^16 / 16! e^x; taken for x <= kMom8XLim (tau <= 5.7e-9) or by the
// weighted criterion as the 16-wide form.  128 B = two 64-B scalar loads.
constexpr int kMom8Deg = 15;
constexpr float kMom8XLim = 1.85f;          // tau(1.85) = 5.7e-9, kMomXLim's budget
constexpr float kMom8Log2Fact = 44.25014f;  // log2(16!)
constexpr int64_t kMom16MinK = 4000;
struct __attribute__((aligned(128))) CoefM8 {
  double center;   // mu' midpoint of the block (fp64), as Coef32::center
  float xh;        // max_k |q_k| (nats per unit v), rounded up; +inf: not eligible
  float base;      // integer near T*
  float cm;        // T* - base
  float gam;       // -a^2 (log2 units)
  float m[kMom8Deg + 1];
  float pad[8];
};
static_assert(sizeof(CoefM8) == 128, "two 64-B scalar loads");
// 16-wide plans also keep the degree-15 form of every 16-component chunk
// (CoefM8 layout, one entry per chunk: "CoefMH"), taken for the chunks the
// degree-9 form leaves out -- waves whose candidate window is wide (sparse
// tails of the draw), where x exceeds kMomXLim and the chunk weighs too much
// for the weighted criterion: config 4's 12 % of evaluated pairs in the
// block-local pair form (3.3 VALU per pair against ~0.9 for a degree-15
// chunk of 16)

struct Partial {  // == tpe_result layout
  double score;
  double value;
  int64_t index;
  int32_t active;
  int32_t pad;
};
static_assert(sizeof(Partial) == sizeof(tpe_result), "layout");

constexpr int kInlineSeeds = 8;  // suggestion seeds passed by value

// Value lattice of a bounded quantized hp: every drawn candidate is j * q for
// an integer j in [j0, j0 + R) (GMM: low <= x < high before rounding, LGMM:
// exp of such a draw; one index of margin on each side).  Its lpdf pair is
// kept at lat[off + j - j0] (k_lattice).  R = 0: no lattice.
struct LatInfo {
  int64_t j0;
  int64_t off;
  int32_t R;
  int32_t pad;
};
// k_lattice keeps one partial sum per 16-component chunk of both mixtures
// of a point in LDS: mixtures of up to 16 * kLatChunks / 2 components
constexpr int kLatChunks = 8192;
constexpr int64_t kLatMaxR = (int64_t)1 << 22;  // lattice points per hp

struct ScoreArgs {
  uint64_t seed_inline[kInlineSeeds];
  int32_t n_inline_seeds;
  const tpe_hp *hps;
  const int32_t *level_hps;  // hp ids of this launch (blockIdx.y)
  const int32_t *cond_parent;
  const int32_t *cond_branch;
  const MixInfo *info;       // [2*P]
  const Coef *coef;          // [2*P][kcap]
  const Coef32 *coef32;      // [2*P][kcap / kCoefBlock] block-local fp32 LSE terms
  const CoefM *coefm;        // [2*P][mom_stride] moment form of 16-component chunks
  const CoefM8 *coefm8;      // [2*P][kcap / kCoefBlock] moment form of 8-component blocks
  const CoefM8 *coefmh;      // [2*P][mom_stride] degree-15 form of 16-component chunks
  const float4 *coefe;       // [2*P][kcap / kCoefBlock] log-sum-exp block envelopes, compact
  const double *mw, *mmu, *msig;  // [2*P][kcap] (sampler reads side 0)
  const uint64_t *seeds;     // [S]
  const double *cand;        // candidates [S][n_slots][n_cand] (drawn or external)
  const int32_t *cand_pos;   // optional: original position of each (sorted) candidate
  double *out_lb, *out_la;   // optional per-candidate lliks (ext only)
  Partial *results;          // [S][P]
  Partial *partial;          // [S][P][pstride] candidate-tile argmax records
  uint32_t *ticket;          // [S][P] tile arrival counters (zero between launches)
  int64_t kcap;
  int64_t n_cand;
  int64_t cand_begin;
  int64_t cand_sstride;      // candidate elements per suggestion in `cand`
  int32_t cand_slot0;        // slot of blockIdx.y == 0 within the candidate buffer
  int32_t pstride;           // partial records per (s, hp)
  int32_t n_hp;
  int32_t n_slots;            // hps of this launch
  int32_t n_suggest;         // grid.y
  // scoring grid: kind groups of consecutive slots (set_score_groups)
  int32_t n_groups;
  int32_t grp_kind[kMaxGroups];
  int32_t grp_slot0[kMaxGroups];
  int32_t grp_tiles[kMaxGroups];       // tiles per slot of the group
  int32_t grp_block0[kMaxGroups + 1];  // first block of each group; [n_groups] = total
  int32_t grp_slots[kMaxGroups];       // slots of each group
  // active-slot grids (conditional levels): a launch has rows for at most
  // slot_rows slots per suggestion (the most its hps can have active
  // together, active_bound) instead of one per slot; row j takes the j-th
  // active slot (active_slot), so the inactive branches of a choice cost no
  // blocks.  compact = 0: row j is slot j (every slot has its rows).
  int32_t compact;
  int32_t slot_rows;                   // draw / bucket grids: rows over the level's slots
  int32_t force_active;      // ignore conditions (operator-level scoring)
  int32_t accumulate;        // merge with results of an earlier candidate chunk
  unsigned long long *census;  // optional [kCensus] pair counters (tpe_plan_census)
  int32_t lse_pos;           // LSE slots' candidates are value-bucketed (cand_pos valid)
  int32_t sort_log2;         // their sort blocks: 1 << sort_log2 candidates (sort_log2_for)
  int32_t lse_prune;         // skip log-sum-exp blocks of exact-zero terms (needs lse_pos)
  int32_t lse_shift_min;     // lse_prune 2: smallest mixture (components) for one wave exponent
  int32_t lse_f32;           // unpruned log-sum-exp slots also take the block-local fp32
                             // pairs (prune mode 3's arithmetic on small draws)
  int32_t lse_mom;           // prune mode 3 wave tiles take the moment form of eligible
                             // chunks: 16 (CoefM), 8 (CoefM8, blocks) or 0 (TPE_MOMENT=0,
                             // or no table written by the last fit)
  int32_t lse_momh;          // with 16: the degree-15 chunk table (coefmh) is there too
  int32_t lookup_draw;       // the sorted draw leaves the lookup slots (categorical, value
                             // lattice) unwritten and the scoring tile draws them itself,
                             // for below mixtures of 1 .. kFuseTab components (lookup_inline)
  int64_t lookup_seg;        // candidates per lookup-scan block (set by the lookup launch)
  int32_t l2_warm;           // scoring tiles touch their mixtures' coefficient lines first
  int32_t lse_tight;         // wave tiles tighten the skip threshold from the top block (default 1)
                             // (one load per 128-B line; TPE_L2_WARM=1, A/B; default off)
  int32_t tile_draw;         // tiny unsorted draws: every tile draws its own candidates
                             // (k_score_tdraw; no k_draw launch, nothing written)
  const LatInfo *lat_info;   // [P] value lattices (KIND_LAT slots)
  const double2 *lat;        // lattice (lpdf below, lpdf above) pairs
  // a tile_draw launch that ends its call (pub_flag non-null): the last of its
  // pub_events final records copies all pub_words words of results into the
  // pinned pub_dst and then stores pub_seq into *pub_flag -- k_publish's
  // work without its launch (pub_ticket: a counter, zero between launches)
  uint64_t *pub_dst;
  uint64_t *pub_flag;
  uint32_t *pub_ticket;
  uint64_t pub_seq;
  int32_t pub_words;
  int32_t pub_events;
};

// Arguments of the fit kernels (tpe_fit.hip), one block per (hp, side) slot.
struct FitArgs {
  const tpe_hp *hps;
  const double *vals;        // [P][ld] history values (tid order)
  const uint8_t *active;     // [P][ld]
  const double *losses;      // [n]
  int64_t n;
  int64_t ld;                // row stride of vals / active (the plan's trial capacity)
  int32_t n_below;
  int32_t lf;
  int32_t pad0;
  double prior_weight;
  const double *pprior;
  double *mw, *mmu, *msig;   // [2P][kcap] fitted mixtures
  MixInfo *info;             // [2P]
  Coef *coef;                // [2P][kcap]
  Coef32 *coef32;            // [2P][kcap / kCoefBlock]
  CoefM *coefm;              // [2P][mom_stride(kcap)] (null: not written)
  CoefM8 *coefm8;            // [2P][kcap / kCoefBlock] (null: not written; at most one of the two)
  CoefM8 *coefmh;            // [2P][mom_stride(kcap)] degree-15 16-wide form (with coefm)
  float4 *coefe;             // [2P][kcap / kCoefBlock] compact envelopes (store_lse_envelope)
  int64_t kcap;
  double *ob;                // [2P][kcap] scratch: observations of the slot
  double *tmp;               // [2P][kcap] scratch (may alias ob)
  unsigned char *sortbuf;    // [2P][16 * scap] global sort keys + permutations
  int64_t scap;              // >= n
};

// ---- launch wrappers (tpe_fit.hip / tpe_kernels.hip) ----
hipError_t launch_split(const FitArgs &a, uint8_t *below, hipStream_t st);
struct HistPatch;
// patch: history rows / losses the fit blocks write before they read the
// history (a deferred tpe_plan_update_history; null: none)
hipError_t launch_fit(const FitArgs &a, int32_t n_hp, hipStream_t st,
                      const HistPatch *patch = nullptr);
bool fit_small(int64_t n);                 // k_fit<true> (all-LDS variant) serves n trials
const void *fit_kernel_fn(bool small);     // k_fit's host stub (graph node lookup)
bool is_draw_kernel_fn(const void *f);     // one of k_draw's / k_draw_sorted's host stubs
bool is_sorted_draw_kernel_fn(const void *f);
const void *lattice_draw_kernel_fn();      // k_lattice<true> (lattice + fused draw)
hipError_t launch_prep(const tpe_hp *hps, int32_t n_hp, const double *mw,
                       const double *mmu, const double *msig, MixInfo *info,
                       Coef *coef, Coef32 *coef32, CoefM *coefm, CoefM8 *coefm8,
                       float4 *coefe, int64_t kcap, double *scratch, hipStream_t st);
// a level mixing wave-tile log-sum-exp groups with other kinds runs two
// launches: the other kinds on `side` between fork / join events (when side
// is given; st waits for the join), the log-sum-exp groups on st
// classes: bit mask of the launch classes to run (score_classes)
hipError_t launch_score(const ScoreArgs &a, bool has_erf, hipStream_t st,
                        hipStream_t side = nullptr, hipEvent_t ev_fork = nullptr,
                        hipEvent_t ev_join = nullptr, int classes = 7);
// the launch classes present among a launch's kind groups (bit c: class c;
// 0 wave-tile log-sum-exp, 1 lookups drawing their own candidates, 2 the rest)
int score_classes(const ScoreArgs &a);
// lpdf pairs of every lattice point of the first n_lat hps of a level
// (hps_of_level[], host arrays; one block of kLatThreads per point, up to
// kLatJobs hps per launch), written to lat_out
constexpr int kLatThreads = 256;
struct LatJob {  // one lattice hp of a k_lattice launch (kernel argument)
  tpe_hp H;
  LatInfo L;
  int32_t hp;
  int32_t pad;
};
constexpr int kLatJobs = 8;  // lattice hps per k_lattice launch
struct LatJobs {
  LatJob job[kLatJobs];
  // fused candidate draw (launch_lattice_draw): grid rows y >= n_jobs are
  // draw blocks d = (y - n_jobs) * gridDim.x + x of a (draw_gx, slots, S) grid
  int32_t n_jobs;
  int32_t draw_gx;
  int32_t draw_blocks;
  // compact: grid row y < n_jobs is the y-th of the level's first n_lat
  // (lattice) slots active in some suggestion, its descriptor read from
  // A.hps / A.lat_info (job[] unused); one launch for every lattice hp
  int32_t compact;
  int32_t n_lat;
  int32_t pad[3];
};
constexpr int kFuseTab = 32;  // below K of a draw fused into k_lattice (LDS table)
// lat_rows in (0, n_lat): compact rows (LatJobs::compact), one launch
hipError_t launch_lattice(const ScoreArgs &a, const int32_t *hps_of_level, const tpe_hp *hps,
                          const LatInfo *lat, int32_t n_lat, double2 *lat_out, hipStream_t st,
                          int32_t lat_rows);
// the same lattice launch with the level's candidate draw (draw args `a`, one
// candidate per thread, every below K <= kFuseTab) in extra blocks of it: the
// two only need the fitted mixtures and run side by side
hipError_t launch_lattice_draw(const ScoreArgs &a, const int32_t *hps_of_level, const tpe_hp *hps,
                               const LatInfo *lat, int32_t n_lat, double2 *lat_out,
                               hipStream_t st, int32_t lat_rows);
constexpr int kTabCap = 2048;  // below-mixture components of the LDS draw table
hipError_t launch_draw(const ScoreArgs &a, bool table, hipStream_t st);
// large draws: each block draws kSortedBlock consecutive candidates of a slot
// and, for the per-candidate log-sum-exp / erf kinds, writes them grouped
// into value buckets with their chunk positions in pos_out (tile coherence
// for the log-sum-exp block skip and the erf dead-zone skip); small_table:
// every below K <= kFuseTab
constexpr int kSortedBlock = TPE_SHARD_ALIGN;  // the largest sort block (LDS sizing)
// sort blocks of a launch: 1 << ScoreArgs::sort_log2 candidates -- 8192 for
// suggestions of > kWaveRowSplitMax candidates (two-row wave tiles: a wave's
// 128 candidates are 1/64 of its block's value quantiles, so its window and
// the live component blocks in it are half those of 4096-candidate blocks),
// 4096 below (fewer, shorter draw blocks for the small launches)
constexpr int kSortLog2Large = 13, kSortLog2Small = 12;
static_assert((1 << kSortLog2Large) == kSortedBlock, "largest sort block");
__host__ __device__ constexpr int sort_log2_for(int64_t n_total) {
  return n_total > kWaveRowSplitMax ? kSortLog2Large : kSortLog2Small;
}
// fast: every slot the launch draws is a bounded continuous one (low and
// high) whose below mixture fits the table, the rest lookup slots their tiles
// draw (lookup_draw) -- the kernel without the out-of-line draws
hipError_t launch_draw_sorted(const ScoreArgs &a, bool small_table, bool fast, int32_t *pos_out,
                              hipStream_t st);
static_assert(kSortedBlock == TPE_SHARD_ALIGN, "shard alignment is the sorted-draw block");
// given candidates src[slot][n_cand] (one suggestion) bucketed exactly as
// k_draw_sorted buckets its draws (tpe_plan_score_candidates_sorted)
hipError_t launch_sort_ext(const ScoreArgs &a, const double *src, int32_t *pos_out,
                           hipStream_t st);
// slots slot_begin .. n_slots-1 (the lattice slots before them are not bucketed)
hipError_t launch_bucket(const ScoreArgs &a, int32_t slot_begin, int32_t *pos_out, hipStream_t st);
// copy `bytes` (a multiple of 8) to the pinned host buffer dst, then store
// seq to the pinned word *flag (k_publish)
hipError_t launch_publish(const void *src, void *dst, size_t bytes, uint64_t *flag, uint64_t seq,
                          hipStream_t st);
hipError_t launch_merge(const int32_t *level_hps, int32_t n_slots,
                        int32_t n_suggest, int32_t n_hp, int32_t world,
                        const Partial *gathered, Partial *results,
                        hipStream_t st, Partial *out2 = nullptr);
hipError_t launch_sample(const tpe_hp *hp_dev, const double *mw,
                         const double *mmu, const double *msig,
                         const MixInfo *info, uint64_t seed, uint64_t stream,
                         int64_t offset, int64_t n, double *out,
                         hipStream_t st);

hipError_t launch_micro(int which, int blocks, int iters, double *sink, hipStream_t st);

// small history updates travel as kernel arguments (tpe_plan_update_history):
// one launch, no staging copy and no host synchronisation
constexpr int kPatchVals = 192;   // n_rows * P doubles / bytes
constexpr int kPatchLoss = 16;    // losses
struct HistPatch {
  int64_t row0, n_rows, loss0, n_loss, ld;
  int32_t P;
  int32_t pad;
  double vals[kPatchVals];        // [P][n_rows]
  double losses[kPatchLoss];
  uint8_t active[kPatchVals];     // [P][n_rows]
};
hipError_t launch_hist_patch(const HistPatch &h, double *vals, uint8_t *active, double *losses,
                             hipStream_t st);

// prior draws of whole suggestions (rand.suggest on the device): one block
// per suggestion walks the levels of the compiled space
struct PriorArgs {
  const tpe_hp *hps;
  int32_t n_hp;
  int32_t n_levels;
  const int32_t *level_hps;   // hp ids, level by level
  const int32_t *level_off;   // [n_levels + 1] (device)
  const int32_t *cond_parent;
  const int32_t *cond_branch;
  const double *pprior;
  const uint64_t *seeds;      // [S]
  Partial *results;           // [S][P]
};
hipError_t launch_prior(const PriorArgs &a, int32_t n_suggest, hipStream_t st);

}  // namespace tpe
