// tpe_engine.hip -- C ABI (include/tpe_engine.h) over the gfx950 kernels.
//
// Host-side ownership: a tpe_engine binds one device and owns an internal
// stream plus a cached one-hp "operator plan" used by the operator-level
// entry points; a tpe_plan owns the device-resident history, the fitted
// mixtures of every hp and the per-suggestion results.  No global state.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "tpe_internal.hpp"

using namespace tpe;

static int lse_shift_min();
static bool small_sort_on();
static int64_t chunk_budget();
// TPE_SIDE_STREAMS=1: the lattice launch and a mixed level's lookup launch
// run on auxiliary streams beside the draw / the wave-tile launch (fork and
// join events); default off: every launch in order on the suggest stream
// lookup slots drawn inside their scoring tiles (ScoreArgs::lookup_draw);
// TPE_LOOKUP_DRAW=0 writes them from the sorted draw instead (A/B)
static bool lookup_draw_on() {
  static const bool on = [] {
    const char *e = std::getenv("TPE_LOOKUP_DRAW");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}
// TPE_LOOKUP_FORK=0: a chunk's self-drawing lookup launch in order on the
// suggest stream instead of beside its draw
static bool lookup_fork_on() {
  static const bool on = [] {
    const char *e = std::getenv("TPE_LOOKUP_FORK");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}
// TPE_PUBLISH=0: results to the host by a runtime copy + stream synchronize
// instead of k_publish + a spin on its completion word
static bool publish_on() {
  static const bool on = [] {
    const char *e = std::getenv("TPE_PUBLISH");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}
// TPE_PATCH_DEFER=0: small history updates go out at once (k_hist_patch)
// instead of riding the next fit's arguments
static bool patch_defer_on() {
  static const bool on = [] {
    const char *e = std::getenv("TPE_PATCH_DEFER");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}
// TPE_TILE_DRAW=0: tiny unsorted draws by k_draw instead of their tiles
static bool tile_draw_on() {
  static const bool on = [] {
    const char *e = std::getenv("TPE_TILE_DRAW");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}
// TPE_PUBLISH_FUSE=0: a call whose last launch is a tile_draw scoring launch
// still ends with k_publish (default: that launch's last record publishes)
static bool publish_fuse_on() {
  static const bool on = [] {
    const char *e = std::getenv("TPE_PUBLISH_FUSE");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}
// TPE_L2_WARM=1: scoring tiles first touch every 128-B line of both
// mixtures' coefficient tables (round 2's L2 warm-up).  Off by default since
// round 6: the same-box A/B (gpurun_out/r6_05) gave config 4 127.3 -> 124.2 ms
// and config 5 543 -> 536 ms per step without it -- the waves' first envelope
// reads waited on those loads, and the tables are L2-resident after the first
// blocks anyway
// TPE_TIGHTEN=0: wave tiles keep lse_window's skip threshold (no tightening
// from the block of the highest bound) -- A/B
static bool tighten_on() {
  static const bool on = [] {
    const char *e = std::getenv("TPE_TIGHTEN");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}
static bool l2_warm_on() {
  static const bool on = [] {
    const char *e = std::getenv("TPE_L2_WARM");
    return e && std::atoi(e) != 0;
  }();
  return on;
}
static bool side_streams_on() {
  static const bool on = std::getenv("TPE_SIDE_STREAMS") != nullptr;
  return on;
}
static bool moment_on();
// TPE_MOMENT_H=0: 16-wide plans without the degree-15 chunk table (A/B)
static bool moment_h_on() {
  static const bool on = [] {
    const char *e = std::getenv("TPE_MOMENT_H");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}
constexpr int64_t kSmallSortMin = 2048;  // candidates per chunk worth bucketing a small draw

struct tpe_engine {
  int32_t device = 0;
  hipStream_t stream = nullptr;
  static constexpr int kAux = 4;
  hipStream_t aux[kAux] = {};  // concurrent scoring kinds of one level
  std::string err;
  tpe_plan *op = nullptr;  // cached single-hp plan for operator-level calls
};

struct tpe_plan {
  tpe_engine *eng = nullptr;
  int32_t P = 0;
  int64_t ncap = 0, kcap = 0;
  int32_t last_nb = -1;  // n_below of the last tpe_plan_fit (below K <= n_below + 1)
  std::vector<tpe_hp> hps;
  std::vector<int32_t> cond_parent, cond_branch;
  std::vector<double> pprior;
  std::vector<std::vector<int32_t>> levels;
  std::vector<int32_t> level_off;  // offsets of each level in d_level_hps
  struct Group { int32_t kind, off, count; };
  std::vector<std::vector<Group>> groups;  // per level, hps grouped by lpdf kind
  // device buffers
  tpe_hp *d_hps = nullptr;
  int32_t *d_cp = nullptr, *d_cb = nullptr, *d_level_hps = nullptr, *d_all_hps = nullptr;
  int32_t *d_level_off = nullptr;  // level_off on the device (k_prior)
  double *d_pprior = nullptr;
  double *d_losses = nullptr, *d_vals = nullptr;
  uint8_t *d_active = nullptr, *d_below = nullptr;
  double *d_mw = nullptr, *d_mmu = nullptr, *d_msig = nullptr, *d_scratch = nullptr;
  unsigned char *d_sortbuf = nullptr;  // [2P][16 * scap] fit sort scratch
  int64_t scap = 0;
  MixInfo *d_info = nullptr;
  Coef *d_coef = nullptr;
  Coef32 *d_coef32 = nullptr;  // [2P][kcap / kCoefBlock] block-local fp32 LSE terms
  CoefM *d_coefm = nullptr;    // [2P][mom_stride(kcap)] moment form of 16-component chunks
  CoefM8 *d_coefm8 = nullptr;  // [2P][kcap / kCoefBlock] moment form of 8-component blocks
  float4 *d_coefe = nullptr;   // [2P][kcap / kCoefBlock] compact log-sum-exp block envelopes
  CoefM8 *d_coefmh = nullptr;  // [2P][mom_stride(kcap)] degree-15 form of 16-component chunks
  std::vector<double> act_frac;  // per hp: expected share of the trials it is active in
  int64_t n = 0;  // history length
  // suggestion state
  int64_t s_cap = 0;
  Partial *d_results = nullptr;
  tpe_result *h_results = nullptr;  // pinned host staging of the results copy
  size_t h_results_cap = 0;
  uint64_t *h_flag = nullptr;       // pinned completion word of k_publish
  uint64_t seq = 0;
  // this call's results go to the host and its last launch may publish them
  // itself (tpe_plan_fit_suggest); pub_fired: it does, with sequence seq
  bool pub_arm = false;
  bool pub_fired = false;
  uint64_t *d_seeds = nullptr;
  Partial *d_partial = nullptr;
  size_t partial_cap = 0;
  unsigned long long *d_census = nullptr;  // [kCensus] pair census (tpe_plan_census)
  bool census = false;
  uint32_t *d_ticket = nullptr;
  std::vector<uint64_t> h_seeds;  // this call's seeds (inline kernel args when <= 8)
  bool has_erf = false;
  // value lattices of the bounded quantized hps (KIND_LAT, k_lattice)
  std::vector<LatInfo> lat;
  LatInfo *d_lat_info = nullptr;
  double2 *d_lat = nullptr;
  bool lattice_on = true;
  int32_t prune_mode = 3;  // log-sum-exp on bucketed tiles (tpe_plan_set_prune): 0 full,
                           // 1 block skip, 2 block skip + one exponent per wave,
                           // 3 the same with block-local fp32 pairs
  hipEvent_t ev_fork = nullptr, ev_join[8] = {};
  double *d_ext = nullptr, *d_lb = nullptr, *d_la = nullptr;
  size_t ext_cap = 0;
  double *d_cand = nullptr;
  int32_t *d_cpos = nullptr;
  size_t cand_cap = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // per-kind event ring around every scoring launch (tpe_plan_profile)
  struct Prof {
    std::vector<hipEvent_t> a, b;
    std::vector<double> pairs;  // candidate-component pairs the launch covers
    int64_t n = 0;
  };
  Prof prof[KIND_CAT + 1];
  int32_t prof_cap = 0;
  bool timed = false;
  bool evs = false;  // ev0/ev1 bracket the last suggest (recorded only while profiling:
                     // an event record costs a ~6 us pipeline drain between launches)
  int64_t last_ncand = 0, last_nsug = 0;
  int32_t last_level = -1;
  // fit + suggest captured as one hipGraph (tpe_plan_fit_suggest): replayed
  // with the history length / n_below of the fit node and the seeds of the
  // draw nodes patched per call
  struct StepKey {
    double prior_weight = 0;
    int32_t lf = 0;
    int64_t n_sug = 0, n_cand = 0;
    void *stream = nullptr;
    bool table = false;  // below mixtures fit the LDS draw table (kTabCap)
    bool fuse = false;   // ... and the fused k_lattice draw rows' table (kFuseTab)
    bool small = false;  // k_fit<true> serves the history (fit_small)
    bool operator==(const StepKey &o) const {
      return prior_weight == o.prior_weight && lf == o.lf && n_sug == o.n_sug &&
             n_cand == o.n_cand && stream == o.stream && table == o.table && fuse == o.fuse &&
             small == o.small;
    }
  };
  StepKey graph_key, pending_key;
  bool graph_ok = false, pending = false;
  bool capturing = false;  // enqueue_step under graph capture (no per-call patch of score seeds)
  int32_t mom_w = 0;       // moment table the last fit wrote: 16 (CoefM), 8 (CoefM8), 0 none
  bool mom_h = false;      // ... and with 16, the degree-15 table (CoefMH)
  bool graph_mom_h = false;
  int32_t graph_mom_w = 0; // ... the captured graph's fit (launch_step restores it)
  HistPatch pend{};        // a small history update not yet on the device: the next
  bool has_pend = false;   // fit writes it (k_fit's patch), anything else flushes it
  hipGraph_t graph = nullptr;
  hipGraphExec_t graph_exec = nullptr;
  std::vector<hipGraphNode_t> fit_nodes, draw_nodes;
  std::vector<hipKernelNodeParams> fit_params, draw_params;
  std::vector<FitArgs> fit_args0;
  std::vector<ScoreArgs> draw_args0;
};

namespace {

#define CKH(expr)                                                        \
  do {                                                                   \
    hipError_t e_ = (expr);                                              \
    if (e_ != hipSuccess) {                                              \
      return fail(h, TPE_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    }                                                                    \
  } while (0)

int fail(tpe_engine *h, int code, const std::string &msg) {
  if (h) h->err = msg;
  return code;
}

template <typename T>
hipError_t dalloc(T **p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  return hipMalloc((void **)p, count * sizeof(T));
}

void dfree(void *p) {
  if (p) (void)hipFree(p);
}

// drop the captured fit + suggest graph (buffers it points to change)
void graph_reset(tpe_plan *p) {
  if (p->graph_exec) (void)hipGraphExecDestroy(p->graph_exec);
  if (p->graph) (void)hipGraphDestroy(p->graph);
  p->graph_exec = nullptr;
  p->graph = nullptr;
  p->graph_ok = p->pending = false;
  p->fit_nodes.clear(); p->draw_nodes.clear();
  p->fit_params.clear(); p->draw_params.clear();
  p->fit_args0.clear(); p->draw_args0.clear();
}

hipStream_t pick_stream(tpe_engine *h, void *s) {
  return s ? (hipStream_t)s : h->stream;
}

void plan_free_buffers(tpe_plan *p) {
  void *bufs[] = {p->d_hps, p->d_cp, p->d_cb, p->d_level_hps, p->d_all_hps, p->d_pprior,
                  p->d_level_off,
                  p->d_losses, p->d_vals, p->d_active, p->d_below, p->d_mw, p->d_mmu,
                  p->d_msig, p->d_scratch, p->d_info, p->d_coef, p->d_results, p->d_seeds,
                  p->d_partial, p->d_ext, p->d_lb, p->d_la, p->d_cand, p->d_cpos,
                  p->d_ticket, p->d_sortbuf, p->d_census, p->d_lat_info, p->d_lat, p->d_coef32, p->d_coefm,
                  p->d_coefm8, p->d_coefe, p->d_coefmh};
  for (void *b : bufs) dfree(b);
  if (p->h_results) (void)hipHostFree(p->h_results);
  p->h_results = nullptr;
  p->h_results_cap = 0;
  if (p->h_flag) (void)hipHostFree(p->h_flag);
  p->h_flag = nullptr;
  if (p->ev0) (void)hipEventDestroy(p->ev0);
  if (p->ev1) (void)hipEventDestroy(p->ev1);
  if (p->ev_fork) (void)hipEventDestroy(p->ev_fork);
  for (auto e : p->ev_join) if (e) (void)hipEventDestroy(e);
  for (auto &pr : p->prof) {
    for (auto e : pr.a) (void)hipEventDestroy(e);
    for (auto e : pr.b) (void)hipEventDestroy(e);
    pr.a.clear(); pr.b.clear(); pr.pairs.clear(); pr.n = 0;
  }
}

int validate_space(tpe_engine *h, const tpe_space *sp) {
  if (!sp || sp->n_hp <= 0 || !sp->hp) return fail(h, TPE_E_INVALID, "empty space");
  for (int i = 0; i < sp->n_hp; ++i) {
    const tpe_hp &x = sp->hp[i];
    if (x.family < TPE_GMM || x.family > TPE_CAT)
      return fail(h, TPE_E_INVALID, "hp " + std::to_string(i) + ": bad family");
    if (x.family == TPE_CAT && x.upper <= 0)
      return fail(h, TPE_E_INVALID, "hp " + std::to_string(i) + ": categorical upper <= 0");
    if (x.family != TPE_CAT) {
      const bool hl = x.flags & TPE_HAS_LOW, hh = x.flags & TPE_HAS_HIGH;
      if (hl != hh)
        return fail(h, TPE_E_INVALID, "hp " + std::to_string(i) + ": one-sided truncation");
      if (hl && !(x.low < x.high))
        return fail(h, TPE_E_BOUNDS, "low >= high");
      if (!(x.prior_sigma > 0))
        return fail(h, TPE_E_INVALID, "hp " + std::to_string(i) + ": prior_sigma <= 0");
    }
    if (x.cond_count < 0 || x.cond_begin < 0 || x.cond_begin + x.cond_count > sp->n_cond)
      return fail(h, TPE_E_INVALID, "hp " + std::to_string(i) + ": bad condition range");
    for (int c = 0; c < x.cond_count; ++c) {
      const int par = sp->cond_parent[x.cond_begin + c];
      if (par < 0 || par >= sp->n_hp || par == i)
        return fail(h, TPE_E_INVALID, "hp " + std::to_string(i) + ": bad condition parent");
    }
    if ((x.flags & TPE_PCHOICE) &&
        (x.pprior_begin < 0 || x.pprior_begin + x.upper > sp->n_pprior))
      return fail(h, TPE_E_INVALID, "hp " + std::to_string(i) + ": bad pchoice prior");
  }
  return TPE_OK;
}

// level(h) = 0 without conditions, else 1 + max(level(parent))
// The value lattice of a bounded quantized hp (LatInfo): drawn values lie in
// [low, high) (GMM) or [exp(low), exp(high)] (LGMM) before rounding to j * q;
// two indices of margin on each side absorb host/device exp and division
// rounding.  R = 0 (no lattice) for unbounded or huge ranges.
LatInfo lattice_of(const tpe_hp &x) {
  LatInfo L{0, 0, 0, 0};
  const int k = score_kind(x);
  if (k != KIND_ERF_G && k != KIND_ERF_L) return L;
  if (!(x.flags & TPE_HAS_LOW) || !(x.flags & TPE_HAS_HIGH) || !(x.q > 0.0)) return L;
  double lo = x.low, hi = x.high;
  if (k == KIND_ERF_L) {
    lo = std::exp(lo);
    hi = std::exp(hi);
  }
  const double a = std::rint(lo / x.q) - 2.0, b = std::rint(hi / x.q) + 2.0;
  if (!(std::fabs(a) < 1e15 && std::fabs(b) < 1e15) || b - a + 1.0 > (double)kLatMaxR)
    return L;
  L.j0 = (int64_t)a;
  L.R = (int32_t)(b - a + 1.0);
  return L;
}

int compute_levels(tpe_engine *h, tpe_plan *p) {
  std::vector<int> lev(p->P, -1);
  for (int iter = 0; iter <= p->P; ++iter) {
    bool changed = false;
    for (int i = 0; i < p->P; ++i) {
      const tpe_hp &x = p->hps[i];
      int l = 0;
      bool ready = true;
      for (int c = 0; c < x.cond_count; ++c) {
        const int par = p->cond_parent[x.cond_begin + c];
        if (lev[par] < 0) { ready = false; break; }
        l = std::max(l, lev[par] + 1);
      }
      if (ready && lev[i] != l) { lev[i] = l; changed = true; }
    }
    if (!changed) break;
  }
  int nl = 0;
  for (int i = 0; i < p->P; ++i) {
    if (lev[i] < 0 || lev[i] > p->P) return fail(h, TPE_E_INVALID, "cyclic conditions");
    nl = std::max(nl, lev[i] + 1);
  }
  p->levels.assign(nl, {});
  // quantized hps with a value lattice first (run_level scores them on it),
  // then the heaviest lpdf kind first: the scoring grid's low slots are
  // dispatched first, so the long quantized tiles do not form the launch's tail
  for (int lat : {1, 0})
    for (int kind : {KIND_ERF_L, KIND_ERF_G})
      for (int i = 0; i < p->P; ++i)
        if (score_kind(p->hps[i]) == kind && (lattice_of(p->hps[i]).R > 0) == (lat == 1))
          p->levels[lev[i]].push_back(i);
  for (int kind : {KIND_LSE_L, KIND_LSE_G, KIND_CAT})
    for (int i = 0; i < p->P; ++i)
      if (score_kind(p->hps[i]) == kind) p->levels[lev[i]].push_back(i);
  p->level_off.assign(nl + 1, 0);
  p->groups.assign(nl, {});
  for (int l = 0; l < nl; ++l) {
    p->level_off[l + 1] = p->level_off[l] + (int)p->levels[l].size();
    int j = 0;
    const auto &L = p->levels[l];
    while (j < (int)L.size()) {
      const int kind = score_kind(p->hps[L[j]]);
      int k = j;
      while (k < (int)L.size() && score_kind(p->hps[L[k]]) == kind) ++k;
      p->groups[l].push_back({kind, p->level_off[l] + j, k - j});
      j = k;
    }
  }
  return TPE_OK;
}

int plan_build(tpe_engine *h, const tpe_space *sp, int64_t max_trials, tpe_plan *p) {
  int rc = validate_space(h, sp);
  if (rc) return rc;
  if (max_trials < 0) return fail(h, TPE_E_INVALID, "max_trials < 0");
  p->eng = h;
  p->P = sp->n_hp;

  p->hps.assign(sp->hp, sp->hp + sp->n_hp);
  p->cond_parent.assign(sp->cond_parent, sp->cond_parent + sp->n_cond);
  p->cond_branch.assign(sp->cond_branch, sp->cond_branch + sp->n_cond);
  p->pprior.assign(sp->pprior, sp->pprior + sp->n_pprior);
  rc = compute_levels(h, p);
  if (rc) return rc;
  p->ncap = std::max<int64_t>(max_trials, 1);
  int64_t kcap = p->ncap + 1;
  for (const auto &x : p->hps)
    if (x.family == TPE_CAT) kcap = std::max<int64_t>(kcap, x.upper);
  // whole coefficient blocks per slot (coef_at, tpe_internal.hpp)
  kcap = (kcap + kCoefBlock - 1) / kCoefBlock * kCoefBlock;
  p->kcap = kcap;
  for (const auto &x : p->hps) {
    const int k = score_kind(x);
    if (k == KIND_ERF_G || k == KIND_ERF_L) p->has_erf = true;
  }
  const int64_t slots = 2 * (int64_t)p->P;
  p->lat.assign(p->P, LatInfo{0, 0, 0, 0});
  int64_t lat_total = 0;
  for (int i = 0; i < p->P; ++i) {
    p->lat[i] = lattice_of(p->hps[i]);
    p->lat[i].off = lat_total;
    lat_total += p->lat[i].R;
  }
  CKH(hipSetDevice(h->device));
  CKH(dalloc(&p->d_lat_info, p->P));
  CKH(dalloc(&p->d_lat, std::max<int64_t>(1, lat_total)));
  CKH(dalloc(&p->d_hps, p->P));
  CKH(dalloc(&p->d_cp, p->cond_parent.size()));
  CKH(dalloc(&p->d_cb, p->cond_branch.size()));
  CKH(dalloc(&p->d_pprior, p->pprior.size()));
  CKH(dalloc(&p->d_level_hps, p->P));
  CKH(dalloc(&p->d_all_hps, p->P));
  CKH(dalloc(&p->d_level_off, p->level_off.size()));
  CKH(dalloc(&p->d_losses, p->ncap));
  CKH(dalloc(&p->d_vals, (size_t)p->ncap * p->P));
  CKH(dalloc(&p->d_active, (size_t)p->ncap * p->P));
  CKH(dalloc(&p->d_below, p->ncap));
  CKH(dalloc(&p->d_mw, (size_t)slots * kcap));
  CKH(dalloc(&p->d_mmu, (size_t)slots * kcap));
  CKH(dalloc(&p->d_msig, (size_t)slots * kcap));
  CKH(dalloc(&p->d_scratch, (size_t)slots * kcap));
  p->scap = p->ncap + 1;
  CKH(dalloc(&p->d_sortbuf, (size_t)slots * 16 * p->scap));
  CKH(dalloc(&p->d_info, slots));
  CKH(dalloc(&p->d_census, kCensus));
  CKH(hipMemset(p->d_census, 0, kCensus * sizeof(unsigned long long)));
  CKH(dalloc(&p->d_coef, (size_t)slots * kcap));
  CKH(dalloc(&p->d_coef32, (size_t)slots * (kcap / kCoefBlock)));
  CKH(dalloc(&p->d_coefm, (size_t)slots * mom_stride(kcap)));
  CKH(dalloc(&p->d_coefm8, (size_t)slots * (kcap / kCoefBlock)));
  CKH(dalloc(&p->d_coefe, (size_t)slots * (kcap / kCoefBlock)));
  CKH(dalloc(&p->d_coefmh, (size_t)slots * mom_stride(kcap)));
  // expected activity of every hp (mom_width): an hp conditioned on branch b
  // of a categorical parent is active in ~1 / upper of the parent's trials
  // (levels are in dependency order: parents first)
  p->act_frac.assign(p->P, 1.0);
  for (const auto &lv : p->levels)
    for (int i : lv) {
      const tpe_hp &x = p->hps[i];
      if (x.cond_count == 0) continue;
      double f = 0.0;
      for (int c = 0; c < x.cond_count; ++c) {
        const int par = p->cond_parent[x.cond_begin + c];
        const tpe_hp &y = p->hps[par];
        f += p->act_frac[par] / (y.family == TPE_CAT ? std::max(1, (int)y.upper) : 1);
      }
      p->act_frac[i] = std::min(1.0, f);
    }
  CKH(hipEventCreate(&p->ev0));
  CKH(hipEventCreate(&p->ev1));
  CKH(hipEventCreateWithFlags(&p->ev_fork, hipEventDisableTiming));
  for (auto &e : p->ev_join) CKH(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  std::vector<int32_t> lh;
  for (auto &l : p->levels) lh.insert(lh.end(), l.begin(), l.end());
  std::vector<int32_t> all(p->P);
  for (int i = 0; i < p->P; ++i) all[i] = i;
  hipStream_t st = h->stream;
  CKH(hipMemcpyAsync(p->d_hps, p->hps.data(), p->P * sizeof(tpe_hp), hipMemcpyHostToDevice, st));
  CKH(hipMemcpyAsync(p->d_lat_info, p->lat.data(), p->P * sizeof(LatInfo), hipMemcpyHostToDevice,
                     st));
  if (!p->cond_parent.empty()) {
    CKH(hipMemcpyAsync(p->d_cp, p->cond_parent.data(), p->cond_parent.size() * 4, hipMemcpyHostToDevice, st));
    CKH(hipMemcpyAsync(p->d_cb, p->cond_branch.data(), p->cond_branch.size() * 4, hipMemcpyHostToDevice, st));
  }
  if (!p->pprior.empty())
    CKH(hipMemcpyAsync(p->d_pprior, p->pprior.data(), p->pprior.size() * 8, hipMemcpyHostToDevice, st));
  CKH(hipMemcpyAsync(p->d_level_hps, lh.data(), lh.size() * 4, hipMemcpyHostToDevice, st));
  CKH(hipMemcpyAsync(p->d_all_hps, all.data(), all.size() * 4, hipMemcpyHostToDevice, st));
  CKH(hipMemcpyAsync(p->d_level_off, p->level_off.data(), p->level_off.size() * 4,
                     hipMemcpyHostToDevice, st));
  CKH(hipMemsetAsync(p->d_info, 0, slots * sizeof(MixInfo), st));
  CKH(hipStreamSynchronize(st));
  return TPE_OK;
}

int ensure_suggest_state(tpe_engine *h, tpe_plan *p, int64_t n_sug, size_t partials) {
  if (n_sug > p->s_cap || partials > p->partial_cap) graph_reset(p);
  if (n_sug > p->s_cap) {
    dfree(p->d_results);
    dfree(p->d_seeds);
    dfree(p->d_ticket);
    p->d_results = nullptr;
    p->d_seeds = nullptr;
    p->d_ticket = nullptr;
    CKH(dalloc(&p->d_results, (size_t)n_sug * p->P));
    CKH(dalloc(&p->d_seeds, n_sug));
    // (+1: the launch-wide arrival counter of a publishing launch, pub_ticket)
    CKH(dalloc(&p->d_ticket, (size_t)n_sug * p->P + 1));
    CKH(hipMemset(p->d_ticket, 0, ((size_t)n_sug * p->P + 1) * sizeof(uint32_t)));
    p->s_cap = n_sug;
  }
  if (partials > p->partial_cap) {
    dfree(p->d_partial);
    p->d_partial = nullptr;
    CKH(dalloc(&p->d_partial, partials));
    p->partial_cap = partials;
  }
  return TPE_OK;
}

int ensure_ext(tpe_engine *h, tpe_plan *p, size_t n) {
  if (n > p->ext_cap) {
    dfree(p->d_ext); dfree(p->d_lb); dfree(p->d_la);
    p->d_ext = p->d_lb = p->d_la = nullptr;
    CKH(dalloc(&p->d_ext, n));
    CKH(dalloc(&p->d_lb, n));
    CKH(dalloc(&p->d_la, n));
    p->ext_cap = n;
  }
  return TPE_OK;
}

// Scoring grid of one launch over n_slots slots whose lpdf kinds are `kinds`
// (consecutive slots of one kind form a group, tiles of 64 * tile_rows(kind)
// candidates).  Returns the partial-record stride (max tiles per slot), or -1
// when the slots are not grouped by kind.
// Runs of equal-kind slots become groups of the 1-D scoring grid, emitted
// heaviest kind first (per-candidate erf, then log-sum-exp, then the lattice /
// categorical lookups): the dispatcher hands out the long blocks first and the
// short ones fill the CUs that finish early.
// rows(b, e) (optional, compact grids): block rows for the slots [b, e) of a
// group (active_bound), else one row per slot.
template <typename Rows>
int32_t set_score_groups(ScoreArgs &a, const int *kinds, int n_slots, int64_t cn, Rows rows) {
  a.n_groups = 0;
  int32_t blocks = 0, pstride = 1;
  auto weight = [](int kind) {
    switch (kind) {
      case KIND_ERF_G: case KIND_ERF_L: return 0;
      case KIND_LSE_G: case KIND_LSE_L: case KIND_LSE_G1: case KIND_LSE_L1:
      case KIND_LSE_GW: case KIND_LSE_LW: case KIND_LSE_GW1: case KIND_LSE_LW1: return 1;
      case KIND_LAT: return 2;
      default: return 3;
    }
  };
  for (int pass = 0; pass < 4; ++pass) {
    for (int j = 0; j < n_slots;) {
      int k = j;
      while (k < n_slots && kinds[k] == kinds[j]) ++k;
      if (weight(kinds[j]) != pass) { j = k; continue; }
      if (a.n_groups == kMaxGroups) return -1;
      const int g = a.n_groups++;
      const int64_t tc = tile_cands(kinds[j]);
      const int32_t nt = (int32_t)((std::max<int64_t>(cn, 0) + tc - 1) / tc);
      a.grp_kind[g] = kinds[j];
      a.grp_slot0[g] = j;
      a.grp_slots[g] = k - j;
      a.grp_tiles[g] = nt;
      a.grp_block0[g] = blocks;
      blocks += nt * std::min<int32_t>(k - j, rows(j, k));
      pstride = std::max(pstride, nt);
      j = k;
    }
  }
  a.grp_block0[a.n_groups] = blocks;
  return pstride;
}
int32_t set_score_groups(ScoreArgs &a, const int *kinds, int n_slots, int64_t cn) {
  return set_score_groups(a, kinds, n_slots, cn, [](int b, int e) { return e - b; });
}

// The most hps of hps[b, e) active together in one suggestion: the
// unconditional ones, plus, for every condition parent, the most hps that
// share one of its branch values.  (A parent takes one value per suggestion
// and an active hp has a true condition: charge it to that condition's
// parent; the hps charged to a parent share the branch it took.)
int32_t active_bound(const tpe_plan *p, const int32_t *hps, int b, int e) {
  int32_t n = 0;
  std::vector<std::pair<int32_t, int32_t>> pb;  // (parent, branch) of every condition
  for (int i = b; i < e; ++i) {
    const tpe_hp &x = p->hps[hps[i]];
    if (x.cond_count == 0) { ++n; continue; }
    std::vector<std::pair<int32_t, int32_t>> mine;
    for (int c = 0; c < x.cond_count; ++c)
      mine.emplace_back(p->cond_parent[x.cond_begin + c], p->cond_branch[x.cond_begin + c]);
    std::sort(mine.begin(), mine.end());
    mine.erase(std::unique(mine.begin(), mine.end()), mine.end());
    pb.insert(pb.end(), mine.begin(), mine.end());
  }
  std::sort(pb.begin(), pb.end());
  for (size_t i = 0; i < pb.size();) {
    int32_t best = 0;
    size_t j = i;
    while (j < pb.size() && pb[j].first == pb[i].first) {
      size_t k = j;
      while (k < pb.size() && pb[k] == pb[j]) ++k;
      best = std::max<int32_t>(best, (int32_t)(k - j));
      j = k;
    }
    n += best;
    i = j;
  }
  return std::min<int32_t>(n, e - b);
}

void copy_groups(ScoreArgs &a, const ScoreArgs &g) {
  a.n_groups = g.n_groups;
  a.compact = g.compact;
  for (int i = 0; i < kMaxGroups; ++i) {
    a.grp_slots[i] = g.grp_slots[i];
    a.grp_kind[i] = g.grp_kind[i];
    a.grp_slot0[i] = g.grp_slot0[i];
    a.grp_tiles[i] = g.grp_tiles[i];
  }
  for (int i = 0; i <= kMaxGroups; ++i) a.grp_block0[i] = g.grp_block0[i];
}

int ensure_cand(tpe_engine *h, tpe_plan *p, size_t n) {
  if (n > p->cand_cap) {
    graph_reset(p);
    dfree(p->d_cand);
    dfree(p->d_cpos);
    p->d_cand = nullptr;
    p->d_cpos = nullptr;
    CKH(dalloc(&p->d_cand, n));
    CKH(dalloc(&p->d_cpos, n));
    p->cand_cap = n;
  }
  return TPE_OK;
}

// Pairs a scoring launch evaluates if every hp of the group is active: uses
// the host copy of the mixture sizes refreshed by tpe_plan_profile_read.
double group_pairs(tpe_plan *p, int kind, int32_t n_slots, int64_t cn, int64_t n_sug) {
  (void)p; (void)kind; (void)n_slots;
  return (double)cn * (double)n_sug;  // x (K_b + K_a) applied at read time
}

ScoreArgs base_args(tpe_plan *p, int64_t n_sug) {
  ScoreArgs a{};
  a.sort_log2 = kSortLog2Small;
  a.hps = p->d_hps;
  a.cond_parent = p->d_cp;
  a.cond_branch = p->d_cb;
  a.info = p->d_info;
  a.coef = p->d_coef;
  a.coef32 = p->d_coef32;
  a.coefm = p->d_coefm;
  a.coefm8 = p->d_coefm8;
  a.coefmh = p->d_coefmh;
  a.coefe = p->d_coefe;
  a.mw = p->d_mw;
  a.mmu = p->d_mmu;
  a.msig = p->d_msig;
  a.seeds = p->d_seeds;
  a.results = p->d_results;
  a.partial = p->d_partial;
  a.ticket = p->d_ticket;
  a.census = p->census ? p->d_census : nullptr;
  a.kcap = p->kcap;
  a.n_hp = p->P;
  a.n_suggest = (int32_t)n_sug;
  a.lat_info = p->d_lat_info;
  a.lat = p->d_lat;
  a.lse_mom = p->mom_w;
  a.lse_momh = p->mom_w == 16 && p->mom_h ? 1 : 0;
  a.l2_warm = l2_warm_on() ? 1 : 0;
  a.lse_tight = tighten_on() ? 1 : 0;
  return a;
}

// The moment width of the plan's log-sum-exp mixtures (tpe_internal.hpp
// CoefM8): 16 when the largest expected above-side mixture (history length
// x the hp's expected activity) has >= kMom16MinK components (neighbour gaps
// << sigma floor: 16-component chunks qualify), 8 from the one-exponent size
// (lse_shift_min) up, else 0.  (tools/moment_error.py: at N = 5000 the 16-wide
// form covers 72 % of the live chunks at 0.6 VALU per pair, the 8-wide 99 %
// at ~1.7; at N = 3000, 36 % against 98 %.)  A function of the plan and its
// history length only, so tpe_plan_fit and fit_suggest write the same table.
// TPE_MOM16_MIN_K: the 16-wide threshold (A/B; default kMom16MinK)
static double mom16_min_k() {
  static const double v = [] {
    const char *e = std::getenv("TPE_MOM16_MIN_K");
    return e ? std::atof(e) : (double)kMom16MinK;
  }();
  return v;
}
int32_t mom_width(const tpe_plan *p) {
  if (!moment_on()) return 0;
  double kmax = 0.0;
  for (int i = 0; i < p->P; ++i) {
    const int k = score_kind(p->hps[i]);
    if (k == KIND_LSE_G || k == KIND_LSE_L) kmax = std::max(kmax, (double)p->n * p->act_frac[i]);
  }
  if (kmax >= mom16_min_k()) return 16;
  if (kmax >= (double)lse_shift_min()) return 8;
  return 0;
}

// mom: write the moment table of the plan's width (mom_width) -- only the
// wave tiles of sorted draws read it; plan.mom_w records which one the tables
// hold (the scoring launches read that one: base_args)
FitArgs fit_args(tpe_plan *p, int32_t n_below, double prior_weight, int32_t lf, bool mom = true) {
  p->mom_w = mom ? mom_width(p) : 0;
  FitArgs a{};
  a.hps = p->d_hps;
  a.vals = p->d_vals;
  a.active = p->d_active;
  a.losses = p->d_losses;
  a.n = p->n;
  a.ld = p->ncap;
  a.n_below = n_below;
  a.lf = lf;
  a.prior_weight = prior_weight;
  a.pprior = p->d_pprior;
  a.mw = p->d_mw;
  a.mmu = p->d_mmu;
  a.msig = p->d_msig;
  a.info = p->d_info;
  a.coef = p->d_coef;
  a.coef32 = p->d_coef32;
  a.coefm = p->mom_w == 16 ? p->d_coefm : nullptr;
  a.coefm8 = p->mom_w == 8 ? p->d_coefm8 : nullptr;
  a.coefmh = p->mom_w == 16 && moment_h_on() ? p->d_coefmh : nullptr;
  p->mom_h = a.coefmh != nullptr;
  a.coefe = p->d_coefe;
  a.kcap = p->kcap;
  a.ob = p->d_scratch;
  a.tmp = p->d_scratch;
  a.sortbuf = p->d_sortbuf;
  a.scap = p->scap;
  return a;
}

// a deferred history update onto the device now (k_hist_patch), for every
// reader other than the fit
int flush_patch(tpe_engine *h, tpe_plan *p, hipStream_t st) {
  if (!p->has_pend) return TPE_OK;
  p->has_pend = false;
  CKH(launch_hist_patch(p->pend, p->d_vals, p->d_active, p->d_losses, st));
  return TPE_OK;
}
// the fit of a plan, with the deferred history update (if any) written by
// its blocks first
int fit_launch(tpe_engine *h, tpe_plan *p, const FitArgs &a, int32_t n_hp, hipStream_t st) {
  CKH(launch_fit(a, n_hp, st, p->has_pend ? &p->pend : nullptr));
  p->has_pend = false;
  return TPE_OK;
}

int score_launch(tpe_engine *h, tpe_plan *p, ScoreArgs a, bool has_erf, int64_t cn,
                 hipStream_t sg, bool record, int classes = 7) {
  tpe_plan::Prof *pr = nullptr;
  if (record && p->prof_cap > 0) {
    pr = &p->prof[0];
    if (pr->n >= p->prof_cap) pr = nullptr;  // ring full: stop recording
  }
  if (pr) CKH(hipEventRecord(pr->a[pr->n], sg));
  // (a level mixing wave-tile log-sum-exp slots with other kinds: those run
  // beside it on an auxiliary stream; the events are free at scoring time)
  CKH(launch_score(a, has_erf, sg, side_streams_on() ? h->aux[1] : nullptr, p->ev_join[1],
                   p->ev_join[2], classes));
  if (pr) {
    CKH(hipEventRecord(pr->b[pr->n], sg));
    pr->pairs[pr->n] = (double)cn * (double)a.n_suggest;
    pr->n++;
  }
  return TPE_OK;
}

// One level of conditional hps: one draw(+bucket) launch and one scoring
// launch (every lpdf kind) for all of its hps.  Candidates are processed in
// chunks so the buffer stays <= 2 GB (chunk_budget).
// n_total: the candidates of the whole suggestion this call scores [cand_begin,
// cand_begin + n_cand) of (a shard's is the unsharded count): it picks the
// wave-tile shape, so every shard and batch of one suggestion takes the same
int run_level(tpe_engine *h, tpe_plan *p, int level, int64_t n_sug, int64_t n_cand,
              int64_t cand_begin, int64_t n_total, hipStream_t st) {
  const int32_t n_level = (int32_t)p->levels[level].size();
  const int32_t *lvl = p->d_level_hps + p->level_off[level];
  if (n_cand == 0) {
    // no candidates (an empty shard of a small suggest, n_EI_candidates = 0):
    // broadcast_best of no samples is [] (tpe.py:750-759) -- every hp of the
    // level gets the neutral record (NaN, NaN, -1, inactive), which k_merge
    // treats as "nothing here" (a merge of zero records writes exactly that)
    if (n_level > 0) CKH(launch_merge(lvl, n_level, (int32_t)n_sug, p->P, 0, nullptr, p->d_results, st));
    return TPE_OK;
  }
  bool erf_level = false;
  std::vector<int> kinds;
  // largest below mixture the draw can meet: the LDS table sampler fits it?
  int64_t kmax = p->last_nb >= 0 ? (int64_t)p->last_nb + 1 : p->kcap;
  for (int hp : p->levels[level]) {
    const int k = score_kind(p->hps[hp]);
    kinds.push_back(k);
    erf_level |= k == KIND_ERF_G || k == KIND_ERF_L;
    if (k == KIND_CAT) kmax = std::max<int64_t>(kmax, p->hps[hp].upper);
  }
  const bool table_draw = kmax <= kTabCap;
  // the level's leading quantized hps with a value lattice are scored on it
  // (k_lattice once per call, then lookups) when no lattice is larger than
  // the candidate count; the other quantized hps per candidate (bucketed)
  int32_t n_lat = 0;
  int64_t rmax = 0;
  while (n_lat < n_level && (kinds[n_lat] == KIND_ERF_G || kinds[n_lat] == KIND_ERF_L) &&
         p->lat[p->levels[level][n_lat]].R > 0) {
    rmax = std::max<int64_t>(rmax, p->lat[p->levels[level][n_lat]].R);
    ++n_lat;
  }
  const bool lat_level = n_lat > 0 && p->lattice_on && rmax <= n_cand * n_sug &&
                         2 * ((p->kcap + 15) / 16) <= (int64_t)kLatChunks;
  if (!lat_level) n_lat = 0;
  // conditional level: grids sized for the hps that can be active together
  // (ScoreArgs::compact), not one row per hp -- the other branches of a
  // choice cost no blocks
  const int32_t *hl = p->levels[level].data();
  const int32_t lvl_rows = active_bound(p, hl, 0, n_level);
  const bool compact = lvl_rows < n_level;
  const int32_t slot_rows = compact ? lvl_rows : n_level;
  const int32_t lat_rows =
      compact ? (int32_t)std::min<int64_t>(n_lat, n_sug * (int64_t)active_bound(p, hl, 0, n_lat))
              : n_lat;
  const int64_t budget = chunk_budget();  // doubles
  int64_t chunk = std::max<int64_t>(
      1, std::min<int64_t>(std::max<int64_t>(n_cand, 1),
                           budget / std::max<int64_t>(1, n_sug * n_level)));
  // several chunks: each a whole number of sorted-draw blocks, so the blocks
  // (and with them every pruned log-sum-exp) sit at the same global candidate
  // indices however [0, n) is chunked or sharded (TPE_SHARD_ALIGN)
  if (chunk < n_cand) chunk = std::max<int64_t>(kSortedBlock, chunk / kSortedBlock * kSortedBlock);
  // a small one-chunk draw whose tables fit kFuseTab runs in extra blocks of
  // the lattice launch (both only need the fitted mixtures): one launch less
  // and the draw hidden behind the lattice points
  const bool fuse_draw = lat_level && n_lat <= kLatJobs && table_draw &&
                         kmax <= kFuseTab && chunk >= n_cand &&
                         n_cand * n_sug * n_level < ((int64_t)1 << 22);
  if (lat_level) {
    for (int i = 0; i < n_lat; ++i) kinds[i] = KIND_LAT;
    erf_level = false;  // per-candidate quantized slots left after the lattice ones?
    for (int i = n_lat; i < n_level; ++i)
      erf_level |= kinds[i] == KIND_ERF_G || kinds[i] == KIND_ERF_L;
  }
  // the lattice needs only the fitted mixtures: with TPE_SIDE_STREAMS=1 (and
  // unless it carries the draw, fuse_draw) it runs on a side stream beside the
  // candidate draw (fork / join events; a parallel branch of the captured
  // graph), and the scoring launch waits for it.  Default: in order on the
  // suggest stream -- round 5, config 3: 0.193 ms per suggest in order against
  // 0.201 ms forked (the cross-stream joins cost more than the overlap saves;
  // configs 2 and 5 unchanged, profiles/rd5h_*)
  const bool lat_side = lat_level && !fuse_draw && side_streams_on();
  // the lattice's readers are the lookup tiles: when those are forked beside
  // a sorted draw (below), the lattice goes first on the same auxiliary
  // stream -- in order before its readers, beside the draw and the
  // log-sum-exp scoring, one join after them (lat_defer; no fork of its own)
  bool has_other = false;
  for (int i = 0; i < n_level; ++i) has_other |= !(kinds[i] == KIND_LAT || kinds[i] == KIND_CAT);
  const bool sorted0 = !fuse_draw && table_draw &&
                       std::min(chunk, n_cand) * n_sug * n_level >= ((int64_t)1 << 22);
  const bool lk_inline = sorted0 && kmax <= kFuseTab && !p->capturing && lookup_draw_on();
  const bool lat_defer = lat_level && !fuse_draw && !lat_side && has_other && lk_inline &&
                         lookup_fork_on();
  ScoreArgs la = base_args(p, n_sug);
  la.level_hps = lvl;
  la.n_slots = n_level;
  la.slot_rows = slot_rows;
  la.compact = compact ? 1 : 0;
  auto lattice = [&](hipStream_t sl) -> int {
    tpe_plan::Prof *pr = nullptr;
    if (p->prof_cap > 0 && p->prof[1].n < p->prof_cap) pr = &p->prof[1];
    if (pr) CKH(hipEventRecord(pr->a[pr->n], sl));
    CKH(launch_lattice(la, p->levels[level].data(), p->hps.data(), p->lat.data(), n_lat,
                       p->d_lat, sl, lat_rows));
    if (pr) {
      CKH(hipEventRecord(pr->b[pr->n], sl));
      pr->pairs[pr->n] = (double)level;
      pr->n++;
    }
    return TPE_OK;
  };
  bool lat_pending = lat_defer;
  if (lat_level && !fuse_draw && !lat_defer) {
    hipStream_t sl = st;
    if (lat_side) {
      sl = h->aux[0];
      CKH(hipEventRecord(p->ev_fork, st));
      CKH(hipStreamWaitEvent(sl, p->ev_fork, 0));
    }
    // everything after the fork: a failure still records the join event on
    // the side stream and waits on it from st, so a captured graph is never
    // left forked (the chunk loop below joins on its own exits likewise)
    const int lrc = lattice(sl);
    if (lat_side) {
      const hipError_t e1 = hipEventRecord(p->ev_join[0], sl);
      if (lrc) {
        if (e1 == hipSuccess) (void)hipStreamWaitEvent(st, p->ev_join[0], 0);
        return lrc;
      }
      if (e1 != hipSuccess) return fail(h, TPE_E_HIP, "lattice side stream join event");
    } else if (lrc) {
      return lrc;
    }
  }
  bool joined = !lat_side;
  // log-sum-exp tiles: two candidate rows per lane, unless that leaves fewer
  // than ~3 blocks per CU (then whole-block work units are few and coarse, and
  // a CU with one more of them than its neighbours sets the launch time):
  // one-row tiles double the count at the same per-pair arithmetic
  {
    int64_t lse_slots = 0;
    for (int j = 0; j < n_level;) {  // active rows of the log-sum-exp runs
      int k = j;
      while (k < n_level && kinds[k] == kinds[j]) ++k;
      if (kinds[j] == KIND_LSE_G || kinds[j] == KIND_LSE_L)
        lse_slots += compact ? active_bound(p, hl, j, k) : k - j;
      j = k;
    }
    const int64_t blocks2 = n_sug * lse_slots * ((n_cand + 127) / 128);
    if (lse_slots > 0 && blocks2 < 3 * kNumCUs)
      for (int &k : kinds)
        k = k == KIND_LSE_G ? KIND_LSE_G1 : k == KIND_LSE_L ? KIND_LSE_L1 : k;
  }
  // every exit of the chunk loop (errors included) joins the lattice side
  // stream back, so a failed call never leaves a captured graph forked
  auto chunks = [&]() -> int {
  int64_t c0 = 0;
  do {
    const int64_t cn = std::min(chunk, n_cand - c0);
    // large draws: each draw block writes its candidates value-bucketed (LSE
    // and per-candidate erf slots) with their positions; the log-sum-exp
    // tiles then skip the component blocks that are exact zeros for them,
    // on wave tiles when the wave-wide exponent is on (prune mode 2)
    const bool sorted_draw = !fuse_draw && table_draw &&
                             cn * n_sug * n_level >= ((int64_t)1 << 22);
    // small draws of >= kSmallSortMin candidates: the log-sum-exp slots are
    // value-bucketed too (k_bucket, stable, <= 8192 per bucketing chunk) and
    // pruned on the 8-wave tiles
    bool small_sort = false;
    if (!sorted_draw && small_sort_on() && cn >= kSmallSortMin)
      for (int k : kinds) small_sort |= k == KIND_LSE_G || k == KIND_LSE_L || k == KIND_LSE_G1 ||
                                        k == KIND_LSE_L1;
    std::vector<int> ck(kinds);
    if (sorted_draw && p->prune_mode > 1)
      // pruned log-sum-exp slots on wave tiles: each wave its own 128
      // candidates and every live block, so its one exponent and its accuracy
      // guard see the whole sum.  (Round 4, config 3: 8-wave component-split
      // tiles below 2^18 candidates measured 0.265 ms with the one-exponent
      // form -- a wave's guard sees 1/8 of the components and 3e7 pairs per
      // launch were retried -- and 0.236 ms without it, against 0.234 ms here.)
      // (suggestions of <= kWaveRowSplitMax candidates: one-row wave tiles,
      // 64 candidates per wave -- the dense windows' waves carry half the
      // pairs; a small level leaves the GPU room for twice the waves)
      for (int &k : ck) {
        const bool one = n_total <= kWaveRowSplitMax;
        k = (k == KIND_LSE_G || k == KIND_LSE_G1) ? (one ? KIND_LSE_GW1 : KIND_LSE_GW)
          : (k == KIND_LSE_L || k == KIND_LSE_L1) ? (one ? KIND_LSE_LW1 : KIND_LSE_LW) : k;
      }
    else if (small_sort)
      // one-row tiles whatever the batch size: the pruned sums depend on the
      // tile's candidate window, so a batched suggestion stays bit-identical
      // to the same seed's single one
      for (int &k : ck)
        k = k == KIND_LSE_G ? KIND_LSE_G1 : k == KIND_LSE_L ? KIND_LSE_L1 : k;
    ScoreArgs grid{};
    grid.compact = compact ? 1 : 0;
    const int32_t pstride = set_score_groups(grid, ck.data(), n_level, cn, [&](int b, int e) {
      return compact ? active_bound(p, hl, b, e) : e - b;
    });
    if (pstride < 0) return fail(h, TPE_E_INVALID, "level slots not grouped by lpdf kind");
    int rc = ensure_suggest_state(h, p, n_sug, (size_t)n_sug * p->P * pstride);
    if (rc) return rc;
    rc = ensure_cand(h, p, (size_t)std::max<int64_t>(1, n_sug * n_level * cn));
    if (rc) return rc;
    // buffers (re)allocated above: take their pointers only now
    ScoreArgs a = base_args(p, n_sug);
    copy_groups(a, grid);
    a.cand = p->d_cand;
    a.cand_sstride = (int64_t)n_level * cn;
    a.n_cand = cn;
    a.cand_begin = cand_begin + c0;
    a.pstride = pstride;
    a.accumulate = c0 > 0 ? 1 : 0;
    a.level_hps = lvl;
    a.n_slots = n_level;
    a.slot_rows = slot_rows;
    a.cand_slot0 = 0;
    for (int i = 0; i < kInlineSeeds && i < n_sug; ++i) a.seed_inline[i] = p->h_seeds[i];
    a.n_inline_seeds = (int32_t)std::min<int64_t>(n_sug, kInlineSeeds);
    a.lse_pos = (sorted_draw || small_sort) ? 1 : 0;
    a.sort_log2 = sort_log2_for(n_total);  // (the whole suggestion's: shards agree)
    // lookup slots drawn by their scoring tiles (no write / read-back of their
    // candidates); not in a captured graph, whose replays patch the seeds of
    // the draw nodes only
    // (every lookup slot's below mixture within the tile's LDS table, so all
    // of them are drawn in their tiles and none reads the draw's output)
    a.lookup_draw = sorted_draw && kmax <= kFuseTab && !p->capturing && lookup_draw_on() ? 1 : 0;
    a.lse_prune = (sorted_draw || small_sort) ? p->prune_mode : 0;
    a.lse_shift_min = lse_shift_min();
    // prune mode 3's block-local fp32 pairs on every log-sum-exp slot of the
    // suggest, pruned (large draws) or not (small draws: every pair, 8-wave
    // component-split tiles)
    a.lse_f32 = p->prune_mode == 3 ? 1 : 0;
    // lookup tiles drawing their own candidates need nothing from this
    // chunk's draw: forked onto an auxiliary stream, they run beside the draw
    // and the log-sum-exp scoring, and st waits for them before the next
    // chunk (TPE_LOOKUP_FORK=0: in order on st)
    const int cls = score_classes(a);
    const bool lk_fork = (cls & 2) && (cls & ~2) && lookup_fork_on();
    if (lk_fork) {
      CKH(hipEventRecord(p->ev_join[3], st));
      CKH(hipStreamWaitEvent(h->aux[2], p->ev_join[3], 0));
      int lrc = TPE_OK;
      if (lat_pending) {  // the deferred lattice, ahead of its readers
        lrc = lattice(h->aux[2]);
        lat_pending = false;
      }
      const hipError_t el = lrc ? hipErrorUnknown
                                : launch_score(a, erf_level, h->aux[2], nullptr, nullptr, nullptr, 2);
      CKH(hipEventRecord(p->ev_join[4], h->aux[2]));
      if (el != hipSuccess) {
        (void)hipStreamWaitEvent(st, p->ev_join[4], 0);
        return fail(h, TPE_E_HIP, "lookup launch");
      }
    }
    if (lat_pending) {  // (no lookup fork after all: the lattice in order)
      lat_pending = false;
      const int lrc = lattice(st);
      if (lrc) return lrc;
    }
    // (every exit below joins the lookup stream back first)
    auto join_lk = [&]() {
      if (lk_fork) (void)hipStreamWaitEvent(st, p->ev_join[4], 0);
    };
    // tiny unsorted draws of levels with no lattice and no per-candidate erf
    // slots: the scoring tiles draw their own candidates (k_score_tdraw) --
    // one launch less (the config-1 shape: 24 candidates of one hp)
    const bool tdraw = !sorted_draw && !small_sort && !fuse_draw && !lat_level && !erf_level &&
                       table_draw && kmax <= kFuseTab && cn <= 4096 && !p->capturing &&
                       tile_draw_on();
    a.tile_draw = tdraw ? 1 : 0;
    // the call's last launch (its last level, one chunk, a full grid): its
    // last final record publishes the call's results (k_publish's work)
    if (tdraw && p->pub_arm && level + 1 == (int)p->levels.size() && cn == n_cand &&
        cand_begin == 0 && n_total == n_cand && !compact && !lk_fork && a.n_groups > 0 &&
        a.grp_block0[a.n_groups] > 0 && publish_fuse_on()) {
      a.pub_dst = reinterpret_cast<uint64_t *>(p->h_results);
      a.pub_flag = p->h_flag;
      a.pub_ticket = p->d_ticket + (size_t)p->s_cap * p->P;
      a.pub_seq = ++p->seq;
      a.pub_words = (int32_t)(n_sug * p->P * (int64_t)(sizeof(tpe_result) / 8));
      a.pub_events = (int32_t)(n_sug * n_level);
      p->pub_fired = true;
    }
    if (tdraw) {
    } else if (fuse_draw) {
      tpe_plan::Prof *pr = nullptr;
      if (p->prof_cap > 0 && p->prof[1].n < p->prof_cap) pr = &p->prof[1];
      if (pr) CKH(hipEventRecord(pr->a[pr->n], st));
      CKH(launch_lattice_draw(a, p->levels[level].data(), p->hps.data(), p->lat.data(), n_lat,
                              p->d_lat, st, lat_rows));
      if (pr) {
        CKH(hipEventRecord(pr->b[pr->n], st));
        pr->pairs[pr->n] = (double)level;
        pr->n++;
      }
    } else if (sorted_draw) {
      // the inline-draw kernel when every slot it draws is bounded continuous
      // (the lookup slots drawn in their tiles are skipped by it); kmax within
      // the table (table_draw) holds here
      bool fast = true;
      for (int i = 0; i < n_level && fast; ++i) {
        const tpe_hp &x = p->hps[p->levels[level][i]];
        const bool lookup = ck[i] == KIND_CAT || ck[i] == KIND_LAT;
        fast = lookup ? (a.lookup_draw != 0 && kmax <= kFuseTab)
                      : (x.family != TPE_CAT && (x.flags & TPE_HAS_LOW) && (x.flags & TPE_HAS_HIGH));
      }
      const hipError_t e = launch_draw_sorted(a, kmax <= kFuseTab, fast, p->d_cpos, st);
      if (e != hipSuccess) { join_lk(); return fail(h, TPE_E_HIP, hipGetErrorString(e)); }
    } else {
      CKH(launch_draw(a, table_draw, st));
    }
    if ((erf_level || small_sort) && !sorted_draw) CKH(launch_bucket(a, n_lat, p->d_cpos, st));
    a.cand_pos = (erf_level || sorted_draw || small_sort) ? p->d_cpos : nullptr;
    if (!joined) {
      CKH(hipStreamWaitEvent(st, p->ev_join[0], 0));
      joined = true;
    }
    rc = score_launch(h, p, a, erf_level, cn, st, true, lk_fork ? 5 : 7);
    join_lk();
    if (rc) return rc;
    c0 += cn;
  } while (c0 < n_cand);
  return TPE_OK;
  };
  const int rc = chunks();
  if (!joined) {
    const hipError_t e = hipStreamWaitEvent(st, p->ev_join[0], 0);
    if (!rc && e != hipSuccess) return fail(h, TPE_E_HIP, "join of the lattice side stream");
  }
  return rc;
}

// Externally supplied candidates of one hp (parity / operator path).
// sorted_mode < 0: every candidate scored on its own (exact sums, any
// tiling); >= 0: the large-draw production form -- value-bucketed in
// kSortedBlock blocks as k_draw_sorted writes them, log-sum-exp prune mode
// sorted_mode on the tiles run_level picks for it.
int run_external(tpe_engine *h, tpe_plan *p, int32_t hp, const double *ext, int64_t n,
                 double *lb, double *la, hipStream_t st, int32_t sorted_mode = -1) {
  int kind = score_kind(p->hps[hp]);
  const bool sorted = sorted_mode >= 0;
  if (sorted && sorted_mode > 1)
    kind = kind == KIND_LSE_G ? KIND_LSE_GW : kind == KIND_LSE_L ? KIND_LSE_LW : kind;
  ScoreArgs grid{};
  const int32_t pstride = set_score_groups(grid, &kind, 1, n);
  int rc = ensure_suggest_state(h, p, 1, (size_t)p->P * pstride);
  if (rc) return rc;
  if (sorted) {
    rc = ensure_cand(h, p, (size_t)std::max<int64_t>(1, n));
    if (rc) return rc;
  }
  ScoreArgs a = base_args(p, 1);
  copy_groups(a, grid);
  a.cand = ext;
  a.cand_sstride = n;
  a.n_cand = n;
  a.pstride = pstride;
  a.level_hps = p->d_all_hps + hp;
  a.n_slots = 1;
  a.slot_rows = 1;
  a.out_lb = lb;
  a.out_la = la;
  a.force_active = 1;
  if (sorted) {
    a.cand = p->d_cand;
    a.sort_log2 = sort_log2_for(n);
    CKH(launch_sort_ext(a, ext, p->d_cpos, st));
    a.cand_pos = p->d_cpos;
    a.lse_pos = 1;
    a.lse_prune = sorted_mode;
    a.lse_shift_min = lse_shift_min();
  }
  return score_launch(h, p, a, kind == KIND_ERF_G || kind == KIND_ERF_L, n, st, false);
}

int host_results(tpe_engine *h, tpe_plan *p, int64_t n_sug);

int copy_results(tpe_engine *h, tpe_plan *p, int64_t n_sug, tpe_result *out, int32_t on_dev,
                 hipStream_t st) {
  if (!out || on_dev) p->pub_fired = false;  // (armed for host output only)
  if (!out) return TPE_OK;
  const size_t bytes = (size_t)n_sug * p->P * sizeof(tpe_result);
  if (on_dev) {
    CKH(hipMemcpyAsync(out, p->d_results, bytes, hipMemcpyDeviceToDevice, st));
    return TPE_OK;
  }
  // to the host through a pinned staging buffer of the plan: a DMA copy
  // without the runtime's pageable-memory staging (a few hundred bytes; the
  // copy's latency is most of what the caller waits for after the kernels)
  // (fine-grained coherent pinned memory: the kernel's stores reach it
  // directly and the host reads them without a runtime copy)
  const int rc = host_results(h, p, n_sug);
  if (rc) return rc;
  if (!publish_on()) {
    CKH(hipMemcpyAsync(p->h_results, p->d_results, bytes, hipMemcpyDeviceToHost, st));
    CKH(hipStreamSynchronize(st));
    std::memcpy(out, p->h_results, bytes);
    return TPE_OK;
  }
  // (the call's last launch published already: pub_fired, sequence p->seq)
  const bool fired = p->pub_fired;
  p->pub_fired = false;
  const uint64_t seq = fired ? p->seq : ++p->seq;
  if (!fired) CKH(launch_publish(p->d_results, p->h_results, bytes, p->h_flag, seq, st));
  // spin on the completion word (a stream synchronize's wake-up is the
  // larger part of a small suggest's host-side wait); every 2^12 polls the
  // stream is asked for an error, so a failed launch cannot spin forever
  for (uint64_t it = 1;; ++it) {
    if (__atomic_load_n(p->h_flag, __ATOMIC_ACQUIRE) == seq) break;
    __builtin_ia32_pause();
    if ((it & 4095) == 0) {
      const hipError_t q = hipStreamQuery(st);
      if (q != hipSuccess && q != hipErrorNotReady) return fail(h, TPE_E_HIP, hipGetErrorString(q));
      if (q == hipSuccess && __atomic_load_n(p->h_flag, __ATOMIC_ACQUIRE) != seq) {
        // a fused publish short of arrivals leaves its launch-wide ticket
        // counting: clear it, or the next fused publish of this plan would
        // fire early and copy records not yet written
        if (fired) {
          (void)hipMemsetAsync(p->d_ticket + (size_t)p->s_cap * p->P, 0, sizeof(uint32_t), st);
          (void)hipStreamSynchronize(st);
        }
        return fail(h, TPE_E_HIP, "k_publish finished without its completion word");
      }
    }
  }
  std::memcpy(out, p->h_results, bytes);
  return TPE_OK;
}

// the pinned host buffers of a call's results (copy_results; armed before a
// call whose last launch publishes them itself)
int host_results(tpe_engine *h, tpe_plan *p, int64_t n_sug) {
  const size_t bytes = (size_t)n_sug * p->P * sizeof(tpe_result);
  if (bytes > p->h_results_cap) {
    if (p->h_results) (void)hipHostFree(p->h_results);
    p->h_results = nullptr;
    p->h_results_cap = 0;
    const size_t cap = std::max<size_t>(bytes, 4096);
    CKH(hipHostMalloc((void **)&p->h_results, cap, hipHostMallocCoherent | hipHostMallocMapped));
    p->h_results_cap = cap;
  }
  if (publish_on() && !p->h_flag) {
    CKH(hipHostMalloc((void **)&p->h_flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    __atomic_store_n(p->h_flag, (uint64_t)0, __ATOMIC_RELEASE);
  }
  return TPE_OK;
}

// one-hp operator plan cached in the engine
int op_plan(tpe_engine *h, int32_t family, uint32_t flags, int32_t upper, double low,
            double high, double q, int64_t ncap, tpe_plan **out) {
  tpe_hp x{};
  x.family = family;
  x.flags = flags & (TPE_HAS_LOW | TPE_HAS_HIGH | TPE_HAS_Q);
  x.obs_transform = TPE_OBS_IDENT;
  x.upper = upper;
  x.prior_mu = 0.0;
  x.prior_sigma = 1.0;
  x.low = low;
  x.high = high;
  x.q = q;
  tpe_plan *p = h->op;
  const int64_t need_k = std::max<int64_t>(ncap + 1, upper);
  if (!p || p->ncap < ncap || p->kcap < need_k) {
    if (p) { plan_free_buffers(p); delete p; h->op = nullptr; }
    p = new tpe_plan();
    tpe_space sp{};
    sp.n_hp = 1;
    sp.hp = &x;
    x.upper = std::max<int32_t>(upper, 1);
    const int64_t cap = std::max<int64_t>(ncap, 1024);
    std::vector<double> pp_room((size_t)std::max<int64_t>(cap + 1, upper), 0.0);
    sp.n_pprior = (int64_t)pp_room.size();
    sp.pprior = pp_room.data();
    int rc = plan_build(h, &sp, cap, p);
    if (rc) { plan_free_buffers(p); delete p; return rc; }
    h->op = p;
  }
  p->hps[0] = x;
  CKH(hipMemcpyAsync(p->d_hps, &p->hps[0], sizeof(tpe_hp), hipMemcpyHostToDevice, h->stream));
  *out = p;
  return TPE_OK;
}

// upload an explicit mixture into slot `slot` of an operator plan
int put_mixture(tpe_engine *h, tpe_plan *p, int slot, const double *w, const double *mu,
                const double *sg, int64_t k, int32_t kind) {
  hipStream_t st = h->stream;
  CKH(hipMemcpyAsync(p->d_mw + slot * p->kcap, w, k * 8, hipMemcpyHostToDevice, st));
  if (mu) CKH(hipMemcpyAsync(p->d_mmu + slot * p->kcap, mu, k * 8, hipMemcpyHostToDevice, st));
  if (sg) CKH(hipMemcpyAsync(p->d_msig + slot * p->kcap, sg, k * 8, hipMemcpyHostToDevice, st));
  MixInfo mi{};
  mi.K = (int32_t)k;
  mi.kind = kind;
  CKH(hipMemcpyAsync(p->d_info + slot, &mi, sizeof(MixInfo), hipMemcpyHostToDevice, st));
  CKH(hipStreamSynchronize(st));  // mi lives on this frame
  return TPE_OK;
}

bool bad_family(int32_t f) { return f < TPE_GMM || f > TPE_CAT; }

}  // namespace

// ======================================================================
// C ABI
// ======================================================================
extern "C" {

const char *tpe_version(void) { return "tpe-mi355x 0.1 (gfx950)"; }

int tpe_device_count(int32_t *n) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  if (n) *n = c;
  return TPE_OK;
}

int tpe_create(int32_t device, tpe_handle_t *out) {
  if (!out) return TPE_E_INVALID;
  *out = nullptr;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess || c <= 0) return TPE_E_NODEVICE;
  if (device < 0 || device >= c) return TPE_E_NODEVICE;
  if (hipSetDevice(device) != hipSuccess) return TPE_E_HIP;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return TPE_E_HIP;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return TPE_E_NODEVICE;
  auto *h = new tpe_engine();
  h->device = device;
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return TPE_E_HIP;
  }
  for (auto &a : h->aux)
    if (hipStreamCreateWithFlags(&a, hipStreamNonBlocking) != hipSuccess) {
      tpe_destroy(h);
      return TPE_E_HIP;
    }
  *out = h;
  return TPE_OK;
}

int tpe_destroy(tpe_handle_t h) {
  if (!h) return TPE_OK;
  (void)hipSetDevice(h->device);
  if (h->op) { plan_free_buffers(h->op); delete h->op; }
  if (h->stream) (void)hipStreamDestroy(h->stream);
  for (auto a : h->aux) if (a) (void)hipStreamDestroy(a);
  delete h;
  return TPE_OK;
}

const char *tpe_last_error(tpe_handle_t h) { return h ? h->err.c_str() : "null handle"; }

int tpe_synchronize(tpe_handle_t h) {
  if (!h) return TPE_E_INVALID;
  CKH(hipSetDevice(h->device));
  CKH(hipDeviceSynchronize());
  return TPE_OK;
}

int tpe_split(tpe_handle_t h, const double *losses, int64_t n, double gamma,
              int32_t gamma_cap, uint8_t *below_mask) {
  if (!h) return TPE_E_INVALID;
  if (n < 0 || (n > 0 && (!losses || !below_mask))) return fail(h, TPE_E_INVALID, "bad args");
  if (n == 0) return TPE_OK;
  CKH(hipSetDevice(h->device));
  tpe_plan *p;
  int rc = op_plan(h, TPE_GMM, 0, 1, 0, 0, 0, n, &p);
  if (rc) return rc;
  const int32_t nb = (int32_t)std::min<double>(std::ceil(gamma * std::sqrt((double)n)), gamma_cap);
  CKH(hipMemcpyAsync(p->d_losses, losses, n * 8, hipMemcpyHostToDevice, h->stream));
  p->n = n;
  CKH(launch_split(fit_args(p, std::max(nb, 0), 1.0, 25), p->d_below, h->stream));
  CKH(hipMemcpyAsync(below_mask, p->d_below, n, hipMemcpyDeviceToHost, h->stream));
  CKH(hipStreamSynchronize(h->stream));
  return TPE_OK;
}

static int fit_one(tpe_handle_t h, int32_t family, const double *obs, int64_t n,
                   double prior_weight, double prior_mu, double prior_sigma, int32_t upper,
                   const double *pprior, int32_t lf, tpe_plan **pout) {
  tpe_plan *p;
  int rc = op_plan(h, family, 0, upper, 0, 0, 0, n, &p);
  if (rc) return rc;
  p->hps[0].prior_mu = prior_mu;
  p->hps[0].prior_sigma = prior_sigma;
  p->hps[0].upper = upper;
  if (pprior) {
    p->hps[0].flags |= TPE_PCHOICE;
    p->hps[0].pprior_begin = 0;
    CKH(hipMemcpyAsync(p->d_pprior, pprior, upper * 8, hipMemcpyHostToDevice, h->stream));
  }
  CKH(hipMemcpyAsync(p->d_hps, &p->hps[0], sizeof(tpe_hp), hipMemcpyHostToDevice, h->stream));
  if (n > 0) {
    CKH(hipMemcpyAsync(p->d_vals, obs, n * 8, hipMemcpyHostToDevice, h->stream));
    CKH(hipMemsetAsync(p->d_active, 1, n, h->stream));
    CKH(hipMemsetAsync(p->d_below, 1, n, h->stream));
  }
  if (n > 0) CKH(hipMemsetAsync(p->d_losses, 0, n * 8, h->stream));
  p->n = n;
  CKH(launch_fit(fit_args(p, (int32_t)n, prior_weight, lf), 1, h->stream));
  *pout = p;
  return TPE_OK;
}

int tpe_parzen_fit(tpe_handle_t h, const double *obs, int64_t n, double prior_weight,
                   double prior_mu, double prior_sigma, int32_t lf, double *w, double *mu,
                   double *sigma) {
  if (!h) return TPE_E_INVALID;
  if (n < 0 || (n > 0 && !obs) || !w || !mu || !sigma) return fail(h, TPE_E_INVALID, "bad args");
  if (!(prior_sigma > 0)) return fail(h, TPE_E_INVALID, "prior_sigma <= 0");
  CKH(hipSetDevice(h->device));
  tpe_plan *p;
  int rc = fit_one(h, TPE_GMM, obs, n, prior_weight, prior_mu, prior_sigma, 1, nullptr, lf, &p);
  if (rc) return rc;
  const int64_t K = n + 1;
  CKH(hipMemcpyAsync(w, p->d_mw, K * 8, hipMemcpyDeviceToHost, h->stream));
  CKH(hipMemcpyAsync(mu, p->d_mmu, K * 8, hipMemcpyDeviceToHost, h->stream));
  CKH(hipMemcpyAsync(sigma, p->d_msig, K * 8, hipMemcpyDeviceToHost, h->stream));
  CKH(hipStreamSynchronize(h->stream));
  return TPE_OK;
}

int tpe_categorical_posterior(tpe_handle_t h, const int64_t *obs, int64_t n, int32_t upper,
                              double prior_weight, const double *pprior, int32_t lf,
                              double *p_out) {
  if (!h) return TPE_E_INVALID;
  if (n < 0 || (n > 0 && !obs) || upper <= 0 || !p_out) return fail(h, TPE_E_INVALID, "bad args");
  for (int64_t i = 0; i < n; ++i)
    if (obs[i] < 0) return fail(h, TPE_E_INVALID, "negative categorical observation");
  CKH(hipSetDevice(h->device));
  std::vector<double> dv(obs, obs + n);
  tpe_plan *p;
  int rc = fit_one(h, TPE_CAT, dv.data(), n, prior_weight, 0, 1, upper, pprior, lf, &p);
  if (rc) return rc;
  CKH(hipMemcpyAsync(p_out, p->d_mw, upper * 8, hipMemcpyDeviceToHost, h->stream));
  CKH(hipStreamSynchronize(h->stream));
  return TPE_OK;
}

int tpe_score(tpe_handle_t h, int32_t family, const double *x, int64_t n, const double *wb,
              const double *mb, const double *sb, int64_t kb, const double *wa, const double *ma,
              const double *sa, int64_t ka, double low, double high, double q, uint32_t flags,
              double *llik_b, double *llik_a, int64_t *best_index, double *best_score) {
  if (!h) return TPE_E_INVALID;
  if (bad_family(family) || n < 0 || kb <= 0 || ka <= 0 || !wb || !wa)
    return fail(h, TPE_E_INVALID, "bad args");
  if (family != TPE_CAT && (!mb || !sb || !ma || !sa)) return fail(h, TPE_E_INVALID, "bad args");
  if (family == TPE_CAT && kb != ka) return fail(h, TPE_E_INVALID, "p length mismatch");
  const bool hl = flags & TPE_HAS_LOW, hh = flags & TPE_HAS_HIGH;
  if (family != TPE_CAT && (hl || hh)) {
    if (hl != hh) return fail(h, TPE_E_INVALID, "one-sided truncation");
    if (!(low < high)) return fail(h, TPE_E_BOUNDS, "low >= high");
  }
  if (best_index) *best_index = -1;
  if (best_score) *best_score = NAN;
  if (n == 0) return TPE_OK;
  if (family == TPE_CAT) {
    for (int64_t i = 0; i < n; ++i)
      if (!(x[i] >= 0 && x[i] < kb && x[i] == std::floor(x[i])))
        return fail(h, TPE_E_INDEX, "categorical sample out of range");
  }
  if (family == TPE_LGMM && (flags & TPE_HAS_Q)) {
    const double hq = q / 2.0, eh = hh ? std::exp(high) : INFINITY;
    for (int64_t i = 0; i < n; ++i) {
      const double ub = std::min(x[i] + hq, eh);
      if (ub < 0) return fail(h, TPE_E_NEGATIVE, "negative arg to lognormal_cdf");
    }
  }
  CKH(hipSetDevice(h->device));
  tpe_plan *p;
  const int64_t kmax = std::max(kb, ka);
  int rc = op_plan(h, family, flags, family == TPE_CAT ? (int32_t)kb : 1, low, high, q,
                   std::max<int64_t>(kmax, 1), &p);
  if (rc) return rc;
  const int32_t kind = family == TPE_CAT ? 2 : ((flags & TPE_HAS_Q) ? 1 : 0);
  rc = put_mixture(h, p, 0, wb, mb, sb, kb, kind);
  if (rc) return rc;
  rc = put_mixture(h, p, 1, wa, ma, sa, ka, kind);
  if (rc) return rc;
  CKH(launch_prep(p->d_hps, 1, p->d_mw, p->d_mmu, p->d_msig, p->d_info, p->d_coef, p->d_coef32,
                  p->d_coefm, nullptr, p->d_coefe, p->kcap, p->d_scratch, h->stream));
  p->mom_w = moment_on() ? 16 : 0;
  p->mom_h = false;
  rc = ensure_ext(h, p, n);
  if (rc) return rc;
  CKH(hipMemcpyAsync(p->d_ext, x, n * 8, hipMemcpyHostToDevice, h->stream));
  rc = run_external(h, p, 0, p->d_ext, n, llik_b ? p->d_lb : nullptr,
                    llik_a ? p->d_la : nullptr, h->stream);
  if (rc) return rc;
  tpe_result r;
  CKH(hipMemcpyAsync(&r, p->d_results, sizeof(r), hipMemcpyDeviceToHost, h->stream));
  if (llik_b) CKH(hipMemcpyAsync(llik_b, p->d_lb, n * 8, hipMemcpyDeviceToHost, h->stream));
  if (llik_a) CKH(hipMemcpyAsync(llik_a, p->d_la, n * 8, hipMemcpyDeviceToHost, h->stream));
  CKH(hipStreamSynchronize(h->stream));
  if (best_index) *best_index = r.index;
  if (best_score) *best_score = r.score;
  return TPE_OK;
}

int tpe_lpdf(tpe_handle_t h, int32_t family, const double *x, int64_t n, const double *w,
             const double *mu, const double *sigma, int64_t k, double low, double high, double q,
             uint32_t flags, double *out) {
  if (!out && n > 0) return fail(h, TPE_E_INVALID, "bad args");
  return tpe_score(h, family, x, n, w, mu, sigma, k, w, mu, sigma, k, low, high, q, flags, out,
                   nullptr, nullptr, nullptr);
}

int tpe_sample(tpe_handle_t h, int32_t family, const double *w, const double *mu,
               const double *sigma, int64_t k, double low, double high, double q, uint32_t flags,
               uint64_t seed, uint64_t stream, int64_t offset, int64_t n, double *out) {
  if (!h) return TPE_E_INVALID;
  if (bad_family(family) || k <= 0 || !w || n < 0 || (n > 0 && !out))
    return fail(h, TPE_E_INVALID, "bad args");
  if (family != TPE_CAT && (!mu || !sigma)) return fail(h, TPE_E_INVALID, "bad args");
  const bool hl = flags & TPE_HAS_LOW, hh = flags & TPE_HAS_HIGH;
  if (family != TPE_CAT && (hl || hh)) {
    if (hl != hh) return fail(h, TPE_E_INVALID, "one-sided truncation");
    if (!(low < high)) return fail(h, TPE_E_BOUNDS, "low >= high");
  }
  if (n == 0) return TPE_OK;
  CKH(hipSetDevice(h->device));
  tpe_plan *p;
  int rc = op_plan(h, family, flags, family == TPE_CAT ? (int32_t)k : 1, low, high, q, k, &p);
  if (rc) return rc;
  const int32_t kind = family == TPE_CAT ? 2 : ((flags & TPE_HAS_Q) ? 1 : 0);
  rc = put_mixture(h, p, 0, w, mu, sigma, k, kind);
  if (rc) return rc;
  rc = put_mixture(h, p, 1, w, mu, sigma, k, kind);
  if (rc) return rc;
  CKH(launch_prep(p->d_hps, 1, p->d_mw, p->d_mmu, p->d_msig, p->d_info, p->d_coef, p->d_coef32,
                  p->d_coefm, nullptr, p->d_coefe, p->kcap, p->d_scratch, h->stream));
  p->mom_w = moment_on() ? 16 : 0;
  p->mom_h = false;
  rc = ensure_ext(h, p, n);
  if (rc) return rc;
  CKH(launch_sample(p->d_hps, p->d_mw, p->d_mmu, p->d_msig, p->d_info, seed, stream, offset, n,
                    p->d_ext, h->stream));
  CKH(hipMemcpyAsync(out, p->d_ext, n * 8, hipMemcpyDeviceToHost, h->stream));
  CKH(hipStreamSynchronize(h->stream));
  return TPE_OK;
}

// ---------------------------------------------------------------- plans
int tpe_plan_create(tpe_handle_t h, const tpe_space *space, int64_t max_trials, tpe_plan_t *out) {
  if (!h || !out) return TPE_E_INVALID;
  *out = nullptr;
  auto *p = new tpe_plan();
  int rc = plan_build(h, space, max_trials, p);
  if (rc) {
    plan_free_buffers(p);
    delete p;
    return rc;
  }
  *out = p;
  return TPE_OK;
}

int tpe_plan_destroy(tpe_plan_t p) {
  if (!p) return TPE_OK;
  (void)hipSetDevice(p->eng->device);
  graph_reset(p);
  plan_free_buffers(p);
  delete p;
  return TPE_OK;
}

int tpe_plan_num_levels(tpe_plan_t p, int32_t *n) {
  if (!p || !n) return TPE_E_INVALID;
  *n = (int32_t)p->levels.size();
  return TPE_OK;
}

int tpe_plan_set_history(tpe_plan_t p, const double *losses, const double *vals,
                         const uint8_t *active, int64_t n, int32_t on_device, void *stream) {
  if (!p) return TPE_E_INVALID;
  return tpe_plan_update_history(p, n, 0, n, vals, active, n, 0, losses, on_device, stream);
}

// Rows live at stride ncap (FitArgs::ld), so appending trials leaves the rows
// already on the device in place: a call copies only the rows it is given.
int tpe_plan_update_history(tpe_plan_t p, int64_t n, int64_t row0, int64_t n_rows,
                            const double *vals, const uint8_t *active, int64_t src_ld,
                            int64_t loss0, const double *losses, int32_t on_device,
                            void *stream) {
  if (!p) return TPE_E_INVALID;
  tpe_engine *h = p->eng;
  if (n < 0 || n > p->ncap) return fail(h, TPE_E_INVALID, "history larger than max_trials");
  if (row0 < 0 || n_rows < 0 || row0 + n_rows > n || loss0 < 0 || loss0 > n)
    return fail(h, TPE_E_INVALID, "history rows out of range");
  if (n_rows > 0 && (!vals || !active || src_ld < n_rows))
    return fail(h, TPE_E_INVALID, "bad history rows");
  if (loss0 < n && !losses) return fail(h, TPE_E_INVALID, "losses missing");
  CKH(hipSetDevice(h->device));
  hipStream_t st = pick_stream(h, stream);
  const int64_t n_loss = n - loss0;
  if (!on_device && n_rows * p->P <= kPatchVals && n_loss <= kPatchLoss) {
    // the fmin steady state (a row or two, a few losses): the values ride in
    // the kernel arguments -- no staging copy, no host synchronisation
    // -- and deferred: the next fit's blocks write it (one launch less per
    // fmin step); an earlier one still pending goes out first (an empty
    // update -- tpe.suggest's own push after the caller's -- keeps it)
    if (n_rows == 0 && n_loss == 0) {
      p->n = n;
      return TPE_OK;
    }
    int rc = flush_patch(h, p, st);
    if (rc) return rc;
    HistPatch &hp = p->pend;
    hp = HistPatch{};
    hp.row0 = row0; hp.n_rows = n_rows; hp.loss0 = loss0; hp.n_loss = n_loss;
    hp.ld = p->ncap; hp.P = p->P;
    for (int i = 0; i < p->P; ++i)
      for (int64_t r = 0; r < n_rows; ++r) {
        hp.vals[i * n_rows + r] = vals[(int64_t)i * src_ld + r];
        hp.active[i * n_rows + r] = active[(int64_t)i * src_ld + r];
      }
    for (int64_t i = 0; i < n_loss; ++i) hp.losses[i] = losses[i];
    p->has_pend = n_rows > 0 || n_loss > 0;
    if (p->has_pend && !patch_defer_on()) rc = flush_patch(h, p, st);
    if (rc) return rc;
    p->n = n;
    return TPE_OK;
  }
  {
    const int rc = flush_patch(h, p, st);
    if (rc) return rc;
  }
  const hipMemcpyKind kd = on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  if (n_rows > 0 && p->P > 0) {
    CKH(hipMemcpy2DAsync(p->d_vals + row0, (size_t)p->ncap * 8, vals, (size_t)src_ld * 8,
                         (size_t)n_rows * 8, (size_t)p->P, kd, st));
    CKH(hipMemcpy2DAsync(p->d_active + row0, (size_t)p->ncap, active, (size_t)src_ld,
                         (size_t)n_rows, (size_t)p->P, kd, st));
  }
  if (loss0 < n)
    CKH(hipMemcpyAsync(p->d_losses + loss0, losses, (size_t)(n - loss0) * 8, kd, st));
  p->n = n;
  if (!on_device) CKH(hipStreamSynchronize(st));
  return TPE_OK;
}

int tpe_plan_fit(tpe_plan_t p, double gamma, int32_t gamma_cap, double prior_weight, int32_t lf,
                 void *stream) {
  if (!p) return TPE_E_INVALID;
  tpe_engine *h = p->eng;
  CKH(hipSetDevice(h->device));
  hipStream_t st = pick_stream(h, stream);
  const double nbf = std::ceil(gamma * std::sqrt((double)p->n));
  const int32_t nb = (int32_t)std::max(0.0, std::min<double>(nbf, gamma_cap));
  const int rc = fit_launch(h, p, fit_args(p, nb, prior_weight, lf, true), p->P, st);
  if (rc) return rc;
  p->last_nb = nb;
  return TPE_OK;
}

int tpe_plan_get_mixture(tpe_plan_t p, int32_t hp, int32_t side, double *w, double *mu,
                         double *sigma, int64_t cap, int64_t *k) {
  if (!p || !k) return TPE_E_INVALID;
  tpe_engine *h = p->eng;
  if (hp < 0 || hp >= p->P || side < 0 || side > 1) return fail(h, TPE_E_INVALID, "bad hp/side");
  CKH(hipSetDevice(h->device));
  CKH(hipDeviceSynchronize());
  const int64_t slot = 2 * (int64_t)hp + side;
  MixInfo mi;
  CKH(hipMemcpy(&mi, p->d_info + slot, sizeof(mi), hipMemcpyDeviceToHost));
  *k = mi.K;
  if (mi.K > cap) return fail(h, TPE_E_INVALID, "capacity too small");
  if (w) CKH(hipMemcpy(w, p->d_mw + slot * p->kcap, mi.K * 8, hipMemcpyDeviceToHost));
  if (mu) CKH(hipMemcpy(mu, p->d_mmu + slot * p->kcap, mi.K * 8, hipMemcpyDeviceToHost));
  if (sigma) CKH(hipMemcpy(sigma, p->d_msig + slot * p->kcap, mi.K * 8, hipMemcpyDeviceToHost));
  return TPE_OK;
}

int tpe_plan_get_table(tpe_plan_t p, int32_t hp, int32_t side, int32_t which, void *out,
                       int64_t cap_bytes, int64_t *bytes) {
  if (!p || !bytes) return TPE_E_INVALID;
  tpe_engine *h = p->eng;
  if (hp < 0 || hp >= p->P || side < 0 || side > 1 || which < 0 || which > 4)
    return fail(h, TPE_E_INVALID, "bad hp/side/table");
  CKH(hipSetDevice(h->device));
  CKH(hipDeviceSynchronize());
  const int64_t slot = 2 * (int64_t)hp + side;
  const void *src = nullptr;
  if (which == 0) {
    *bytes = p->kcap * (int64_t)sizeof(Coef);
    src = p->d_coef + slot * p->kcap;
  } else if (which == 1) {
    *bytes = p->kcap / kCoefBlock * (int64_t)sizeof(Coef32);
    src = p->d_coef32 + slot * (p->kcap / kCoefBlock);
  } else if (which == 2) {
    *bytes = mom_stride(p->kcap) * (int64_t)sizeof(CoefM);
    src = p->d_coefm + slot * mom_stride(p->kcap);
  } else if (which == 3) {
    *bytes = p->kcap / kCoefBlock * (int64_t)sizeof(CoefM8);
    src = p->d_coefm8 + slot * (p->kcap / kCoefBlock);
  } else {
    *bytes = mom_stride(p->kcap) * (int64_t)sizeof(CoefM8);
    src = p->d_coefmh + slot * mom_stride(p->kcap);
  }
  if (!out) return TPE_OK;
  if (*bytes > cap_bytes) return fail(h, TPE_E_INVALID, "capacity too small");
  CKH(hipMemcpy(out, src, (size_t)*bytes, hipMemcpyDeviceToHost));
  return TPE_OK;
}

int tpe_plan_suggest(tpe_plan_t p, const uint64_t *seeds, int64_t n_sug, int64_t n_cand,
                     int64_t cand_begin, int32_t level, tpe_result *out, int32_t out_on_device,
                     void *stream) {
  return tpe_plan_suggest_shard(p, seeds, n_sug, cand_begin + n_cand, cand_begin, n_cand, level,
                                out, out_on_device, stream);
}

int tpe_plan_suggest_shard(tpe_plan_t p, const uint64_t *seeds, int64_t n_sug, int64_t n_total,
                           int64_t cand_begin, int64_t n_cand, int32_t level, tpe_result *out,
                           int32_t out_on_device, void *stream) {
  if (!p) return TPE_E_INVALID;
  tpe_engine *h = p->eng;
  if (n_sug <= 0 || n_cand < 0 || cand_begin < 0 || !seeds || n_total < cand_begin + n_cand)
    return fail(h, TPE_E_INVALID, "bad args");
  if (level >= (int32_t)p->levels.size()) return fail(h, TPE_E_INVALID, "bad level");
  CKH(hipSetDevice(h->device));
  hipStream_t st = pick_stream(h, stream);
  int rc = ensure_suggest_state(h, p, n_sug, 1);
  if (rc) return rc;
  p->h_seeds.assign(seeds, seeds + n_sug);
  if (n_sug > kInlineSeeds)
    CKH(hipMemcpyAsync(p->d_seeds, seeds, n_sug * 8, hipMemcpyHostToDevice, st));
  if (p->prof_cap > 0) CKH(hipEventRecord(p->ev0, st));
  const int l0 = level < 0 ? 0 : level;
  const int l1 = level < 0 ? (int)p->levels.size() : level + 1;
  for (int l = l0; l < l1; ++l) {
    rc = run_level(h, p, l, n_sug, n_cand, cand_begin, n_total, st);
    if (rc) return rc;
  }
  if (p->prof_cap > 0) CKH(hipEventRecord(p->ev1, st));
  p->timed = true;
  p->evs = p->prof_cap > 0;
  p->last_ncand = n_cand;
  p->last_nsug = n_sug;
  p->last_level = level;
  return copy_results(h, p, n_sug, out, out_on_device, st);
}

// ---- fit + suggest as one captured graph ---------------------------------
namespace {

// enqueue fit + every level's suggest on st (eager or under capture)
int enqueue_step(tpe_engine *h, tpe_plan *p, int32_t nb, double prior_weight, int32_t lf,
                 int64_t n_sug, int64_t n_cand, hipStream_t st) {
  // the moment table only for a step whose suggest takes a sorted draw
  // (run_level's sorted_draw: n_cand x n_sug x level hps >= 2^22) on two-row
  // wave tiles (> kWaveRowSplitMax candidates per suggestion), the only
  // launches that read it; the others skip its ~3-5 us in k_fit.  Whenever it
  // is read, the table is the one tpe_plan_fit writes (mom_width), so a
  // fit_suggest and a fit + suggest score alike (test_fit_suggest_matches_*)
  bool sorted = false;
  for (const auto &l : p->levels)
    sorted |= n_cand * n_sug * (int64_t)l.size() >= ((int64_t)1 << 22);
  {
    const bool mom = sorted && n_cand > kWaveRowSplitMax;
    const int rc = fit_launch(h, p, fit_args(p, nb, prior_weight, lf, mom), p->P, st);
    if (rc) return rc;
  }
  p->last_nb = nb;
  for (int l = 0; l < (int)p->levels.size(); ++l) {
    const int rc = run_level(h, p, l, n_sug, n_cand, 0, n_cand, st);
    if (rc) return rc;
  }
  return TPE_OK;
}

// capture the step, instantiate it and find the nodes patched per call
int capture_step(tpe_engine *h, tpe_plan *p, int32_t nb, double prior_weight, int32_t lf,
                 int64_t n_sug, int64_t n_cand, hipStream_t st) {
  graph_reset(p);
  CKH(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  p->capturing = true;
  const int rc = enqueue_step(h, p, nb, prior_weight, lf, n_sug, n_cand, st);
  p->capturing = false;
  hipGraph_t g = nullptr;
  const hipError_t ec = hipStreamEndCapture(st, &g);
  if (rc || ec != hipSuccess || !g) {
    if (g) (void)hipGraphDestroy(g);
    return rc ? rc : fail(h, TPE_E_HIP, "graph capture failed");
  }
  p->graph = g;
  p->graph_mom_w = p->mom_w;  // the table the captured fit writes (its args are fixed)
  p->graph_mom_h = p->mom_h;
  CKH(hipGraphInstantiate(&p->graph_exec, g, nullptr, nullptr, 0));
  size_t nn = 0;
  CKH(hipGraphGetNodes(g, nullptr, &nn));
  std::vector<hipGraphNode_t> nodes(nn);
  CKH(hipGraphGetNodes(g, nodes.data(), &nn));
  for (hipGraphNode_t nd : nodes) {
    hipGraphNodeType ty;
    CKH(hipGraphNodeGetType(nd, &ty));
    if (ty != hipGraphNodeTypeKernel) continue;
    hipKernelNodeParams kp{};
    CKH(hipGraphKernelNodeGetParams(nd, &kp));
    if (kp.func == fit_kernel_fn(true) || kp.func == fit_kernel_fn(false)) {
      p->fit_nodes.push_back(nd);
      p->fit_params.push_back(kp);
      p->fit_args0.push_back(*static_cast<const FitArgs *>(kp.kernelParams[0]));
    } else if (is_draw_kernel_fn(kp.func) || kp.func == lattice_draw_kernel_fn()) {
      p->draw_nodes.push_back(nd);
      p->draw_params.push_back(kp);
      p->draw_args0.push_back(*static_cast<const ScoreArgs *>(kp.kernelParams[0]));
    }
  }
  if (p->fit_nodes.size() != 1) {
    graph_reset(p);
    return fail(h, TPE_E_HIP, "graph capture: fit node not found");
  }
  p->graph_ok = true;
  return TPE_OK;
}

// patch this call's history length / n_below and seeds, then launch
int launch_step(tpe_engine *h, tpe_plan *p, int32_t nb, const uint64_t *seeds, int64_t n_sug,
                hipStream_t st) {
  for (size_t i = 0; i < p->fit_nodes.size(); ++i) {
    FitArgs fa = p->fit_args0[i];
    fa.n = p->n;
    fa.n_below = nb;
    HistPatch none{};  // (the caller flushed any deferred history update)
    void *args[2] = {&fa, &none};
    hipKernelNodeParams kp = p->fit_params[i];
    kp.kernelParams = args;
    kp.extra = nullptr;
    CKH(hipGraphExecKernelNodeSetParams(p->graph_exec, p->fit_nodes[i], &kp));
  }
  for (size_t i = 0; i < p->draw_nodes.size(); ++i) {
    ScoreArgs da = p->draw_args0[i];
    for (int64_t j = 0; j < n_sug; ++j) da.seed_inline[j] = seeds[j];
    da.n_inline_seeds = (int32_t)n_sug;
    hipKernelNodeParams kp = p->draw_params[i];
    // k_lattice<true> (fused draw) also takes its jobs and output pointer,
    // k_draw_sorted its position buffer
    LatJobs jobs{};
    double2 *lat_out = nullptr;
    int32_t *pos_out = nullptr;
    void *args[3] = {&da, &jobs, &lat_out};
    if (kp.func == lattice_draw_kernel_fn()) {
      jobs = *static_cast<const LatJobs *>(kp.kernelParams[1]);
      lat_out = *static_cast<double2 *const *>(kp.kernelParams[2]);
    } else if (is_sorted_draw_kernel_fn(kp.func)) {
      pos_out = *static_cast<int32_t *const *>(kp.kernelParams[1]);
      args[1] = &pos_out;
    }
    kp.kernelParams = args;
    kp.extra = nullptr;
    CKH(hipGraphExecKernelNodeSetParams(p->graph_exec, p->draw_nodes[i], &kp));
  }
  CKH(hipGraphLaunch(p->graph_exec, st));
  p->last_nb = nb;
  p->mom_w = p->graph_mom_w;  // (no fit_args on replay: the captured fit's table)
  p->mom_h = p->graph_mom_h;
  return TPE_OK;
}

}  // namespace

int tpe_plan_fit_suggest(tpe_plan_t p, double gamma, int32_t gamma_cap, double prior_weight,
                         int32_t lf, const uint64_t *seeds, int64_t n_sug, int64_t n_cand,
                         tpe_result *out, int32_t out_on_device, void *stream) {
  if (!p) return TPE_E_INVALID;
  tpe_engine *h = p->eng;
  if (n_sug <= 0 || n_cand < 0 || !seeds) return fail(h, TPE_E_INVALID, "bad args");
  CKH(hipSetDevice(h->device));
  hipStream_t st = pick_stream(h, stream);
  const double nbf = std::ceil(gamma * std::sqrt((double)p->n));
  const int32_t nb = (int32_t)std::max(0.0, std::min<double>(nbf, gamma_cap));
  // Graph replay is opt-in (TPE_GRAPH=1): on the measured ROCm 7 / MI355X
  // stack a replayed graph starts ~18 us after the previous one, against
  // back-to-back eager launches of one call (tools/host_cost.py).
  static const bool use_graph = std::getenv("TPE_GRAPH") != nullptr;
  const bool graphable = use_graph && n_sug <= kInlineSeeds && p->prof_cap == 0 && !p->census;
  tpe_plan::StepKey key;
  key.prior_weight = prior_weight;
  key.lf = lf;
  key.n_sug = n_sug;
  key.n_cand = n_cand;
  key.stream = (void *)st;
  key.table = (int64_t)nb + 1 <= kTabCap;
  key.fuse = (int64_t)nb + 1 <= kFuseTab;
  key.small = fit_small(p->n);
  int rc = ensure_suggest_state(h, p, n_sug, 1);
  if (rc) return rc;
  p->h_seeds.assign(seeds, seeds + n_sug);
  if (graphable) {  // (a graph's fit node carries no history patch)
    rc = flush_patch(h, p, st);
    if (rc) return rc;
  }
  if (!graphable || !((p->graph_ok && p->graph_key == key) || (p->pending && p->pending_key == key))) {
    // eager (first sight of this shape: it also sizes every buffer)
    if (n_sug > kInlineSeeds)
      CKH(hipMemcpyAsync(p->d_seeds, seeds, n_sug * 8, hipMemcpyHostToDevice, st));
    if (p->prof_cap > 0) CKH(hipEventRecord(p->ev0, st));
    // results to the host: the step's last launch may publish them itself
    // (run_level, tile_draw levels), with the pinned buffers in place first
    p->pub_fired = false;
    p->pub_arm = out && !out_on_device && publish_on() && p->prof_cap == 0 && !p->census;
    if (p->pub_arm) {
      rc = host_results(h, p, n_sug);
      if (rc) { p->pub_arm = false; return rc; }
    }
    rc = enqueue_step(h, p, nb, prior_weight, lf, n_sug, n_cand, st);
    p->pub_arm = false;
    if (rc) {
      // (a publishing launch that went out counts its arrivals: clear the
      // ticket for the plan's next fused publish)
      if (p->pub_fired)
        (void)hipMemsetAsync(p->d_ticket + (size_t)p->s_cap * p->P, 0, sizeof(uint32_t), st);
      p->pub_fired = false;
      return rc;
    }
    if (p->prof_cap > 0) CKH(hipEventRecord(p->ev1, st));
    if (graphable && !(p->graph_ok && p->graph_key == key)) {
      p->pending = true;
      p->pending_key = key;
    }
  } else {
    if (!(p->graph_ok && p->graph_key == key)) {
      rc = capture_step(h, p, nb, prior_weight, lf, n_sug, n_cand, st);
      if (rc) return rc;
      p->graph_key = key;
    }
    if (p->prof_cap > 0) CKH(hipEventRecord(p->ev0, st));
    rc = launch_step(h, p, nb, seeds, n_sug, st);
    if (rc) return rc;
    if (p->prof_cap > 0) CKH(hipEventRecord(p->ev1, st));
  }
  p->timed = true;
  p->evs = p->prof_cap > 0;
  p->last_ncand = n_cand;
  p->last_nsug = n_sug;
  p->last_level = -1;
  return copy_results(h, p, n_sug, out, out_on_device, st);
}

int tpe_plan_get_results(tpe_plan_t p, tpe_result *out, int32_t out_on_device, void *stream) {
  if (!p || !out) return TPE_E_INVALID;
  tpe_engine *h = p->eng;
  CKH(hipSetDevice(h->device));
  return copy_results(h, p, p->last_nsug, out, out_on_device, pick_stream(h, stream));
}

const tpe_result *tpe_plan_results_device(tpe_plan_t p) {
  return p ? reinterpret_cast<const tpe_result *>(p->d_results) : nullptr;
}

int tpe_plan_merge(tpe_plan_t p, const tpe_result *gathered, int32_t world, int32_t level,
                   tpe_result *out, int32_t out_on_device, void *stream) {
  if (!p || !gathered || world <= 0) return TPE_E_INVALID;
  tpe_engine *h = p->eng;
  if (level < 0 || level >= (int32_t)p->levels.size()) return fail(h, TPE_E_INVALID, "bad level");
  CKH(hipSetDevice(h->device));
  hipStream_t st = pick_stream(h, stream);
  const int32_t ns = (int32_t)p->levels[level].size();
  // out_on_device 2: out already holds this plan's records but for the
  // level's merged slots (the level's tpe_plan_suggest_shard wrote them
  // there); k_merge stores those slots into out too, so no copy launch
  // follows the merge
  const bool direct = out && out_on_device == 2;
  CKH(launch_merge(p->d_level_hps + p->level_off[level], ns, (int32_t)p->last_nsug, p->P, world,
                   reinterpret_cast<const Partial *>(gathered), p->d_results, st,
                   direct ? reinterpret_cast<Partial *>(out) : nullptr));
  if (direct) {
    p->pub_fired = false;
    return TPE_OK;
  }
  return copy_results(h, p, p->last_nsug, out, out_on_device, st);
}

int tpe_plan_score_candidates(tpe_plan_t p, int32_t hp, const double *x, int64_t n,
                              double *llik_b, double *llik_a, int64_t *best_index,
                              double *best_score) {
  return tpe_plan_score_candidates_sorted(p, hp, -1, x, n, llik_b, llik_a, best_index,
                                          best_score);
}

int tpe_plan_score_candidates_sorted(tpe_plan_t p, int32_t hp, int32_t mode, const double *x,
                                     int64_t n, double *llik_b, double *llik_a,
                                     int64_t *best_index, double *best_score) {
  if (!p) return TPE_E_INVALID;
  tpe_engine *h = p->eng;
  if (hp < 0 || hp >= p->P || n < 0 || (n > 0 && !x) || mode < -1 || mode > 3)
    return fail(h, TPE_E_INVALID, "bad args");
  if (n > (int64_t)INT32_MAX) return fail(h, TPE_E_INVALID, "too many candidates");
  if (best_index) *best_index = -1;
  if (best_score) *best_score = NAN;
  if (n == 0) return TPE_OK;
  const tpe_hp &H = p->hps[hp];
  if (H.family == TPE_CAT) {
    for (int64_t i = 0; i < n; ++i)
      if (!(x[i] >= 0 && x[i] < H.upper && x[i] == std::floor(x[i])))
        return fail(h, TPE_E_INDEX, "categorical sample out of range");
  }
  CKH(hipSetDevice(h->device));
  hipStream_t st = h->stream;
  CKH(hipDeviceSynchronize());
  int rc = ensure_ext(h, p, n);
  if (rc) return rc;
  CKH(hipMemcpyAsync(p->d_ext, x, n * 8, hipMemcpyHostToDevice, st));
  rc = run_external(h, p, hp, p->d_ext, n, llik_b ? p->d_lb : nullptr,
                    llik_a ? p->d_la : nullptr, st, mode);
  if (rc) return rc;
  tpe_result r;
  CKH(hipMemcpyAsync(&r, p->d_results + hp, sizeof(r), hipMemcpyDeviceToHost, st));
  if (llik_b) CKH(hipMemcpyAsync(llik_b, p->d_lb, n * 8, hipMemcpyDeviceToHost, st));
  if (llik_a) CKH(hipMemcpyAsync(llik_a, p->d_la, n * 8, hipMemcpyDeviceToHost, st));
  CKH(hipStreamSynchronize(st));
  if (best_index) *best_index = r.index;
  if (best_score) *best_score = r.score;
  return TPE_OK;
}

int tpe_plan_profile(tpe_plan_t p, int32_t capacity) {
  if (!p || capacity < 0) return TPE_E_INVALID;
  tpe_engine *h = p->eng;
  CKH(hipSetDevice(h->device));
  CKH(hipDeviceSynchronize());
  for (auto &pr : p->prof) {
    for (auto e : pr.a) (void)hipEventDestroy(e);
    for (auto e : pr.b) (void)hipEventDestroy(e);
    pr.a.assign(capacity, nullptr);
    pr.b.assign(capacity, nullptr);
    pr.pairs.assign(capacity, 0.0);
    pr.n = 0;
    for (int i = 0; i < capacity; ++i) {
      CKH(hipEventCreate(&pr.a[i]));
      CKH(hipEventCreate(&pr.b[i]));
    }
  }
  p->prof_cap = capacity;
  return TPE_OK;
}

int tpe_plan_profile_read(tpe_plan_t p, int32_t kind, double *avg_ms, int64_t *launches,
                          double *pairs_per_launch) {
  if (!p || kind < 0 || kind > KIND_LAT) return TPE_E_INVALID;
  tpe_engine *h = p->eng;
  CKH(hipSetDevice(h->device));
  CKH(hipDeviceSynchronize());
  if (kind == KIND_LAT) {  // k_lattice launches: lattice points x (K_b + K_a)
    auto &pl = p->prof[1];
    std::vector<MixInfo> info(2 * (size_t)p->P);
    CKH(hipMemcpy(info.data(), p->d_info, info.size() * sizeof(MixInfo), hipMemcpyDeviceToHost));
    double tot = 0.0, pairs = 0.0;
    for (int64_t i = 0; i < pl.n; ++i) {
      float ms = 0.f;
      CKH(hipEventElapsedTime(&ms, pl.a[i], pl.b[i]));
      tot += ms;
      for (int hp : p->levels[(int)pl.pairs[i]]) {
        const int k = score_kind(p->hps[hp]);
        if (k == KIND_ERF_G || k == KIND_ERF_L)
          pairs += (double)p->lat[hp].R * ((double)info[2 * hp].K + info[2 * hp + 1].K);
      }
    }
    if (avg_ms) *avg_ms = pl.n ? tot / pl.n : 0.0;
    if (launches) *launches = pl.n;
    if (pairs_per_launch) *pairs_per_launch = pl.n ? pairs / pl.n : 0.0;
    return TPE_OK;
  }
  auto &pr = p->prof[0];  // every scoring launch (all lpdf kinds of a level)
  double tot = 0.0, pairs = 0.0;
  // this kind's pairs in those launches: components per candidate of the
  // kind's hps (all levels), active in the last suggestion (levels' activity
  // is the same for every profiled step)
  std::vector<MixInfo> info(2 * (size_t)p->P);
  std::vector<Partial> res((size_t)std::max<int64_t>(1, p->last_nsug) * p->P);
  CKH(hipMemcpy(info.data(), p->d_info, info.size() * sizeof(MixInfo), hipMemcpyDeviceToHost));
  if (p->d_results)
    CKH(hipMemcpy(res.data(), p->d_results, res.size() * sizeof(Partial), hipMemcpyDeviceToHost));
  double kk = 0.0;  // sum over suggestions of active (K_b + K_a), per suggestion avg
  for (int hp = 0; hp < p->P; ++hp) {
    if (score_kind(p->hps[hp]) != kind || kind == KIND_CAT) continue;
    double act = 0;
    for (int64_t s = 0; s < std::max<int64_t>(1, p->last_nsug); ++s) act += res[s * p->P + hp].active;
    act /= (double)std::max<int64_t>(1, p->last_nsug);
    kk += act * ((double)info[2 * hp].K + info[2 * hp + 1].K);
  }
  for (int64_t i = 0; i < pr.n; ++i) {
    float ms = 0.f;
    CKH(hipEventElapsedTime(&ms, pr.a[i], pr.b[i]));
    tot += ms;
    pairs += pr.pairs[i] * kk;
  }
  if (avg_ms) *avg_ms = pr.n ? tot / pr.n : 0.0;
  if (launches) *launches = pr.n;
  if (pairs_per_launch) *pairs_per_launch = pr.n ? pairs / pr.n : 0.0;
  return TPE_OK;  // the ring is re-armed by tpe_plan_profile
}

int tpe_plan_set_lattice(tpe_plan_t p, int32_t enable) {
  if (!p) return TPE_E_INVALID;
  if (p->lattice_on != (enable != 0)) graph_reset(p);
  p->lattice_on = enable != 0;
  return TPE_OK;
}

int tpe_plan_census(tpe_plan_t p, int32_t enable, int64_t *counts) {
  return tpe_plan_census_n(p, enable, counts, 6);
}

int tpe_plan_census_n(tpe_plan_t p, int32_t enable, int64_t *counts, int32_t n_counts) {
  if (!p || n_counts < 0) return TPE_E_INVALID;
  tpe_engine *h = p->eng;
  CKH(hipSetDevice(h->device));
  CKH(hipDeviceSynchronize());
  if (counts) {
    unsigned long long c[kCensus];
    CKH(hipMemcpy(c, p->d_census, sizeof(c), hipMemcpyDeviceToHost));
    for (int i = 0; i < kCensus && i < n_counts; ++i) counts[i] = (int64_t)c[i];
  }
  CKH(hipMemset(p->d_census, 0, kCensus * sizeof(unsigned long long)));
  p->census = enable != 0;
  return TPE_OK;
}

int tpe_plan_sample_prior(tpe_plan_t p, const uint64_t *seeds, int64_t n_sug, tpe_result *out,
                          int32_t out_on_device, void *stream) {
  if (!p) return TPE_E_INVALID;
  tpe_engine *h = p->eng;
  if (n_sug <= 0 || !seeds) return fail(h, TPE_E_INVALID, "bad args");
  CKH(hipSetDevice(h->device));
  hipStream_t st = pick_stream(h, stream);
  int rc = ensure_suggest_state(h, p, n_sug, 1);
  if (rc) return rc;
  CKH(hipMemcpyAsync(p->d_seeds, seeds, n_sug * 8, hipMemcpyHostToDevice, st));
  PriorArgs a{};
  a.hps = p->d_hps;
  a.n_hp = p->P;
  a.n_levels = (int32_t)p->levels.size();
  a.level_hps = p->d_level_hps;
  a.level_off = p->d_level_off;
  a.cond_parent = p->d_cp;
  a.cond_branch = p->d_cb;
  a.pprior = p->d_pprior;
  a.seeds = p->d_seeds;
  a.results = p->d_results;
  CKH(launch_prior(a, (int32_t)n_sug, st));
  p->last_nsug = n_sug;
  if (!out_on_device) {
    // the host seeds buffer must outlive the async copy: synchronize here
    rc = copy_results(h, p, n_sug, out, 0, st);
    if (rc) return rc;
    return TPE_OK;
  }
  return copy_results(h, p, n_sug, out, out_on_device, st);
}

// value-bucketed, pruned log-sum-exp slots on small draws: opt-in
// (TPE_SMALL_SORT=1, test_gpu_suggest.py).  Measured at config 2 (4096
// candidates): the skip drops 80 % of the pairs and k_score from 33 to 23 us,
// but the extra k_bucket launch costs more than that (suggest 70 -> 78 us)
static bool small_sort_on() {
  static const bool v = [] {
    const char *e = std::getenv("TPE_SMALL_SORT");
    return e && std::atoi(e) != 0;
  }();
  return v;
}

// the moment form of equal-sigma 16-component chunks in prune mode 3
// (CoefM; TPE_MOMENT=0 switches it off: A/B and the parity tests' child
// processes)
static bool moment_on() {
  static const bool v = [] {
    const char *e = std::getenv("TPE_MOMENT");
    return !(e && std::atoi(e) == 0);
  }();
  return v;
}

// candidate buffer per scoring chunk, in doubles (TPE_CHUNK_MB overrides, A/B)
static int64_t chunk_budget() {
  static const int64_t v = [] {
    const char *e = std::getenv("TPE_CHUNK_MB");
    // MB -> doubles.  8 GB (+ 4 GB of positions): config 4's 1e9 candidates
    // of a level in one draw + one scoring launch, config 5's 32-suggestion
    // calls in one chunk -- each launch's tail paid once (config 4 79.3 ->
    // 78.8 ms, config 5 461.3 -> 454.4 ms per step against 2 GB,
    // profiles/rd6/r6_46; 2 GB had been 1-2 % faster than 512 MB)
    return (e ? std::atoll(e) : 8192) << 17;
  }();
  return v;
}

// smallest mixture (components) scored in the one-exponent form on pruned
// tiles; smaller ones keep the per-group lift (TPE_SHIFT_MIN_K overrides:
// A/B and tests).  Round 4: 2048 -> 512 -- config 5 (K_a = 993) 997 -> 885
// ms per 1024-suggestion step, config 3 (K_a ~ 1.4e3) 0.266 -> 0.255 ms;
// below ~128 components (the good-side mixtures) the guard's second attempt
// costs more than the lift saves (0: config 5 905 ms)
static int lse_shift_min() {
  static const int v = [] {
    const char *e = std::getenv("TPE_SHIFT_MIN_K");
    return e ? std::atoi(e) : 512;
  }();
  return v;
}

int tpe_plan_set_prune(tpe_plan_t p, int32_t mode) {
  if (!p || mode < 0 || mode > 3) return TPE_E_INVALID;
  if (p->prune_mode != mode) graph_reset(p);
  p->prune_mode = mode;
  return TPE_OK;
}

int tpe_microbench(tpe_handle_t h, int32_t which, double *per_second) {
  if (!h || !per_second || which < 0 || which > 9) return TPE_E_INVALID;
  CKH(hipSetDevice(h->device));
  hipDeviceProp_t prop;
  CKH(hipGetDeviceProperties(&prop, h->device));
  const int blocks = prop.multiProcessorCount * 8;
  const int iters = which == 2 ? 256 : (which == 3 || which >= 5 ? 512 : (which == 4 ? 128 : 4096));
  double *sink = nullptr;
  CKH(dalloc(&sink, (size_t)blocks * 256));
  hipEvent_t a, b;
  CKH(hipEventCreate(&a));
  CKH(hipEventCreate(&b));
  CKH(launch_micro(which, blocks, iters, sink, h->stream));  // warm-up
  CKH(hipEventRecord(a, h->stream));
  for (int r = 0; r < 4; ++r) CKH(launch_micro(which, blocks, iters, sink, h->stream));
  CKH(hipEventRecord(b, h->stream));
  CKH(hipEventSynchronize(b));
  float ms = 0.f;
  CKH(hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  dfree(sink);
  // results per thread-iteration: exp / FMA chains, erf chains, LSE pairs
  // (4 candidates x 8 components), quantized pairs (2 chains), shifted LSE
  // pairs (4 x 8), block-local fp32 one-exponent LSE pairs (4 x 2 blocks of
  // 8), the fp32 per-group-lift pairs (4 x 8), moment-form pairs (4 x 2
  // chunks of 16), 8-wide moment-form pairs (4 x 2 blocks of 8)
  static const double per_iter[10] = {8.0, 16.0, 4.0, 32.0, 2.0, 32.0, 64.0, 32.0, 128.0, 64.0};
  *per_second = 4.0 * blocks * 256.0 * iters * per_iter[which] / (ms * 1e-3);
  return TPE_OK;
}

int tpe_plan_last_stats(tpe_plan_t p, double *score_ms, double *pairs) {
  if (!p) return TPE_E_INVALID;
  tpe_engine *h = p->eng;
  if (!p->timed) return fail(h, TPE_E_INVALID, "no suggest recorded");
  CKH(hipSetDevice(h->device));
  if (p->evs) {
    CKH(hipEventSynchronize(p->ev1));
    float ms = 0.f;
    CKH(hipEventElapsedTime(&ms, p->ev0, p->ev1));
    if (score_ms) *score_ms = ms;
  } else if (score_ms) {
    *score_ms = NAN;  // not timed: see tpe_plan_profile
  }
  if (pairs) {
    std::vector<MixInfo> info(2 * (size_t)p->P);
    std::vector<Partial> res((size_t)p->last_nsug * p->P);
    CKH(hipMemcpy(info.data(), p->d_info, info.size() * sizeof(MixInfo), hipMemcpyDeviceToHost));
    CKH(hipMemcpy(res.data(), p->d_results, res.size() * sizeof(Partial), hipMemcpyDeviceToHost));
    const int l0 = p->last_level < 0 ? 0 : p->last_level;
    const int l1 = p->last_level < 0 ? (int)p->levels.size() : p->last_level + 1;
    double acc = 0;
    for (int l = l0; l < l1; ++l)
      for (int hp : p->levels[l]) {
        if (p->hps[hp].family == TPE_CAT) continue;
        const double kk = (double)info[2 * hp].K + info[2 * hp + 1].K;
        for (int64_t s = 0; s < p->last_nsug; ++s)
          if (res[s * p->P + hp].active) acc += kk * (double)p->last_ncand;
      }
    *pairs = acc;
  }
  return TPE_OK;
}

}  // extern "C"
