/*
 * tpe_engine.h -- C ABI of the MI355X (gfx950) TPE suggestion engine.
 *
 * Drop-in boundary.  The reference (pminervini/hyperopt, pure Python/numpy)
 * has no FFI of its own; its hot path is a set of pyll `scope` operators
 * evaluated per hyperparameter inside `tpe.suggest`.  Each entry point below
 * replaces one of those operators (operator level, host buffers, synchronous)
 * or the whole evaluation of the posterior graph (plan level, device
 * resident).  The Python binding is hyperopt_amd/_engine.py (ctypes); see
 * INTEGRATION.md for the binding a reference maintainer would add.
 *
 * Conventions: all functions return TPE_OK (0) or a negative TPE_E_* code;
 * tpe_last_error() gives the message.  No exception or abort crosses the ABI.
 * Inputs are never mutated.  One handle must be used by one thread at a
 * time; distinct handles are independent (no global mutable state).
 */
#ifndef TPE_ENGINE_H
#define TPE_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TPE_ENGINE_ABI_VERSION 1

/* Candidate-range alignment of bit-identical sharding: tpe_plan_suggest over
 * [0, n) and over any split of [0, n) into ranges whose boundaries are
 * multiples of TPE_SHARD_ALIGN (merged with tpe_plan_merge) give the same
 * results byte for byte, as long as every part takes the same draw path (the
 * large-draw value-bucketed path runs at >= 2^22 draws per call).  Large
 * draws are value-bucketed in blocks of this many consecutive global
 * candidate indices (of 4096 for suggestions of <= 2^18 candidates, whose
 * block boundaries are among these), and a candidate's pruned log-sum-exp
 * depends on its block.  Unaligned splits still agree under the north-star tie rule. */
#define TPE_SHARD_ALIGN 8192

/* ---- status codes ---------------------------------------------------- */
#define TPE_OK 0
#define TPE_E_INVALID (-1)   /* bad argument / shape  -> TypeError/ValueError     */
#define TPE_E_BOUNDS (-2)    /* low >= high           (tpe.py:80-81, 237-238)     */
#define TPE_E_NEGATIVE (-3)  /* negative lognormal_cdf argument (tpe.py:181-182) */
#define TPE_E_NOMEM (-4)     /* device allocation failed                         */
#define TPE_E_HIP (-5)       /* HIP runtime error                                */
#define TPE_E_NODEVICE (-6)  /* no gfx950 device                                 */
#define TPE_E_INDEX (-7)     /* categorical sample out of range (IndexError)     */

/* ---- posterior families ---------------------------------------------- */
#define TPE_GMM 0  /* GMM1 / GMM1_lpdf          hyperopt/tpe.py:62-166  */
#define TPE_LGMM 1 /* LGMM1 / LGMM1_lpdf        hyperopt/tpe.py:216-301 */
#define TPE_CAT 2  /* categorical / _lpdf       hyperopt/tpe.py:50-57, 573-607 */

/* ---- flags (which optional lpdf / sampler arguments are not None) ----- */
#define TPE_HAS_LOW 1u
#define TPE_HAS_HIGH 2u
#define TPE_HAS_Q 4u
#define TPE_PCHOICE 8u /* categorical with a prior p (hp.pchoice) */

/* ---- observation transform applied before the Parzen fit --------------
 * hyperopt/tpe.py:485-568 (ap_*_sampler).                                  */
#define TPE_OBS_IDENT 0          /* uniform, quniform, normal, qnormal        */
#define TPE_OBS_LOG 1            /* loguniform, lognormal: log(obs)           */
#define TPE_OBS_LOG_CLIP_EXPLOW 2/* qloguniform: log(max(obs, max(EPS, e^low))) */
#define TPE_OBS_LOG_CLIP_EPS 3   /* qlognormal: log(max(obs, EPS))            */

typedef struct tpe_engine *tpe_handle_t;
typedef struct tpe_plan *tpe_plan_t;

/* One hyperparameter of a compiled search space (descriptor
 * table).  For TPE_LGMM, low/high are the log-space bounds exactly as the
 * reference passes them to LGMM1/LGMM1_lpdf. */
typedef struct {
  int32_t family;        /* TPE_GMM / TPE_LGMM / TPE_CAT                  */
  uint32_t flags;        /* TPE_HAS_* / TPE_PCHOICE                       */
  int32_t obs_transform; /* TPE_OBS_*                                     */
  int32_t upper;         /* categorical: number of categories             */
  double prior_mu;       /* Parzen prior (continuous families)            */
  double prior_sigma;
  double low, high, q;   /* sampler / lpdf arguments (valid per flags)    */
  int32_t cond_begin;    /* activity: OR over [cond_begin, +cond_count) of */
  int32_t cond_count;    /*   (parent active && parent value == branch)    */
  int64_t pprior_begin;  /* TPE_PCHOICE: upper probabilities in pprior[]   */
} tpe_hp;

typedef struct {
  int32_t n_hp;
  const tpe_hp *hp;
  int32_t n_cond;
  const int32_t *cond_parent; /* hp index of the controlling choice   */
  const int32_t *cond_branch; /* option index that activates the hp   */
  int64_t n_pprior;
  const double *pprior;
} tpe_space;

/* Per (suggestion, hp) outcome of broadcast_best (tpe.py:749-759). */
typedef struct {
  double score;  /* below_llik - above_llik of the winner (NaN allowed)   */
  double value;  /* the winning candidate                                 */
  int64_t index; /* its global candidate index (-1: hp inactive)          */
  int32_t active;/* 1 if the hp is active in this suggestion              */
  int32_t pad;
} tpe_result;

/* ---- engine ------------------------------------------------------------ */
const char *tpe_version(void);
int tpe_device_count(int32_t *n);
int tpe_create(int32_t device, tpe_handle_t *out);
int tpe_destroy(tpe_handle_t h);
const char *tpe_last_error(tpe_handle_t h);
int tpe_synchronize(tpe_handle_t h);

/* ---- operator level: host buffers, synchronous -------------------------
 * Each mirrors one pyll scope operator of the reference.                   */

/* ap_filter_trials loss ranking (tpe.py:613-641): marks the n_below lowest
 * losses (ties: lowest position first) with 1 in below_mask[n].           */
int tpe_split(tpe_handle_t h, const double *losses, int64_t n, double gamma,
              int32_t gamma_cap, uint8_t *below_mask);

/* adaptive_parzen_normal (tpe.py:398-475): K = n + 1 outputs.             */
int tpe_parzen_fit(tpe_handle_t h, const double *obs, int64_t n,
                   double prior_weight, double prior_mu, double prior_sigma,
                   int32_t lf, double *w, double *mu, double *sigma);

/* categorical posterior (tpe.py:573-607): p[upper].  pprior may be NULL.  */
int tpe_categorical_posterior(tpe_handle_t h, const int64_t *obs, int64_t n,
                              int32_t upper, double prior_weight,
                              const double *pprior, int32_t lf, double *p);

/* GMM1_lpdf / LGMM1_lpdf (tpe.py:104-166, 259-301) of one mixture.  For
 * TPE_CAT, w holds p (k = upper) and mu/sigma are ignored.                */
int tpe_lpdf(tpe_handle_t h, int32_t family, const double *x, int64_t n,
             const double *w, const double *mu, const double *sigma, int64_t k,
             double low, double high, double q, uint32_t flags, double *out);

/* Fused below/above lpdf + broadcast_best argmax (tpe.py:684-698, 749-759).
 * llik_b / llik_a may be NULL (argmax only).                               */
int tpe_score(tpe_handle_t h, int32_t family, const double *x, int64_t n,
              const double *wb, const double *mb, const double *sb, int64_t kb,
              const double *wa, const double *ma, const double *sa, int64_t ka,
              double low, double high, double q, uint32_t flags,
              double *llik_b, double *llik_a, int64_t *best_index,
              double *best_score);

/* GMM1 / LGMM1 / categorical candidate draws (tpe.py:62-93, 216-250,
 * pyll/stochastic.py:104-142) with counter-based Philox4x32-10: draw i uses
 * counter (offset + i, stream), key seed, so any sharding of [0, n) yields
 * the same values.                                                        */
int tpe_sample(tpe_handle_t h, int32_t family, const double *w,
               const double *mu, const double *sigma, int64_t k, double low,
               double high, double q, uint32_t flags, uint64_t seed,
               uint64_t stream, int64_t offset, int64_t n, double *out);

/* ---- plan level: whole tpe.suggest posterior evaluation on device -------
 * A plan holds one compiled space and a device-resident trial history.     */
int tpe_plan_create(tpe_handle_t h, const tpe_space *space, int64_t max_trials,
                    tpe_plan_t *out);
int tpe_plan_destroy(tpe_plan_t p);
int tpe_plan_num_levels(tpe_plan_t p, int32_t *n_levels);

/* History in tid order (tpe.py:820-848): losses[n] (+inf for unfinished),
 * vals[n_hp][n], active[n_hp][n].  on_device != 0: pointers are device
 * memory (e.g. torch tensors); stream: hipStream_t or NULL (the engine's).
 * History updates are stream-ordered, not synchronous: the host buffers may
 * be reused on return, but the device rows change in `stream`'s order, so a
 * fit / suggest on another stream must be ordered after it by the caller
 * (the same stream, or an event).  The same holds for every plan call. */
int tpe_plan_set_history(tpe_plan_t p, const double *losses,
                         const double *vals, const uint8_t *active, int64_t n,
                         int32_t on_device, void *stream);

/* Incremental history update (the columnar trial store appends rows): copy
 * rows [row0, row0 + n_rows) of every hp from vals / active (source layout
 * [n_hp][src_ld]: row r of hp i at vals[i * src_ld + (r - row0)]) and
 * losses [loss0, n) from losses[0 .. n - loss0); the history length becomes
 * n.  Rows outside [row0, row0 + n_rows) keep their device contents.
 * tpe_plan_set_history(n) == update_history(n, 0, n, vals, active, n, 0,
 * losses).  Replaces the per-call re-walk of hyperopt/tpe.py:820-848.      */
int tpe_plan_update_history(tpe_plan_t p, int64_t n, int64_t row0, int64_t n_rows,
                            const double *vals, const uint8_t *active, int64_t src_ld,
                            int64_t loss0, const double *losses, int32_t on_device,
                            void *stream);

/* split + Parzen fit of every hp, both sides (tpe.py:613-641, 398-607).    */
int tpe_plan_fit(tpe_plan_t p, double gamma, int32_t gamma_cap,
                 double prior_weight, int32_t lf, void *stream);

/* Below-side mixture of one hp after tpe_plan_fit (host copy; k = K).     */
int tpe_plan_get_mixture(tpe_plan_t p, int32_t hp, int32_t side, double *w,
                         double *mu, double *sigma, int64_t cap, int64_t *k);

/* Diagnostics / table parity tests: the raw scoring table of slot (hp,
 * side) as written by the last fit -- which 0: the per-component coefficient
 * table (32 B per component, field-major blocks of 8, envelopes in the
 * w-rows), 1: the block-local fp32 table (128 B per block of 8), 2: the
 * moment table of 16-component chunks (64 B each), 3: the 8-wide moment
 * table (128 B per block of 8; written instead of 2 for mixtures of ~1e3
 * components, the other one is then stale), 4: the degree-15 copy of 2's
 * chunks (128 B each, 3's layout; read where a wave's window is too wide
 * for degree 9).  *bytes = the table's
 * size; out may be NULL (size query).  The layouts are internal
 * (tpe_internal.hpp) and may change between versions.                      */
int tpe_plan_get_table(tpe_plan_t p, int32_t hp, int32_t side, int32_t which, void *out,
                       int64_t cap_bytes, int64_t *bytes);

/* Sample + score + argmax for n_suggest suggestions (seeds[s]) on the
 * candidate range [cand_begin, cand_begin + n_cand) of each suggestion, for
 * the hps of one level (level < 0: all levels, single device).  Results for
 * [n_suggest][n_hp] are kept in the plan; out (host or device, may be NULL)
 * receives a copy.                                                         */
int tpe_plan_suggest(tpe_plan_t p, const uint64_t *seeds, int64_t n_suggest,
                     int64_t n_cand, int64_t cand_begin, int32_t level,
                     tpe_result *out, int32_t out_on_device, void *stream);
/* The same for a shard of a larger suggestion: the candidates [cand_begin,
 * cand_begin + n_cand) of an n_total-candidate suggestion (n_total >=
 * cand_begin + n_cand).  n_total picks the scoring tiles (one-row wave tiles
 * up to 2^18 candidates), so the shards of one suggestion score every
 * candidate exactly as the unsharded call does (parallel.ShardedSuggest);
 * tpe_plan_suggest is this with n_total = cand_begin + n_cand.             */
int tpe_plan_suggest_shard(tpe_plan_t p, const uint64_t *seeds, int64_t n_sug, int64_t n_total,
                           int64_t cand_begin, int64_t n_cand, int32_t level, tpe_result *out,
                           int32_t out_on_device, void *stream);

/* tpe_plan_fit + tpe_plan_suggest (all levels, cand_begin 0) in one call:
 * the tpe.suggest posterior evaluation for one history.  Repeated calls of
 * one shape (prior_weight, lf, n_suggest <= 8, n_candidates, stream) may
 * replay a captured hipGraph of the whole step, patched with this call's
 * history length and seeds (opt-in: TPE_GRAPH=1 in the environment; the
 * default enqueues the step's kernels back to back).                      */
int tpe_plan_fit_suggest(tpe_plan_t p, double gamma, int32_t gamma_cap,
                         double prior_weight, int32_t lf, const uint64_t *seeds,
                         int64_t n_suggest, int64_t n_cand, tpe_result *out,
                         int32_t out_on_device, void *stream);

/* Results [n_suggest][n_hp] of the last tpe_plan_suggest (copy), and the
 * device address where the plan keeps them (valid until the next call).   */
int tpe_plan_get_results(tpe_plan_t p, tpe_result *out, int32_t out_on_device,
                         void *stream);
const tpe_result *tpe_plan_results_device(tpe_plan_t p);

/* Multi-device: combine world copies of one level's results ([world][S][P],
 * device memory, e.g. an RCCL all-gather) with numpy argmax semantics and
 * make them the plan's state.  out_on_device 2: `out` is a device buffer
 * that already holds the records the level's tpe_plan_suggest_shard copied
 * out (out_on_device 1); only the level's merged slots are stored into it,
 * by the merge kernel itself (no copy launch after the merge).             */
int tpe_plan_merge(tpe_plan_t p, const tpe_result *gathered, int32_t world,
                   int32_t level, tpe_result *out, int32_t out_on_device,
                   void *stream);

/* Score given candidates of one hp with the plan's fitted mixtures
 * (parity path for reference-sampled candidates).                          */
int tpe_plan_score_candidates(tpe_plan_t p, int32_t hp, const double *x,
                              int64_t n, double *llik_b, double *llik_a,
                              int64_t *best_index, double *best_score);

/* The same, through the production scoring form of large draws: the given
 * candidates are value-bucketed in blocks of TPE_SHARD_ALIGN exactly as
 * k_draw_sorted buckets its draws, then scored on the same tiles with
 * log-sum-exp prune mode `mode` (tpe_plan_set_prune: 0 every pair, 1 block
 * skip, 2 block skip + one exponent per wave, 3 the same in block-local
 * fp32).  Outputs are in the given
 * order.  The parity path of tpe.py:139-144 / 253-256 as the suggest
 * computes it at config 4.                                                 */
int tpe_plan_score_candidates_sorted(tpe_plan_t p, int32_t hp, int32_t mode,
                                     const double *x, int64_t n, double *llik_b,
                                     double *llik_a, int64_t *best_index,
                                     double *best_score);

/* Device time (ms) of the last tpe_plan_suggest, from HIP events on the
 * plan's stream (recorded only while tpe_plan_profile is on, else NaN: an
 * event record drains the pipeline between launches); and the (candidate,
 * component) pairs it evaluated.                                           */
int tpe_plan_last_stats(tpe_plan_t p, double *score_ms, double *pairs);

/* Per-kernel profiling: record HIP events around each of the next `capacity`
 * scoring launches (one per level and candidate chunk; every lpdf kind of the
 * level), then read their average device duration and, for one lpdf kind
 * (0 LSE-GMM, 1 LSE-LGMM, 2 ERF-GMM, 3 ERF-LGMM, 4 categorical), the
 * (candidate, component) pairs per launch of that kind's active hps; kind 5
 * reads the value-lattice launches instead (their average duration and
 * lattice points x components per launch).
 * tpe_plan_profile also clears the ring (capacity 0: off).                  */
int tpe_plan_profile(tpe_plan_t p, int32_t capacity);
int tpe_plan_profile_read(tpe_plan_t p, int32_t kind, double *avg_ms,
                          int64_t *launches, double *pairs_per_launch);

/* Bounded quantized hps (quniform / qloguniform with finite bounds) are by
 * default scored on their value lattice: each distinct value j * q a drawn
 * candidate can take is scored once per suggest call and looked up by every
 * candidate (bit-identical lpdfs; chosen when the lattice is no larger than
 * the candidate count).  enable = 0 scores every candidate on its own (the
 * tpe.py:146-160 / 284-299 work as written), for A/B measurement and tests. */
int tpe_plan_set_lattice(tpe_plan_t p, int32_t enable);

/* Roofline accounting: read (counts may be NULL) and clear the census of the
 * scoring work since the last call -- counts[0] valid quantized (candidate,
 * component) pairs, [1] live ones (not an exact zero), [2] quantized pairs
 * evaluated (live for some lane of their wave), [3] valid log-sum-exp pairs,
 * [4] of [5] the ones evaluated in the one-exponent-per-wave form, [5]
 * log-sum-exp pairs evaluated (outside the component blocks skipped as exact
 * zeros; a wave's retried pass counts again) -- and switch the census on (enable != 0)
 * or off for the following suggests.  counts has 6 entries.               */
int tpe_plan_census(tpe_plan_t p, int32_t enable, int64_t *counts);
/* The same with n_counts entries (up to 12): [6] of [5] the log-sum-exp pairs
 * evaluated in the block-local fp32 per-group-lift form (prune mode 3 on
 * mixtures below the one-exponent size), [7] of [4] the one-exponent pairs
 * evaluated again by a wave's second attempt (its exponent re-centred),
 * [8] of [4] the one-exponent pairs of wide blocks (mode 3's fp64 loop),
 * [9] of [4] the one-exponent pairs evaluated in the moment form of their
 * 16-component chunk (one exp2 + a degree-9 polynomial per chunk) or, [10]
 * of [9], of their 8-component block (one exp2 + a degree-15 polynomial),
 * [11] of [9] the 16-component chunks read at degree 15 (table 4).         */
int tpe_plan_census_n(tpe_plan_t p, int32_t enable, int64_t *counts, int32_t n_counts);

/* Prior draws of n_suggest whole suggestions (rand.suggest, the TPE startup
 * phase: hyperopt/rand.py:14-33, pyll/stochastic.py:30-142): every active hp
 * drawn from its prior, conditional hps routed by their parents' draws;
 * results[s][hp] = (0, value, 0, active=1) or (NaN, NaN, -1, 0) inactive.
 * Counter-based Philox keyed by seeds[s] (stream disjoint from candidate
 * draws); the history is not read.                                          */
int tpe_plan_sample_prior(tpe_plan_t p, const uint64_t *seeds, int64_t n_suggest,
                          tpe_result *out, int32_t out_on_device, void *stream);

/* Large draws score log-sum-exp candidates on value-bucketed tiles.  mode 1
 * skips the blocks of 8 mixture components whose every term is below
 * 2^-(27 + log2 K) of each candidate's largest one (lpdf moved by <= 2^-26
 * ~ 1.5e-8 relative); mode 2 also gives each wave one exponent instead of a
 * per-group max (terms 2^(t - M), M an upper bound of the wave's terms),
 * guarded so no term's fp32 argument exceeds ~|4| where it matters (<= 3e-7
 * relative; else the wave falls back to mode 1); mode 3 (default) computes
 * mode 2's t - M in fp32 about each component block's own centre (packed
 * fp32 FMAs instead of fp64 ones; the exponent difference is exact, the
 * rest O(1), so the error stays at mode 2's level).  mode 0 evaluates every
 * (candidate, component) pair -- A/B measurement, tests.                    */
int tpe_plan_set_prune(tpe_plan_t p, int32_t mode);

/* Register-only microbenchmarks for the roofline: which = 0 v_exp_f32
 * (results/s), 1 fp64 FMA (flop/s), 2 OCML fp64 erf (results/s), 3 the
 * log-sum-exp (candidate, component) pair of the scoring kernel (pairs/s),
 * 4 a live quantized pair (2 fp64 erf; pairs/s), 5 the log-sum-exp pair of
 * the one-exponent-per-wave loop (tpe_plan_set_prune mode 2; pairs/s), 6 the
 * same pair in block-local fp32 (mode 3; pairs/s), 7 the per-group-lift pair
 * in block-local fp32 (mode 3 below the one-exponent size; pairs/s), 8 the
 * moment form of a 16-component chunk (one exp2 + a degree-9 polynomial per
 * candidate and chunk; pairs/s, 16 per chunk evaluation), 9 the 8-wide moment
 * form (one exp2 + a degree-15 polynomial per candidate and block of 8;
 * pairs/s, 8 per block evaluation).                                         */
int tpe_microbench(tpe_handle_t h, int32_t which, double *per_second);

#ifdef __cplusplus
}
#endif
#endif /* TPE_ENGINE_H */
