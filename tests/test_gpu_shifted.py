"""Parity of the production scoring form of large draws (GPU).

At config 4 almost every evaluated (candidate, component) pair runs in the
large-draw form: candidates value-bucketed in 8192-candidate blocks
(k_draw_sorted), log-sum-exp component blocks whose terms are provably below
2^-(27 + log2 K) of the lane maximum skipped, and one exponent per wave
(``lse_chunks_shifted``: prune mode 2 with an fp64 quadratic, mode 3 -- the
default -- with the block-local fp32 quadratic).  These tests anchor that form to the
CPU oracle (the float64 restatement of tpe.py:104-166 / 259-301 with
``logsum_rows`` tpe.py:253-256, pinned to the reference by
tests/test_oracle_golden.py):

* the reference's own config-4 candidates (suggest_cfg4.npz, K_a ~ 9976)
  pushed through the bucketed / pruned / one-exponent path
  (tpe_plan_score_candidates_sorted) against the reference's lliks;
* every LSE kind at K >= 2048 (GMM bounded / unbounded, LGMM bounded /
  unbounded) against oracle lliks of the same candidates;
* the full 1e7-candidate config-4 suggest: each of the 100 winners rescored
  by the oracle, the winner's value regenerated from its global index
  (tpe_sample at offset = index: broadcast_best returns samples[best],
  tpe.py:756-757), and prune modes 3 and 2 against the exhaustive mode 0;
* the same value/index check on config 2 at 2^18 candidates (sorted draws).

Tolerance (north star): |lpdf - oracle| <= 1e-6 * max(1, |oracle|); argmax
identical or a 1e-6 EI tie.  Measured deltas go to $TPE_PARITY_REPORT.
"""
import json
import math
import os

import numpy as np
import pytest

from hyperopt_amd import hp, _engine as E
from hyperopt_amd.base import Domain

from golden_io import load, load_json, unpack
from gpu_util import RTOL, assert_close, argmax_equiv
import big_configs

pytestmark = pytest.mark.gpu
_REPORT = {}


def _record(key, **kw):
    _REPORT[key] = kw
    path = os.environ.get('TPE_PARITY_REPORT_SHIFTED')
    if path:
        with open(path, 'w') as f:
            json.dump(_REPORT, f, indent=1, sort_keys=True)


def _delta(got, want):
    got, want = np.asarray(got, dtype=float), np.asarray(want, dtype=float)
    fin = np.isfinite(got) & np.isfinite(want)
    d = np.abs(got[fin] - want[fin])
    rel = d / np.maximum(1.0, np.abs(want[fin]))
    return dict(max_abs=float(d.max()) if d.size else 0.0,
                max_rel=float(rel.max()) if rel.size else 0.0, n=int(fin.sum()))


def _oracle_obs(dom, losses, vals, active):
    """Per-label (below, above) observations of the history (stable ties,
    the engine's split; tpe.py:613-641)."""
    from oracle import tpe_oracle as O
    tids = np.arange(losses.size)
    out = {}
    for h in dom.space.hps:
        a = active[h.index] == 1
        out[h.label] = O.split_observations(tids[a], vals[h.index][a], tids, losses, 0.25,
                                            kind='stable')
    return out


def _oracle_score(dom, obs, label, x):
    from oracle import tpe_oracle as O
    from oracle_algo import oracle_hps
    spec = oracle_hps(dom.space)[label]
    bo, ao = obs[label]
    with np.errstate(all='ignore'):
        return O.score_hp(spec['dist'], spec['args'], bo, ao, 1.0, np.atleast_1d(x),
                          kind='stable')


def _regen(plan, tabs, i, seed, index):
    """The candidate a suggest drew at global index ``index`` of hp i:
    tpe_sample with the same Philox key / stream / counter."""
    t = tabs[i]
    w, mu, sg = plan.mixture(i, 0)
    eng = plan.engine
    if t.family == E.CAT:
        return eng.sample(E.CAT, w, seed=seed, stream=i, offset=int(index), n=1)[0]
    lo = t.low if t.flags & E.HAS_LOW else None
    hi = t.high if t.flags & E.HAS_HIGH else None
    q = t.q if t.flags & E.HAS_Q else None
    return eng.sample(t.family, w, mu, sg, lo, hi, q, seed=seed, stream=i,
                      offset=int(index), n=1)[0]


def _check_winners(dom, plan, res, seed, n, obs, key):
    """Every active winner: index in range, value = the draw at that index,
    device score = oracle score of that value (1e-6)."""
    tabs = dom.space.engine_tables()[0]
    dev, orc = [], []
    for h in dom.space.hps:
        r = res[h.index]
        if not r['active']:
            continue
        assert 0 <= r['index'] < n, (h.label, r)
        v = _regen(plan, tabs, h.index, seed, r['index'])
        assert v == r['value'], (key, h.label, int(r['index']), v, r['value'])
        o = _oracle_score(dom, obs, h.label, r['value'])
        dev.append(r['score'])
        orc.append(o['llik_b'][0] - o['llik_a'][0])
    assert_close(dev, orc, msg=key + ' winner score vs oracle')
    return dev, orc


# ---------------------------------------------------------------------------
def test_config4_reference_candidates_production_form(cfg4_plan):
    """suggest_cfg4.npz's candidates (4096 per hp, drawn by the reference
    from the below posterior) through the bucketed path in prune modes 1,
    2 and 3: lliks within 1e-6 of the reference's, argmax equivalent, and
    the one-exponent form demonstrably ran (census)."""
    dom, plan = cfg4_plan
    meta = load_json('suggest_big_meta.json')['cfg4']
    d = load('suggest_cfg4.npz')
    for mode in (1, 2, 3):
        plan.census(True)
        stats = {}
        for k, lab in enumerate(meta['labels']):
            h = dom.space.by_label[lab]
            x = unpack(d, 'samples', k)
            lb, la, bi, bs = plan.score_candidates(h.index, x, sorted_mode=mode)
            rb, ra = unpack(d, 'llik_b', k), unpack(d, 'llik_a', k)
            assert_close(lb, rb, msg='cfg4 %s below, mode %d' % (lab, mode))
            assert_close(la, ra, msg='cfg4 %s above, mode %d' % (lab, mode))
            assert argmax_equiv(rb - ra, bi), (lab, mode)
            stats[lab] = dict(below=_delta(lb, rb), above=_delta(la, ra))
        census = plan.census(False, n=10)
        total, shifted, evaluated = census[3], census[4], census[5]
        # (a wave whose one-exponent guard fails counts its pairs again in
        # the exact loop it falls back to)
        assert total >= sum(4096 * (plan.mixture(dom.space.by_label[l].index, 0)[0].size +
                                    plan.mixture(dom.space.by_label[l].index, 1)[0].size)
                            for l in meta['labels'])
        assert 0 < evaluated < total
        if mode >= 2:
            assert shifted > 0.9 * evaluated, census     # the one-exponent form ran
        else:
            assert shifted == 0
        # the moment form of equal-sigma chunks (CoefM): mode 3 only, most of
        # the config-4 pairs (sigmas at the prior_sigma / 100 floor), unless
        # TPE_MOMENT=0 (test_moment_env_off)
        if mode == 3 and os.environ.get('TPE_MOMENT', '1') != '0':
            assert census[9] > 0.5 * evaluated, census
        else:
            assert census[9] == 0, census
        _record('cfg4_reference_candidates_mode%d' % mode, census=list(census), **stats)


def _lse_space():
    return {'u': hp.uniform('u', -5, 5), 'n': hp.normal('n', 0.5, 2.0),
            'lu': hp.loguniform('lu', math.log(1e-3), math.log(10)),
            'ln': hp.lognormal('ln', -1.0, 1.5)}


def _lse_history(dom, n=10000):
    """N = 1e4 trials of the four-kind space (K_a ~ 9976 on each side)."""
    rs = np.random.RandomState(11)
    cols = {'u': rs.uniform(-5, 5, n), 'n': rs.normal(0.5, 2.0, n),
            'lu': np.exp(rs.uniform(math.log(1e-3), math.log(10), n)),
            'ln': np.exp(rs.normal(-1.0, 1.5, n))}
    labels = dom.space.labels
    vals = np.stack([cols[l] for l in labels])
    return np.random.RandomState(12).rand(n), vals, np.ones_like(vals, dtype=np.uint8)


@pytest.fixture(scope='module')
def lse_plan():
    dom = Domain(lambda x: 0.0, _lse_space())
    L, vals, act = _lse_history(dom)
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=L.size)
    plan.set_history(L, vals, act)
    plan.fit()
    return dom, plan, _oracle_obs(dom, L, vals, act)


def test_shifted_form_every_lse_kind_vs_oracle(lse_plan):
    """GMM (bounded, unbounded) and LGMM (bounded, unbounded) at K ~ 1e4:
    8192 draws of the below posterior plus 4096 spread over the prior range
    (the tails, where the guard and the skip thresholds are tightest),
    scored through the bucketed path in modes 1, 2 and 3 against the oracle."""
    dom, plan, obs = lse_plan
    tabs = dom.space.engine_tables()[0]
    rs = np.random.RandomState(3)
    for h in dom.space.hps:
        i = h.index
        assert plan.mixture(i, 1)[0].size >= 9000
        t = tabs[i]
        w, mu, sg = plan.mixture(i, 0)
        lo = t.low if t.flags & E.HAS_LOW else None
        hi = t.high if t.flags & E.HAS_HIGH else None
        x = plan.engine.sample(t.family, w, mu, sg, lo, hi, None, seed=99, stream=i, n=8192)
        if t.family == E.LGMM:
            wide = np.exp(rs.uniform(t.prior_mu - 2.5 * t.prior_sigma,
                                     t.prior_mu + 2.5 * t.prior_sigma, 4096))
        else:
            wide = rs.uniform(t.prior_mu - 2.5 * t.prior_sigma, t.prior_mu + 2.5 * t.prior_sigma,
                              4096)
        if lo is not None:
            wide = np.clip(wide, math.exp(lo) if t.family == E.LGMM else lo,
                           math.exp(hi) if t.family == E.LGMM else hi)
        x = np.concatenate([x, wide])
        ref = _oracle_score(dom, obs, h.label, x)
        for mode in (1, 2, 3):
            plan.census(True)
            lb, la, bi, bs = plan.score_candidates(i, x, sorted_mode=mode)
            census = plan.census(False)
            assert_close(lb, ref['llik_b'], msg='%s below, mode %d' % (h.label, mode))
            assert_close(la, ref['llik_a'], msg='%s above, mode %d' % (h.label, mode))
            with np.errstate(all='ignore'):
                assert argmax_equiv(ref['llik_b'] - ref['llik_a'], bi), (h.label, mode)
            if mode >= 2:
                assert census[4] > 0, (h.label, census)
            _record('lse_%s_mode%d' % (h.label, mode), census=list(census),
                    below=_delta(lb, ref['llik_b']), above=_delta(la, ref['llik_a']))


def test_exact_wave_loop_every_lse_kind_vs_oracle():
    """Mixtures of K ~ 1.5e3 (config 3's branches; config 5's K_a = 993) on
    the bucketed wave tiles: mode 1 keeps the exact per-group-lift loop (the
    census shows no one-exponent pairs); mode 3 scores them in the
    one-exponent form since round 4 (lse_shift_min 512; the census shows it
    ran) -- judged, as the north star says, against the oracle: every kind
    within 1e-6, argmax identical up to 1e-6 EI ties.  (The per-group-lift
    loop in mode 3 at this size: test_shift_min_env_exact_loop.)"""
    dom = Domain(lambda x: 0.0, _lse_space())
    L, vals, act = _lse_history(dom, n=1500)
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=L.size)
    plan.set_history(L, vals, act)
    plan.fit()
    obs = _oracle_obs(dom, L, vals, act)
    tabs = dom.space.engine_tables()[0]
    rs = np.random.RandomState(4)
    for h in dom.space.hps:
        i = h.index
        assert 1000 < plan.mixture(i, 1)[0].size < 2048
        t = tabs[i]
        w, mu, sg = plan.mixture(i, 0)
        lo = t.low if t.flags & E.HAS_LOW else None
        hi = t.high if t.flags & E.HAS_HIGH else None
        x = plan.engine.sample(t.family, w, mu, sg, lo, hi, None, seed=98, stream=i, n=8192)
        wide = rs.uniform(t.prior_mu - 2.5 * t.prior_sigma, t.prior_mu + 2.5 * t.prior_sigma, 4096)
        if t.family == E.LGMM:
            wide = np.exp(wide)
        if lo is not None:
            wide = np.clip(wide, math.exp(lo) if t.family == E.LGMM else lo,
                           math.exp(hi) if t.family == E.LGMM else hi)
        x = np.concatenate([x, wide])
        ref = _oracle_score(dom, obs, h.label, x)
        for mode in (1, 3):
            plan.census(True)
            lb, la, bi, bs = plan.score_candidates(i, x, sorted_mode=mode)
            census = plan.census(False)
            assert_close(lb, ref['llik_b'], msg='%s below, mode %d' % (h.label, mode))
            assert_close(la, ref['llik_a'], msg='%s above, mode %d' % (h.label, mode))
            with np.errstate(all='ignore'):
                assert argmax_equiv(ref['llik_b'] - ref['llik_a'], bi), (h.label, mode)
            if mode == 1 or os.environ.get('TPE_SHIFT_MIN_K', '512') != '512':
                assert census[4] == 0, census
            else:
                assert census[4] > 0, census
            _record('exact_%s_mode%d' % (h.label, mode), census=list(census),
                    below=_delta(lb, ref['llik_b']), above=_delta(la, ref['llik_a']))


def test_shifted_form_clustered_history_vs_oracle():
    """A history of tight clusters with wide gaps (K_a ~ 1e4, sigmas at the
    prior_sigma / 100 floor): the coefficient blocks that straddle a gap put
    components far from their block's centre in units of their own sigma,
    where the block-local fp32 quadratic of mode 3 would cancel
    catastrophically -- those blocks are flagged (kF32Spread) and keep the
    fp64 quadratic.  Every mode against the oracle, candidates on and
    between the clusters."""
    dom = Domain(lambda x: 0.0, {'u': hp.uniform('u', -5, 5), 'n': hp.normal('n', 0.0, 3.0)})
    rs = np.random.RandomState(17)
    n = 10000
    centres = np.array([-4.0, -1.5, 0.2, 3.0])
    # 'n': four tight clusters; 'u': a dense half plus, in the other half,
    # small tight clusters of 4 (a converged optimizer's repeats) among
    # sparse points -- blocks holding both are wide, and a candidate at a
    # small cluster takes its dominant terms from one such block
    small = np.repeat(np.linspace(0.5, 4.5, 12), 4) + 1e-5 * rs.randn(48)
    cols = {'n': centres[rs.randint(0, 4, n)] + 1e-4 * rs.randn(n),
            'u': np.concatenate([rs.uniform(-5, 0, n - 48 - 40), small, rs.uniform(0, 5, 40)])}
    rs.shuffle(cols['u'])
    clusters = {'n': centres, 'u': np.concatenate([centres, np.linspace(0.5, 4.5, 12)])}
    labels = dom.space.labels
    vals = np.stack([cols[l] for l in labels])
    L = np.random.RandomState(18).rand(n)
    act = np.ones_like(vals, dtype=np.uint8)
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=n)
    plan.set_history(L, vals, act)
    plan.fit()
    obs = _oracle_obs(dom, L, vals, act)
    for h in dom.space.hps:
        i = h.index
        cc = clusters[h.label]
        x = np.concatenate([cc[rs.randint(0, cc.size, 6000)] + 0.05 * rs.randn(6000),
                            rs.uniform(-5, 5, 6000)])
        x = np.clip(x, -5, 4.999999)
        ref = _oracle_score(dom, obs, h.label, x)
        for mode in (1, 2, 3):
            lb, la, bi, bs = plan.score_candidates(i, x, sorted_mode=mode)
            assert_close(lb, ref['llik_b'], msg='%s below, mode %d' % (h.label, mode))
            assert_close(la, ref['llik_a'], msg='%s above, mode %d' % (h.label, mode))
            _record('clustered_%s_mode%d' % (h.label, mode),
                    below=_delta(lb, ref['llik_b']), above=_delta(la, ref['llik_a']))


def test_shifted_form_suggest_winners_vs_oracle(lse_plan):
    """A 2^20-candidate suggest of the four-kind space (sorted draws, mode
    2): winners rescored by the oracle and regenerated from their index."""
    dom, plan, obs = lse_plan
    n, seed = 1 << 20, 31
    res = plan.suggest([seed], n)[0]
    dev, orc = _check_winners(dom, plan, res, seed, n, obs, 'lse suggest')
    _record('lse_suggest_winners', **_delta(dev, orc))


def test_config4_full_suggest_winners_vs_oracle(cfg4_plan):
    """The bench workload (config 4, 1e7 candidates per hp; the default
    prune mode 3, and mode 2): every winner's value is the draw at its
    reported global index, and its score is the oracle's lpdf difference at
    that value within 1e-6.  Mode 0 (every pair, exact per-group lift) on
    the same draw: same winners up to 1e-6 EI ties, and each pruned winner
    scores (by the oracle) within 1e-6 of the mode-0 winner."""
    dom, plan = cfg4_plan
    _, L, vals, act = big_configs.cfg4_domain_history(hp, Domain)
    obs = _oracle_obs(dom, L, vals, act)
    n, seed = 10_000_000, 7
    res, dev, orc = {}, {}, {}
    try:
        for mode in (3, 2, 0):
            plan.set_prune(mode)
            res[mode] = plan.suggest([seed], n)[0]
            dev[mode], orc[mode] = _check_winners(dom, plan, res[mode], seed, n, obs,
                                                  'cfg4 mode %d' % mode)
    finally:
        plan.set_prune(3)
    rec = {'mode0_winner_vs_oracle': _delta(dev[0], orc[0])}
    for mode in (3, 2):
        same = res[mode]['index'] == res[0]['index']
        np.testing.assert_array_equal(res[mode]['value'][same], res[0]['value'][same])
        d_same = np.abs(res[mode]['score'][same] - res[0]['score'][same])
        assert (d_same <= RTOL * np.maximum(1.0, np.abs(res[0]['score'][same]))).all()
        o, o0 = np.asarray(orc[mode]), np.asarray(orc[0])
        # the pruned winner is an argmax within tolerance: the oracle ranks it
        # at most 1e-6 below the exhaustive run's winner (and vice versa)
        gap = o0 - o
        assert (np.abs(gap) <= RTOL * np.maximum(1.0, np.abs(o0))).all(), gap.max()
        rec['mode%d_winner_vs_oracle' % mode] = _delta(dev[mode], orc[mode])
        rec['mode%d_vs_mode0_same_index' % mode] = dict(
            n=int(same.sum()), max_abs=float(d_same.max()) if d_same.size else 0.0)
        rec['mode%d_tied_swaps' % mode] = int((~same).sum())
        rec['mode%d_max_oracle_gap' % mode] = float(np.abs(gap).max())
    _record('cfg4_full_suggest', **rec)


def test_config2_sorted_draw_winner_values_regenerate():
    """Config 2 at 2^18 candidates per hp (value-bucketed sorted draws, the
    position arrays in play), two seeds: every winner's value is the draw at
    its global index (the round-2 bisect failure mode: one index reported
    with another candidate's value)."""
    import bench
    dom, losses, vals, act = bench.build_workload('cfg2')
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, act)
    plan.fit()
    obs = _oracle_obs(dom, losses, vals, act)
    n = 1 << 18
    for seed in (5, 123456789):
        res = plan.suggest([seed], n)[0]
        assert res['active'].all()
        _check_winners(dom, plan, res, seed, n, obs, 'cfg2 seed %d' % seed)


def test_config3_wide_and_narrow_sorted_draws_agree():
    """Config 3 (conditional, 1e5 candidates): a single suggestion's level-2
    sorted draw is a launch of <= 2 blocks per CU (k_draw_sorted_wide,
    1024-thread blocks); a batch of 4 is not (256-thread blocks).  The
    draw and its bucket scatter do not depend on the block size, so the
    batch's first suggestion equals the single one bit for bit, and every
    winner's value regenerates from its index."""
    import bench
    dom, losses, vals, act = bench.build_workload('cfg3')
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, act)
    plan.fit()
    n = 100000
    one = plan.suggest([11], n)[0]
    four = plan.suggest([11, 12, 13, 14], n)[0]
    for f in ('active', 'index', 'value', 'score'):
        np.testing.assert_array_equal(one[f], four[f], err_msg=f)
    obs = _oracle_obs(dom, losses, vals, act)
    _check_winners(dom, plan, one, 11, n, obs, 'cfg3 seed 11')


def test_config3_categorical_posteriors_bit_exact():
    """Config 3's categorical hps at N = 1e4 (the root choice: ~1e4 above-side
    observations over 7 bins; each branch's choices ~1.4e3): the plan's fit
    (counting path, no sort, for > 1024 observations over <= 64 bins) gives
    the oracle's posterior bit for bit on both sides (np.bincount order of
    the LF-weighted counts, tpe.py:573-589)."""
    import bench
    from oracle import tpe_oracle as O
    dom, losses, vals, act = bench.build_workload('cfg3')
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, act)
    plan.fit()
    obs = _oracle_obs(dom, losses, vals, act)
    n_checked = 0
    for h in dom.space.hps:
        t = hps[h.index]
        if t.family != E.CAT or t.flags & E.PCHOICE:
            continue
        for side in (0, 1):
            o = obs[h.label][side]
            w = plan.mixture(h.index, side)[0]
            ref = O.categorical_posterior(o, t.upper, 1.0)
            np.testing.assert_array_equal(w[:t.upper], ref, err_msg='%s side %d' % (h.label, side))
            n_checked += o.size > 1024
    assert n_checked >= 2


def test_config5_bench_shape_multichunk_batch_vs_oracle():
    """Config 5 exactly as ``bench.py --config cfg5`` runs it: config 2's
    space and history, one fit_suggest of S = 32 suggestions x 1e6
    candidates, on value-bucketed sorted draws and wave tiles (tpe_engine.hip
    run_level).  Under a 2 GB candidate chunk (TPE_CHUNK_MB=2048, the child
    run of test_config5_multichunk_env) the level runs as several chunks
    whose winners accumulate (ScoreArgs::accumulate); the default 8 GB
    budget runs it in one.
    The reference serves one id per call (tpe.py:812), so parity is per
    suggestion: every winner's value is the draw at its reported global
    index (broadcast_best returns samples[best], tpe.py:756-757), its score
    is the oracle's lpdf difference at that value (1e-6), and suggestion s
    equals the single-seed fit_suggest([seed_s], 1e6) (one chunk) byte for
    byte -- chunk boundaries are multiples of the sorted-draw block
    (TPE_SHARD_ALIGN), so no pruned sum depends on the chunking."""
    import bench
    dom, losses, vals, act = bench.build_workload('cfg2')
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, act)
    obs = _oracle_obs(dom, losses, vals, act)
    n, S = 1_000_000, 32
    seeds = [1_000_003 + 7919 * s for s in range(S)]
    plan.profile(64)
    batch = plan.fit_suggest(seeds, n)
    _, launches, _ = plan.profile_read(0)
    plan.profile(0)
    want = 2 if os.environ.get('TPE_CHUNK_MB') == '2048' else 1
    assert launches >= want, 'the batch ran in %d chunk(s)' % launches
    dev, orc = [], []
    for s, sd in enumerate(seeds):
        assert batch[s]['active'].all()
        d, o = _check_winners(dom, plan, batch[s], sd, n, obs, 'cfg5 batch s=%d' % s)
        dev += d
        orc += o
    _record('cfg5_batch_winners_vs_oracle', **_delta(dev, orc))
    for s in (0, 5, S - 1):
        plan.profile(64)
        one = plan.fit_suggest([seeds[s]], n)[0]
        _, l1, _ = plan.profile_read(0)
        plan.profile(0)
        assert l1 == 1
        np.testing.assert_array_equal(one.view(np.uint8), batch[s].view(np.uint8),
                                      err_msg='suggestion %d: batch vs single' % s)


def _child(code, env):
    """Run ``code`` in a child interpreter (the engine reads its environment
    switches once per process) and return its stdout."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, '-c', code], cwd=root, env=dict(os.environ, **env),
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout


def test_config5_multichunk_env():
    """The config-5 bench-shape test under a 2 GB candidate chunk
    (TPE_CHUNK_MB=2048): the 32-suggestion level in several chunks whose
    winners accumulate, every winner against the oracle and the single-seed
    suggests byte for byte."""
    out = _child('import sys, pytest; sys.exit(pytest.main(["-q", "-x", "-m", "gpu", '
                 '"tests/test_gpu_shifted.py::test_config5_bench_shape_multichunk_batch_vs_oracle"]))',
                 {'TPE_CHUNK_MB': '2048'})
    assert '1 passed' in out, out[-2000:]


def test_shift_min_env_exact_loop():
    """TPE_SHIFT_MIN_K (the engine's one environment switch of the scoring
    form): 100000 keeps every mixture in the per-group-lift loop, whose mode-3
    form (block-local fp32, lse_terms_z / lse_fold_z) is then what K ~ 1.5e3
    mixtures run -- the exact-loop test in a child process with that switch."""
    out = _child('import sys, pytest; sys.exit(pytest.main(["-q", "-x", "-m", "gpu", '
                 '"tests/test_gpu_shifted.py::test_exact_wave_loop_every_lse_kind_vs_oracle"]))',
                 {'TPE_SHIFT_MIN_K': '100000'})
    assert '1 passed' in out, out[-2000:]


def test_moment_env_off():
    """TPE_MOMENT=0 (the moment form of equal-sigma chunks off: every
    one-exponent pair in the block-local fp32 pair form): the config-4
    reference-candidate parity test in a child process with that switch."""
    out = _child('import sys, pytest; sys.exit(pytest.main(["-q", "-x", "-m", "gpu", '
                 '"tests/test_gpu_shifted.py::test_config4_reference_candidates_production_form"]))',
                 {'TPE_MOMENT': '0'})
    assert '1 passed' in out, out[-2000:]


def test_chunk_budget_env_identical_results():
    """TPE_CHUNK_MB (candidate buffer per scoring chunk): a 64 MB budget runs
    a 1e6-candidate config-2 suggest in 3 chunks (accumulated winners), the
    default in one -- byte-identical results (chunk boundaries are multiples
    of the sorted-draw block, TPE_SHARD_ALIGN)."""
    code = """
import sys, numpy as np
sys.path.insert(0, 'tests')
import bench
from hyperopt_amd import _engine as E
dom, losses, vals, act = bench.build_workload('cfg2')
hps, conds, pprior = dom.space.engine_tables()
plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=losses.size)
plan.set_history(losses, vals, act)
plan.profile(64)
res = plan.fit_suggest([424242, 77], 1000000)
print('launches', plan.profile_read(0)[1])
print('hex', res.view(np.uint8).tobytes().hex())
"""
    a = _child(code, {'TPE_CHUNK_MB': '64'})
    b = _child(code, {})
    la = int(a.split('launches ')[1].split()[0])
    lb = int(b.split('launches ')[1].split()[0])
    assert la >= 3 and lb == 1, (la, lb)
    assert a.split('hex ')[1].strip() == b.split('hex ')[1].strip()


@pytest.mark.parametrize('env', [{'TPE_LOOKUP_DRAW': '0'}, {'TPE_LOOKUP_FORK': '0'},
                                 {'TPE_SIDE_STREAMS': '1'}, {'TPE_PUBLISH': '0'},
                                 {'TPE_TILE_DRAW': '0'}, {'TPE_PUBLISH_FUSE': '0'}],
                         ids=['lookup_from_draw', 'lookup_in_order', 'side_streams', 'no_publish',
                              'no_tile_draw', 'publish_launch'])
def test_launch_switches_identical_results(env):
    """The launch-shape switches change no result: lookup slots written by
    the sorted draw instead of drawn in their tiles (TPE_LOOKUP_DRAW=0), the
    lookup launch in order instead of forked (TPE_LOOKUP_FORK=0), the forked
    lattice / mixed-level launches (TPE_SIDE_STREAMS=1), the runtime copy
    of the results (TPE_PUBLISH=0), k_draw for tiny draws instead of the
    tiles drawing (TPE_TILE_DRAW=0) and k_publish after such a call's last
    launch instead of that launch publishing (TPE_PUBLISH_FUSE=0) -- a
    config-3 suggest of 1e5 candidates (two levels, lattice and categorical
    lookups beside log-sum-exp slots), a batched config-2 suggest of 3e5 and
    tpe.suggest batches of 24 and 1000 candidates over a space without
    quantized hps and over a conditional one, identical to the defaults."""
    code = """
import sys, numpy as np
sys.path.insert(0, 'tests')
import bench
from hyperopt_amd import _engine as E
out = []
for cfg, seeds, n in (('cfg3', [31337], 100000), ('cfg2', [5, 6, 7], 300000)):
    dom, losses, vals, act = bench.build_workload(cfg)
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, act)
    res = plan.fit_suggest(seeds, n)
    assert (res['index'][res['active'] != 0] >= 0).all()
    out.append(res.view(np.uint8).tobytes().hex())
# tiny draws of a space without quantized hps (the tile-draw path): tpe.suggest
from hyperopt_amd import hp, tpe, rand, Trials
from hyperopt_amd.base import Domain
space = {'u': hp.uniform('u', -3, 2), 'l': hp.loguniform('l', -4, 1),
         'c': hp.choice('c', [0, 1, 2, 3]), 'n': hp.normal('n', 0, 2)}
cond = {'k': hp.choice('k', [{'a': hp.uniform('a', 0, 1)},
                             {'b': hp.normal('b', 0, 1), 'c2': hp.choice('c2', [0, 1])}]),
        'u': hp.uniform('u', -1, 1)}
for sp in (space, cond):
    dom = Domain(lambda x: 0.0, sp)
    t = Trials()
    docs = rand.suggest(list(range(150)), dom, t, 1)
    for d, l in zip(docs, np.random.RandomState(4).rand(150)):
        d['state'] = 2
        d['result'] = {'status': 'ok', 'loss': float(l)}
    t._insert_trial_docs(docs)
    t.refresh()
    for n_ei in (24, 1000):
        for k in (1, 2, 3):
            got = tpe.suggest(t.new_trial_ids(k), dom, t, 77 + k, n_EI_candidates=n_ei)
            out.append(repr([sorted(g['misc']['vals'].items()) for g in got]))
print('hex', ':'.join(out))
"""
    a = _child(code, env)
    b = _child(code, {})
    assert a.split('hex ')[1].strip() == b.split('hex ')[1].strip()


def test_sorted_wave_tiles_argmax_numpy_semantics():
    """The production large-draw form (value-bucketed blocks, wave tiles,
    prune mode 3) returns numpy's argmax of its own lpdf difference
    (tpe.py:749-759): over 3e5 candidates of a GMM and an LGMM hp the index
    is argmax(lb - la) of the returned lpdfs, and with NaN candidates it is
    the first NaN (every NaN wave falls back to the exact loop; the record
    selects are branch-free)."""
    import bench
    dom, losses, vals, act = bench.build_workload('cfg2')
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, act)
    plan.fit()
    rng = np.random.RandomState(5)
    for lab in ('u0', 'lu0'):
        h = dom.space.by_label[lab]
        x = rng.uniform(-5, 5, 300_000) if lab == 'u0' else np.exp(rng.uniform(-6.9, 2.3, 300_000))
        lb, la, bi, bs = plan.score_candidates(h.index, x, sorted_mode=3)
        assert bi == int(np.argmax(lb - la)), (lab, bi)
        assert bs == (lb - la)[bi]
        y = x.copy()
        y[[250_001, 77_777, 123_456]] = np.nan
        lb, la, bi, bs = plan.score_candidates(h.index, y, sorted_mode=3)
        with np.errstate(invalid='ignore'):
            assert bi == int(np.argmax(lb - la)) == 77_777, (lab, bi)
        assert np.isnan(bs)


_MOM = np.dtype([('center', '<f8'), ('base', '<f4'), ('cm', '<f4'), ('gam', '<f4'),
                 ('m', '<f4', (10,)), ('xh', '<f4')])


def test_moment_table_vs_numpy(cfg4_plan):
    """The fit's moment table (CoefM, tpe_plan_get_table) of config-4
    mixtures against a float64 numpy restatement from the plan's own fitted
    mixture: per 16-component chunk of mu-sorted components, centre = mu'
    midpoint, T_k = c_k - a^2 d_k^2, T* = max, m_j = sum_k 2^(T_k - T*) q_k^j / j!
    with q_k = 2 a^2 ln2 d_k, xh = max |q_k|; chunks whose sigmas differ (the
    prior's) are not eligible (xh = +inf).  The degree-15 copy (CoefMH,
    which=4: same chunks, j <= 15) likewise.  fp32 fields to fp32 rounding."""
    dom, plan = cfg4_plan
    LOG2E, LN2 = 1.4426950408889634, math.log(2.0)
    for lab in ('x0', 'x57'):
        hp_i = dom.space.by_label[lab].index
        for side in (0, 1):
            w, mu, sg = plan.mixture(hp_i, side)
            t = plan.table(hp_i, side, 2).view(_MOM)
            th = plan.table(hp_i, side, 4).view(_MOM8)
            K = w.size
            sgc = np.maximum(sg, 1e-12)
            from oracle import tpe_oracle as O
            pacc = np.sum(w * (O.normal_cdf(5.0, mu, sgc) - O.normal_cdf(-5.0, mu, sgc)))
            c = LOG2E * np.log(w / np.sqrt(2 * np.pi * sgc ** 2) / pacc)
            a2 = LOG2E / (2 * sgc ** 2)
            n_ok = 0
            for ch in range(-(-K // 16)):
                sl = slice(16 * ch, min(K, 16 * ch + 16))
                m_, a2_, c_ = mu[sl], a2[sl], c[sl]
                e = t[ch]
                if not np.all(a2_ == a2_[0]):
                    assert np.isinf(e['xh']), (lab, side, ch)
                    continue
                n_ok += 1
                cen = 0.5 * (m_.min() + m_.max())
                d = m_ - cen
                T = c_ - a2_ * d * d
                Ts = T.max()
                rho = np.exp2(T - Ts)
                q = 2 * a2_[0] * LN2 * d
                mom = np.array([np.sum(rho * q ** j) / math.factorial(j) for j in range(10)])
                assert e['center'] == cen
                np.testing.assert_allclose(e['xh'], np.abs(q).max(), rtol=2e-7)   # (rounded up)
                assert e['base'] == np.floor(Ts)
                np.testing.assert_allclose(e['cm'], Ts - np.floor(Ts), atol=2e-7)
                np.testing.assert_allclose(e['gam'], -a2_[0], rtol=1e-7)
                np.testing.assert_allclose(e['m'], mom, rtol=2e-7, atol=1e-30)
                # the degree-15 copy of the same chunk (CoefMH, which=4)
                eh = th[ch]
                momh = np.array([np.sum(rho * q ** j) / math.factorial(j) for j in range(16)])
                assert eh['center'] == cen
                np.testing.assert_allclose(eh['xh'], np.abs(q).max(), rtol=2e-7)
                assert eh['base'] == np.floor(Ts)
                np.testing.assert_allclose(eh['cm'], Ts - np.floor(Ts), atol=2e-7)
                np.testing.assert_allclose(eh['gam'], -a2_[0], rtol=1e-7)
                np.testing.assert_allclose(eh['m'], momh, rtol=2e-7, atol=1e-30)
            if side == 1:
                assert n_ok >= 0.99 * (-(-K // 16)) - 1, (lab, n_ok)


_MOM8 = np.dtype([('center', '<f8'), ('xh', '<f4'), ('base', '<f4'), ('cm', '<f4'), ('gam', '<f4'),
                  ('m', '<f4', (16,)), ('pad', '<f4', (10,))])


def test_moment8_table_vs_numpy():
    """The 8-wide moment table (CoefM8, tpe_plan_get_table which=3) the fit
    writes for config 2's mixtures (N = 1e3: K_a = 993, mom_width 8) against
    a float64 numpy restatement of the plan's own fitted mixture: per block of
    8 mu-sorted components, centre = mu' midpoint, T_k = c_k - a^2 d_k^2,
    m_j = sum_k 2^(T_k - T*) q_k^j / j! (j <= 15), q_k = 2 a^2 ln2 d_k,
    xh = max |q_k|; blocks whose sigmas differ (the prior's) are not
    eligible (xh = +inf).  fp32 fields to fp32 rounding."""
    import bench
    from oracle import tpe_oracle as O
    assert _MOM8.itemsize == 128
    dom, losses, vals, act = bench.build_workload('cfg2')
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, act)
    plan.fit()
    LOG2E, LN2 = 1.4426950408889634, math.log(2.0)
    for lab in ('u0', 'u3'):
        hp_i = dom.space.by_label[lab].index
        t_pm = hps[hp_i].prior_mu
        for side in (0, 1):
            w, mu, sg = plan.mixture(hp_i, side)
            t = plan.table(hp_i, side, 3).view(_MOM8)
            K = w.size
            sgc = np.maximum(sg, 1e-12)
            pacc = np.sum(w * (O.normal_cdf(5.0, mu, sgc) - O.normal_cdf(-5.0, mu, sgc)))
            c = LOG2E * np.log(w / np.sqrt(2 * np.pi * sgc ** 2) / pacc)
            a2 = LOG2E / (2 * sgc ** 2)
            n_ok = 0
            for b in range(-(-K // 8)):
                sl = slice(8 * b, min(K, 8 * b + 8))
                m_, a2_, c_ = mu[sl] - t_pm, a2[sl], c[sl]
                e = t[b]
                if not np.all(a2_ == a2_[0]):
                    assert np.isinf(e['xh']), (lab, side, b)
                    continue
                n_ok += 1
                cen = 0.5 * (m_.min() + m_.max())
                d = m_ - cen
                T = c_ - a2_ * d * d
                Ts = T.max()
                rho = np.exp2(T - Ts)
                q = 2 * a2_[0] * LN2 * d
                mom = np.array([np.sum(rho * q ** j) / math.factorial(j) for j in range(16)])
                assert e['center'] == cen, (lab, side, b)
                np.testing.assert_allclose(e['xh'], np.abs(q).max(), rtol=2e-7)   # (rounded up)
                assert e['base'] == np.floor(Ts)
                np.testing.assert_allclose(e['cm'], Ts - np.floor(Ts), atol=2e-7)
                np.testing.assert_allclose(e['gam'], -a2_[0], rtol=1e-7)
                np.testing.assert_allclose(e['m'], mom, rtol=2e-7, atol=1e-30)
            if side == 1:
                assert K > 900 and n_ok >= 0.99 * (-(-K // 8)) - 1, (lab, n_ok)


def test_config5_moment8_census():
    """Config 5's shape (config 2's space and history, K_a = 993, 1e6
    candidates per suggestion, two-row wave tiles) scores a large share of
    its evaluated log-sum-exp pairs in the 8-wide moment form (census [10]);
    config 3's one-row tiles (1e5 candidates) never read a moment table."""
    import bench
    for cfg, n, frac in (('cfg2', 1_000_000, 0.3), ('cfg3', 100_000, None)):
        dom, losses, vals, act = bench.build_workload(cfg)
        hps, conds, pprior = dom.space.engine_tables()
        plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=losses.size)
        plan.set_history(losses, vals, act)
        plan.census(True)
        plan.fit_suggest([1234567], n)
        census = plan.census(False, n=11)
        if frac is None:
            assert census[9] == 0 and census[5] > 0, (cfg, census)
        else:
            assert census[10] == census[9] > frac * census[5], (cfg, census)
        _record('moment8_census_%s' % cfg, census=list(census))


def test_lookup_scan_edge_lattice_points():
    """The self-drawing lookup scan's early exit (k_score_lookup) stops at the
    slot's best reachable lattice score, which leaves out the lattice's margin
    points: bounded quantized GMM / LGMM hps whose bounds are exact multiples
    of q and whose best value is an edge point of the lattice (the history's
    good trials sit at the bounds), on sorted draws of 2^21 candidates: the
    early-exit records equal the drawn-and-read full scan's
    (TPE_LOOKUP_DRAW=0) byte for byte, and the winners are edge values."""
    code = """
import sys, math, numpy as np
sys.path.insert(0, 'tests')
from hyperopt_amd import hp, rand, Trials, _engine as E
from hyperopt_amd.base import Domain
from hyperopt_amd.tpe import build_history
space = {'a': hp.quniform('a', 0, 10, 1), 'b': hp.qloguniform('b', 0, math.log(64), 1),
         'c': hp.quniform('c', -4, 4, 2)}
dom = Domain(lambda x: 0.0, space)
t = Trials()
docs = rand.suggest(list(range(400)), dom, t, 3)
edge = {'a': 10.0, 'b': 64.0, 'c': 4.0}
for d in docs:
    v = {k: d['misc']['vals'][k][0] for k in edge}
    d['state'] = 2
    d['result'] = {'status': 'ok', 'loss': float(abs(v['a'] - 10) / 11 + abs(v['c'] - 4) / 5 +
                                               abs(math.log(max(v['b'], 1)) - math.log(64)) / 4)}
t._insert_trial_docs(docs)
t.refresh()
_, losses, vals, act = build_history(dom, t, dom.space.labels)
hps, conds, pprior = dom.space.engine_tables()
plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=losses.size)
plan.set_history(losses, vals, act)
res = plan.fit_suggest([99, 100], 1 << 21)
print('vals', sorted((l, float(res[0]['value'][dom.space.by_label[l].index])) for l in edge))
print('hex', res.view(np.uint8).tobytes().hex())
"""
    a = _child(code, {})
    b = _child(code, {'TPE_LOOKUP_DRAW': '0'})
    assert a.split('hex ')[1].strip() == b.split('hex ')[1].strip()
    vals = dict(eval(a.split('vals ')[1].split('\n')[0]))
    # (the GMM lattices' best points are their top edges; the LGMM one is
    # recorded: its EI peak need not sit on the last point)
    assert vals['a'] == 10.0 and vals['c'] == 4.0, vals
    _record('lookup_edge_winners', **vals)
