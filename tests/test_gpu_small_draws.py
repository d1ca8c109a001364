"""Small draws in prune mode 3 and the suggest's EI-only finalize (GPU).

A draw of fewer than 2^22 (candidate, slot) pairs is scored unbucketed on
8-wave component-split tiles (tpe_engine.hip run_level); in the default
prune mode 3 its log-sum-exp pairs take the block-local fp32 form
(ScoreArgs::lse_f32, the default ``tpe.suggest`` path at n_EI_candidates 24
or 4096).  These tests pin that arithmetic to the oracle (the float64
restatement of tpe.py:104-166 / 259-301) and to the exhaustive fp64 form
(prune mode 0), for GMM, LGMM and a conditional space.

The suggest's finalize computes EI as ((m_b - m_a) + log2(s_b / s_a)) ln 2
(LGMM's log x cancels) when no lpdf is requested; the operator / parity
paths compute lpdf_b - lpdf_a.  ``score_candidates(want_llik=False)`` runs
the EI-only branch, which must return numpy's argmax of the lpdf difference
(first maximum, first NaN, tpe.py:749-759) with NaN and tied candidates
(ADVICE r4, low).
"""
import math

import numpy as np
import pytest

from hyperopt_amd import hp, rand, Trials, trials_from_docs, _engine as E
from hyperopt_amd.base import Domain
from hyperopt_amd.tpe import build_history

from gpu_util import RTOL, argmax_equiv, assert_close
from test_gpu_shifted import _check_winners, _lse_history, _lse_space, _oracle_obs, _oracle_score
import spaces

pytestmark = pytest.mark.gpu


def _plan(dom, L, vals, act):
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=L.size)
    plan.set_history(L, vals, act)
    plan.fit()
    return plan


def _cond_workload(n=400):
    dom = Domain(lambda x: 0.0, spaces.cond_space(hp))
    docs = rand.suggest(list(range(n)), dom, Trials(), 5)
    for d, l in zip(docs, np.random.RandomState(6).rand(n)):
        d['state'] = 2
        d['result'] = {'status': 'ok', 'loss': float(l)}
    _, L, vals, act = build_history(dom, trials_from_docs(docs), dom.space.labels)
    return dom, np.asarray(L), vals, act


@pytest.mark.parametrize('space', ['lse', 'cond'])
def test_small_draw_mode3_winners_vs_oracle_and_mode0(space):
    """n_EI_candidates 24 and 4096, mode 3 (default) and mode 0 on the same
    draw: every winner's value is the draw at its index and its score the
    oracle's lpdf difference at that value (1e-6); where the two modes pick
    different candidates, the oracle ranks them within 1e-6 of each other."""
    if space == 'lse':
        dom = Domain(lambda x: 0.0, _lse_space())
        L, vals, act = _lse_history(dom, n=1500)
    else:
        dom, L, vals, act = _cond_workload()
    plan = _plan(dom, L, vals, act)
    obs = _oracle_obs(dom, L, vals, act)
    try:
        for n in (24, 4096):
            for seed in (3, 1234567):
                res = {}
                orc = {}
                for mode in (3, 0):
                    plan.set_prune(mode)
                    res[mode] = plan.suggest([seed], n)[0]
                    _, orc[mode] = _check_winners(dom, plan, res[mode], seed, n, obs,
                                                  '%s n=%d seed=%d mode %d' % (space, n, seed, mode))
                np.testing.assert_array_equal(res[3]['active'], res[0]['active'])
                same = res[3]['index'] == res[0]['index']
                np.testing.assert_array_equal(res[3]['value'][same], res[0]['value'][same])
                act3 = res[3]['active'] == 1
                assert_close(res[3]['score'][act3], res[0]['score'][act3],
                             msg='%s n=%d mode 3 vs 0 scores' % (space, n))
                o3, o0 = np.asarray(orc[3]), np.asarray(orc[0])
                assert (np.abs(o0 - o3) <= RTOL * np.maximum(1.0, np.abs(o0))).all()
    finally:
        plan.set_prune(3)


def test_ei_only_finalize_numpy_argmax_semantics():
    """The EI-only finalize (no lpdf outputs, the suggest's branch) on GMM
    and LGMM hps, 8-wave tiles (unsorted) and sorted wave tiles: the index is
    argmax(lb - la) of the lpdf path on the same candidates, the score
    equals that difference within 1e-6; tied candidates (duplicated values)
    resolve to the first; a NaN candidate wins at its first index; an LGMM
    candidate x = 0 (log x = -inf, the reference's lpdf - log x is NaN)
    scores NaN as well."""
    import bench
    dom, losses, vals, act = bench.build_workload('cfg2')
    plan = _plan(dom, losses, vals, act)
    rng = np.random.RandomState(8)
    for lab in ('u1', 'lu1'):
        h = dom.space.by_label[lab]
        lg = lab.startswith('lu')
        for mode, n in ((None, 4096), (3, 300_000)):
            x = np.exp(rng.uniform(-6.9, 2.3, n)) if lg else rng.uniform(-5, 5, n)
            lb, la, bi, bs = plan.score_candidates(h.index, x, sorted_mode=mode)
            ei = lb - la
            # tie: the winner's value repeated earlier in the array
            w = int(np.argmax(ei))
            y = x.copy()
            y[w // 3] = x[w]
            lb, la, bi_l, bs_l = plan.score_candidates(h.index, y, sorted_mode=mode)
            _, _, bi_e, bs_e = plan.score_candidates(h.index, y, sorted_mode=mode, want_llik=False)
            assert bi_l == int(np.argmax(lb - la)), (lab, mode, bi_l)
            if mode is None:
                # every candidate's sums in one association: equal values
                # score equal, and the first of them wins on both paths
                assert bi_l == w // 3 and bi_e == bi_l, (lab, bi_l, bi_e, w)
            else:
                # (pruned sums depend on the candidate's wave window: equal
                # values in different waves tie within the skip bound)
                assert argmax_equiv(lb - la, bi_e), (lab, mode, bi_e, bi_l)
            assert abs(bs_e - bs_l) <= RTOL * max(1.0, abs(bs_l)), (bs_e, bs_l)
            # NaN candidates: the first NaN wins on both paths
            z = y.copy()
            z[[n - 5, n // 2, n // 7 + 1]] = np.nan
            if lg:
                z[n // 9] = 0.0          # log x = -inf: NaN lpdf in the reference
            lb, la, bi_l, bs_l = plan.score_candidates(h.index, z, sorted_mode=mode)
            _, _, bi_e, bs_e = plan.score_candidates(h.index, z, sorted_mode=mode, want_llik=False)
            first = min(n // 7 + 1, n // 9) if lg else n // 7 + 1
            with np.errstate(invalid='ignore'):
                assert bi_l == int(np.argmax(lb - la)) == first, (lab, mode, bi_l)
            assert bi_e == first and math.isnan(bs_e), (lab, mode, bi_e, bs_e)
            if lg:
                o = _oracle_score(dom, _oracle_obs(dom, losses, vals, act), lab, np.array([0.0]))
                with np.errstate(invalid='ignore'):
                    assert math.isnan(o['llik_b'][0] - o['llik_a'][0])
