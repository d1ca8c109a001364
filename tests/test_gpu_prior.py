"""Device prior draws (rand.suggest / TPE startup on the GPU):
statistical parity with the reference's priors (pyll/stochastic.py:30-142)
and the conditional routing of hyperopt/vectorize.py:20-38."""
import numpy as np
import pytest
from scipy import stats

from hyperopt_amd import hp, rand, tpe, Trials
from hyperopt_amd.base import Domain
import spaces

pytestmark = pytest.mark.gpu
S = 20000


def _plan(space):
    dom = Domain(lambda x: 0.0, space)
    st = tpe._state(dom)
    from hyperopt_amd import _engine as E
    return dom, st.plan_for(dom, 1, E.default_engine())


def _cdf_q(cdf, q, lo=-np.inf, hi=np.inf):
    """P(round(X / q) * q == v) for the lattice values v seen."""
    def p(v):
        a, b = v - q / 2, v + q / 2
        return cdf(min(max(b, lo), hi)) - cdf(min(max(a, lo), hi))
    return p


def test_prior_distributions_all_kinds():
    dom, plan = _plan(spaces.many_dists_space(hp))
    res = plan.sample_prior(tpe.batch_seeds(99, S))
    cs = dom.space
    assert res['active'].all() and (res['index'] == 0).all()
    col = {h.label: res[:, h.index]['value'] for h in cs.hps}
    alpha = 1e-4
    # continuous: KS against the exact prior
    assert stats.kstest(col['c'], stats.uniform(4, 3).cdf).pvalue > alpha
    assert stats.kstest(np.log(col['d']), stats.uniform(-2, 2).cdf).pvalue > alpha
    assert stats.kstest(col['g'], stats.norm(4, 7).cdf).pvalue > alpha
    assert stats.kstest(np.log(col['h']), stats.norm(-2, 2).cdf).pvalue > alpha
    # categorical: chi-square against p
    for lab, p in (('a', [1 / 3] * 3), ('b', [0.1] * 10), ('k', [0.1, 0.9])):
        cnt = np.bincount(col[lab].astype(int), minlength=len(p))
        assert len(cnt) == len(p)
        assert stats.chisquare(cnt, np.asarray(p) * S).pvalue > alpha, lab
    # quantized: lattice values with the exact rounding probabilities
    checks = {'e': (3.0, stats.uniform(0, 10).cdf, False),
              'i': (2.0, stats.norm(0, 10).cdf, False),
              'f': (2.0, stats.uniform(0, 3).cdf, True),
              'j': (1.0, stats.norm(0, 2).cdf, True)}
    for lab, (q, cdf, logn) in checks.items():
        v = col[lab]
        assert np.all(v == np.round(v / q) * q), lab
        vals, cnt = np.unique(v, return_counts=True)
        if logn:
            probs = np.array([max(0.0, cdf(np.log(max(x + q / 2, 1e-300)))
                                  - (cdf(np.log(x - q / 2)) if x - q / 2 > 0 else 0.0))
                              for x in vals])
        else:
            probs = np.array([cdf(x + q / 2) - cdf(x - q / 2) for x in vals])
        keep = probs * S >= 20
        assert keep.sum() >= 2, lab
        exp = probs[keep] / probs[keep].sum() * cnt[keep].sum()
        assert stats.chisquare(cnt[keep], exp).pvalue > alpha, lab


def test_prior_conditional_routing_and_device_rand_suggest():
    dom, plan = _plan(spaces.cond_space(hp))
    cs = dom.space
    res = plan.sample_prior(tpe.batch_seeds(5, S))
    top = res[:, cs.by_label['top'].index]['value'].astype(int)
    assert set(np.unique(top)) == {0, 1, 2}
    assert stats.chisquare(np.bincount(top, minlength=3)).pvalue > 1e-4
    for b in range(3):
        for lab in ('lr%d' % b, 'units%d' % b, 'act%d' % b, 'zz%d' % b):
            act = res[:, cs.by_label[lab].index]['active'].astype(bool)
            np.testing.assert_array_equal(act, top == b)
    u = res[top == 1, cs.by_label['units1'].index]['value']
    assert np.all((u >= 1) & (u <= 1024) & (u == np.round(u)))
    # rand.suggest on the device: docs shaped like the reference's
    t = Trials()
    docs = rand.suggest(list(range(50)), dom, t, 17, rng_stream='philox')
    again = rand.suggest(list(range(50)), dom, t, 17, rng_stream='philox')
    assert [d['misc']['vals'] for d in docs] == [d['misc']['vals'] for d in again]
    for d in docs:
        v = d['misc']['vals']
        b = v['top'][0]
        assert isinstance(b, int) and len(v['aa']) == 1
        for lab in cs.labels:
            if lab[:-1] in ('lr', 'units', 'act', 'zz'):
                assert (len(v[lab]) == 1) == (int(lab[-1]) == b)
    # the TPE startup phase takes the same device path with startup_stream='philox'
    s1 = tpe.suggest([0], dom, Trials(), 3, startup_stream='philox')[0]['misc']['vals']
    assert s1 == rand.suggest([0], dom, Trials(), 3, rng_stream='philox')[0]['misc']['vals']


def test_tpe_with_device_startup_reaches_optimum():
    """A whole fmin on the device path: startup prior draws + TPE suggests."""
    import functools
    from hyperopt_amd import fmin
    t = Trials()
    fmin(lambda x: (x - 3) ** 2, hp.uniform('x', -5, 5),
         algo=functools.partial(tpe.suggest, startup_stream='philox', n_EI_candidates=256),
         max_evals=80, trials=t, rstate=np.random.RandomState(4))
    assert len(t) == 80 and min(t.losses()) < 1e-2
