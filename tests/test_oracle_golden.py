"""Pin the CPU oracle (oracle/tpe_oracle.py) to the reference's own outputs.

The fixtures in tests/golden/ were produced by running the reference (see
tests/golden/make_golden.py).  If the oracle drifts from them, every GPU
parity test that uses it as the checker becomes meaningless, so these run on
CPU in every round.
"""
import numpy as np
import pytest

from golden_io import load, load_json, unpack, ncases, opt
from oracle import tpe_oracle as O
import spaces


def test_split_matches_reference():
    d = load('split.npz')
    for i in range(len(d['gamma'])):
        tids = unpack(d, 'tids', i)
        losses = unpack(d, 'losses', i)
        ot, ov = unpack(d, 'o_tids', i), unpack(d, 'o_vals', i)
        b, a = O.split_observations(ot, ov, tids, losses, d['gamma'][i])
        # same numpy argsort as the reference -> identical, ties included
        np.testing.assert_array_equal(b, unpack(d, 'below', i))
        np.testing.assert_array_equal(a, unpack(d, 'above', i))


def test_split_stable_differs_only_on_ties():
    d = load('split.npz')
    for i in range(len(d['gamma'])):
        tids = unpack(d, 'tids', i)
        losses = unpack(d, 'losses', i)
        ot, ov = unpack(d, 'o_tids', i), unpack(d, 'o_vals', i)
        b, a = O.split_observations(ot, ov, tids, losses, d['gamma'][i], kind='stable')
        rb = unpack(d, 'below', i)
        if len(np.unique(losses)) == len(losses):
            np.testing.assert_array_equal(b, rb)
        # with tied losses only the membership of tied trials may move
        assert len(b) + len(a) == len(ov)


def test_parzen_matches_reference():
    d = load('parzen.npz')
    for i in range(ncases(d, 'obs')):
        obs = unpack(d, 'obs', i)
        pw, pm, ps = d['prior'][i]
        w, mu, sig = O.parzen_fit(obs, pw, pm, ps)
        np.testing.assert_array_equal(mu, unpack(d, 'mu', i))
        np.testing.assert_array_equal(sig, unpack(d, 'sigma', i))
        np.testing.assert_array_equal(w, unpack(d, 'w', i))


def test_lpdf_matches_reference():
    d = load('lpdf.npz')
    names = load_json('lpdf_names.json')
    for i, nm in enumerate(names):
        lg, low, high, q = d['meta'][i]
        low, high, q = opt(low), opt(high), opt(q)
        mb = unpack(d, 'mix_b', i).reshape(3, -1)
        ma = unpack(d, 'mix_a', i).reshape(3, -1)
        x = unpack(d, 'cand', i)
        f = O.lgmm_lpdf if lg else O.gmm_lpdf
        with np.errstate(all='ignore'):
            yb = f(x, *mb, low=low, high=high, q=q)
            ya = f(x, *ma, low=low, high=high, q=q)
        np.testing.assert_array_equal(yb, unpack(d, 'llik_b', i), err_msg=nm)
        np.testing.assert_array_equal(ya, unpack(d, 'llik_a', i), err_msg=nm)
        with np.errstate(all='ignore'):
            assert O.best_index(yb, ya)[0] == d['best'][i]


def test_categorical_matches_reference():
    d = load('categorical.npz')
    for i in range(len(d['upper'])):
        obs = unpack(d, 'obs', i)
        pp = unpack(d, 'pprior', i)
        pp = None if np.isnan(pp).all() else pp
        p = O.categorical_posterior(obs, int(d['upper'][i]), d['pw'][i], pp)
        np.testing.assert_array_equal(p, unpack(d, 'p', i))
        draws = unpack(d, 'draws', i)
        np.testing.assert_array_equal(O.categorical_lpdf(draws, p), unpack(d, 'lpdf', i))
        rng = np.random.RandomState(2000 + i)
        np.testing.assert_array_equal(O.categorical_sample(rng, p, 64), draws)


def test_reference_sampler_streams():
    d = load('samplers.npz')
    mixes = load_json('samplers_mixes.json')
    for i, (mi, lg, low, high, q, seed) in enumerate(d['meta']):
        mix = mixes[int(mi)]
        x = O.gmm_sample(np.random.RandomState(int(seed)), *mix, low=opt(low),
                         high=opt(high), q=opt(q), n=50, log_space=bool(lg))
        np.testing.assert_array_equal(x, unpack(d, 'x', i))


SPACES = {'cfg2': spaces.cfg2_space, 'many_dists': spaces.many_dists_space,
          'cond': spaces.cond_space, 'cfg3_small': spaces.cfg3_space}


def _history(d, labels):
    n = d['losses'].size
    tids = np.arange(n)
    obs = {}
    for i, lab in enumerate(labels):
        act = d['active'][i].astype(bool)
        obs[lab] = (tids[act], d['vals'][i][act])
    return tids, d['losses'], obs


@pytest.mark.parametrize('name', sorted(SPACES))
def test_whole_suggest_reference_stream(name):
    meta = load_json('suggest_meta.json')[name]
    d = load('suggest_%s.npz' % name)
    hps = spaces.describe(SPACES[name](spaces.RecordingHP()))
    labels = meta['labels']
    assert sorted(hps) == labels
    tids, losses, obs = _history(d, labels)
    kw = meta['kw']
    with np.errstate(all='ignore'):
        chosen, detail = O.suggest_reference_stream(
            hps, tids, losses, obs, meta['suggest_seed'],
            n_ei=kw.get('n_EI_candidates', 24))
    for i, lab in enumerate(labels):
        ref = d['chosen'][i]
        if np.isnan(ref):
            assert lab not in chosen
        else:
            assert chosen[lab] == ref, (lab, chosen[lab], ref)
    # per-hp candidates and lliks in the reference's evaluation order
    order = O.hp_order(hps)
    for k, lab in enumerate(order):
        np.testing.assert_array_equal(detail[lab]['cand'], unpack(d, 'samples', k))
        np.testing.assert_array_equal(detail[lab]['llik_b'], unpack(d, 'llik_b', k))
        np.testing.assert_array_equal(detail[lab]['llik_a'], unpack(d, 'llik_a', k))


@pytest.mark.parametrize('name', ['branin', 'distractor', 'gauss_wave', 'gauss_wave2',
                                  'many_dists', 'n_arms', 'q1_lognormal', 'quadratic1'])
def test_oracle_fmin_trajectories_equal_reference(name):
    """The oracle, driven through hyperopt_amd's fmin/Trials host layer,
    replays the reference's TestOpt runs trial for trial (pins both the
    oracle numerics and the host history/seeding semantics)."""
    import functools
    import hyperopt_amd as H
    from hyperopt_amd import hp, Trials, fmin
    from hyperopt_amd.expr import as_apply
    import domains
    from oracle_algo import oracle_suggest, trajectory
    ref = load_json('testopt_traj.json')[name]
    kw, n = domains.settings(name)
    t = Trials()
    fmin(lambda x: x, domains.build(name, hp, H.scope, as_apply),
         algo=functools.partial(oracle_suggest, **kw), max_evals=n, trials=t,
         rstate=np.random.RandomState(123))
    assert trajectory(t) == ref['vals']


def test_oracle_matches_reference_at_config4_size():
    """K_a ~ 9976 (config 4): the oracle's lliks of the reference-drawn
    candidates equal the reference's bit for bit (hps x0, x42)."""
    from big_configs import cfg4_columns
    meta = load_json('suggest_big_meta.json')['cfg4']
    d = load('suggest_cfg4.npz')
    U, L = cfg4_columns()
    tids = np.arange(L.size)
    for k, lab in enumerate(meta['labels']):
        if lab not in ('x0', 'x42'):
            continue
        i = int(lab[1:])
        bo, ao = O.split_observations(tids, U[:, i], tids, L, 0.25)
        x = unpack(d, 'samples', k)
        assert ao.size + 1 >= 9900
        r = O.score_hp('uniform', (-5, 5), bo, ao, 1.0, x)
        np.testing.assert_array_equal(r['llik_b'], unpack(d, 'llik_b', k))
        np.testing.assert_array_equal(r['llik_a'], unpack(d, 'llik_a', k))
