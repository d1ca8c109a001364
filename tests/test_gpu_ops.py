"""GPU parity of the operator-level C ABI against the reference's golden
vectors and the CPU oracle.  Every call goes through libtpe_engine.so."""
import numpy as np
import pytest

from golden_io import load, load_json, unpack, ncases, opt
from gpu_util import assert_close, argmax_equiv, close
from oracle import tpe_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def eng():
    from hyperopt_amd._engine import Engine
    return Engine(0)


def test_split_matches_oracle(eng):
    d = load('split.npz')
    for i in range(len(d['gamma'])):
        losses = unpack(d, 'losses', i)
        tids = unpack(d, 'tids', i)
        mask = eng.split(losses, d['gamma'][i])
        good, _ = O.below_tids(tids, losses, d['gamma'][i], kind='stable')
        assert set(tids[mask].tolist()) == good
        if len(np.unique(losses)) == len(losses):   # no ties: == reference
            ot, ov = unpack(d, 'o_tids', i), unpack(d, 'o_vals', i)
            keep = set(tids[mask].tolist())
            below = np.array([v for t, v in zip(ot, ov) if t in keep])
            np.testing.assert_array_equal(below, unpack(d, 'below', i))


def test_parzen_bit_exact(eng):
    d = load('parzen.npz')
    for i in range(ncases(d, 'obs')):
        obs = unpack(d, 'obs', i)
        pw, pm, ps = d['prior'][i]
        w, mu, sg = eng.parzen_fit(obs, pw, pm, ps)
        if len(np.unique(obs)) == len(obs):
            ref = (unpack(d, 'w', i), unpack(d, 'mu', i), unpack(d, 'sigma', i))
        else:   # tied observations: the engine's sort is stable
            ref = O.parzen_fit(obs, pw, pm, ps, kind='stable')
        np.testing.assert_array_equal(mu, ref[1], err_msg='case %d mu' % i)
        np.testing.assert_array_equal(sg, ref[2], err_msg='case %d sigma' % i)
        np.testing.assert_array_equal(w, ref[0], err_msg='case %d w' % i)


def test_categorical_posterior(eng):
    d = load('categorical.npz')
    for i in range(len(d['upper'])):
        obs = unpack(d, 'obs', i)
        pp = unpack(d, 'pprior', i)
        pp = None if np.isnan(pp).all() else pp
        p = eng.categorical_posterior(obs, int(d['upper'][i]), d['pw'][i], pp)
        np.testing.assert_array_equal(p, unpack(d, 'p', i))


def test_score_matches_reference(eng):
    from hyperopt_amd._engine import GMM, LGMM
    d = load('lpdf.npz')
    names = load_json('lpdf_names.json')
    for i, nm in enumerate(names):
        lg, low, high, q = d['meta'][i]
        low, high, q = opt(low), opt(high), opt(q)
        mb = unpack(d, 'mix_b', i).reshape(3, -1)
        ma = unpack(d, 'mix_a', i).reshape(3, -1)
        x = unpack(d, 'cand', i)
        lb, la, bi, bs = eng.score(LGMM if lg else GMM, x, mb, ma, low, high, q)
        rb, ra = unpack(d, 'llik_b', i), unpack(d, 'llik_a', i)
        assert_close(lb, rb, msg=nm + ' below')
        assert_close(la, ra, msg=nm + ' above')
        with np.errstate(all='ignore'):
            assert argmax_equiv(rb - ra, bi), (nm, bi, d['best'][i])


def test_lpdf_closed_form(eng):
    """hyperopt/tests/test_tpe.py:105-190 closed-form GMM1_lpdf values."""
    from hyperopt_amd._engine import GMM
    w, mu, sg = [0.25, 0.25, .5], [0.0, 1.0, 2.0], [1.0, 2.0, 5.0]
    a1 = (.25 / np.sqrt(2 * np.pi * 1.0 ** 2) * np.exp(-.5 * 1.0 ** 2)
          + .25 / np.sqrt(2 * np.pi * 2.0 ** 2)
          + .5 / np.sqrt(2 * np.pi * 5.0 ** 2) * np.exp(-.5 * (1.0 / 5.0) ** 2))
    a0 = (.25 / np.sqrt(2 * np.pi * 1.0 ** 2)
          + .25 / np.sqrt(2 * np.pi * 2.0 ** 2) * np.exp(-.5 * (1.0 / 2.0) ** 2)
          + .5 / np.sqrt(2 * np.pi * 5.0 ** 2) * np.exp(-.5 * (2.0 / 5.0) ** 2))
    v = eng.lpdf(GMM, [[1.0, 0.0, 0.0], [0, 0, 1], [0, 0, 1000]], w, mu, sg)
    assert v.shape == (3, 3)
    assert np.allclose(v[0, 0], np.log(a1)) and np.allclose(v[1, 2], np.log(a1))
    for ij in ((0, 1), (0, 2), (1, 0), (1, 1), (2, 0), (2, 1)):
        assert np.allclose(v[ij], np.log(a0))
    assert np.isfinite(v[2, 2])
    one = eng.lpdf(GMM, [1.0], [1.], [1.0], [2.0])
    assert np.allclose(one, np.log(1.0 / np.sqrt(2 * np.pi * 2.0 ** 2)))


def test_score_errors_map_to_reference_exceptions(eng):
    from hyperopt_amd._engine import GMM, CAT
    mix = ([1.0], [0.0], [1.0])
    with pytest.raises(ValueError):
        eng.score(GMM, [0.0], mix, mix, low=1.0, high=0.0)
    with pytest.raises(IndexError):
        eng.score(CAT, [3.0], [0.5, 0.5], [0.5, 0.5])
    lb, la, bi, bs = eng.score(GMM, [], mix, mix)
    assert bi == -1


# ---- statistical sampler parity (hyperopt/tests/test_tpe.py:193-514) -----
def _hist_check(samples, lpdf_fn, per_bin=500):
    samples = np.sort(samples)
    edges = samples[::per_bin]
    pdf = np.exp(lpdf_fn(edges[:-1]))
    dx = edges[1:] - edges[:-1]
    y = 1 / dx / len(dx)
    err = (pdf - y) ** 2
    assert np.max(err) < .1 and np.mean(err) < .01 and np.median(err) < .01, err


@pytest.mark.parametrize('bounds', [(None, None), (2.5, 3.5)])
def test_gmm_sampler_matches_lpdf(eng, bounds):
    from hyperopt_amd._engine import GMM
    w, mu, sg = [.1, .3, .4, .2], [1.0, 2.0, 3.0, 4.0], [.1, .4, .8, 2.0]
    low, high = bounds
    x = eng.sample(GMM, w, mu, sg, low=low, high=high, seed=234, n=10001)
    if low is not None:
        assert np.all((x >= low) & (x < high))
    _hist_check(x, lambda e: O.gmm_lpdf(e, w, mu, sg, low=low, high=high))


@pytest.mark.parametrize('q,bounds', [(1, (None, None)), (2, (None, None)), (0.5, (None, None)),
                                      (1, (2, 4)), (2, (2, 4)), (1, (1, 4.1))])
def test_qgmm_sampler_matches_lpdf(eng, q, bounds):
    from hyperopt_amd._engine import GMM
    w, mu, sg = [.1, .3, .4, .2], [1.0, 2.0, 3.0, 4.0], [.1, .4, .8, 2.0]
    low, high = bounds
    s = eng.sample(GMM, w, mu, sg, low=low, high=high, q=q, seed=234, n=1001) / q
    assert np.all(s == s.astype(int))
    lo = int(s.min())
    counts = np.bincount(s.astype(int) - lo)
    xc = np.arange(lo, int(s.max()) + 1) * q
    prob = np.exp(O.gmm_lpdf(xc, w, mu, sg, low=low, high=high, q=q))
    err = (prob - counts / 1001.0) ** 2
    assert np.max(err) < .1 and np.mean(err) < .01 and np.median(err) < .01


def _mix_cdf(x, w, mu, sg, low, high, log_space):
    from scipy.stats import norm
    t = np.log(x) if log_space else x
    w, mu, sg = (np.asarray(a, dtype=float) for a in (w, mu, sg))
    F = (w * norm.cdf((t[:, None] - mu) / sg)).sum(1)
    if low is None:
        return F / w.sum()
    lo = (w * norm.cdf((low - mu) / sg)).sum()
    hi = (w * norm.cdf((high - mu) / sg)).sum()
    return (F - lo) / (hi - lo)


@pytest.mark.parametrize('log_space', [False, True])
@pytest.mark.parametrize('bounds', [(None, None), (2, 4), (-1.5, 0.5)])
def test_sampler_ks(eng, log_space, bounds):
    """Kolmogorov-Smirnov test of GMM1/LGMM1 draws against the mixture CDF.
    (The reference's LGMM1 histogram test, test_tpe.py:415-458, passes only
    for its RandomState(234) stream; with the reference's own sampler it
    fails for 35% of seeds, so the Philox stream is checked with KS.)"""
    from scipy.stats import kstest
    from hyperopt_amd._engine import GMM, LGMM
    w, mu, sg = [.1, .3, .4, .2], [-2.0, 1.0, 0.0, 3.0], [.1, .4, .8, 2.0]
    low, high = bounds
    x = eng.sample(LGMM if log_space else GMM, w, mu, sg, low=low, high=high, seed=7, n=20000)
    if low is not None:
        t = np.log(x) if log_space else x
        assert np.all((t >= low) & (t < high))
    res = kstest(x, lambda v: _mix_cdf(np.atleast_1d(v), w, mu, sg, low, high, log_space))
    assert res.pvalue > 1e-3, res


def test_sampler_counter_based_sharding(eng):
    from hyperopt_amd._engine import GMM
    w, mu, sg = [.5, .5], [0.0, 1.0], [1.0, 0.3]
    full = eng.sample(GMM, w, mu, sg, low=-1, high=2, seed=99, stream=3, offset=0, n=1000)
    a = eng.sample(GMM, w, mu, sg, low=-1, high=2, seed=99, stream=3, offset=0, n=377)
    b = eng.sample(GMM, w, mu, sg, low=-1, high=2, seed=99, stream=3, offset=377, n=623)
    np.testing.assert_array_equal(full, np.concatenate([a, b]))


def test_categorical_sampler(eng):
    from hyperopt_amd._engine import CAT
    p = np.array([.1, .2, .3, .4])
    x = eng.sample(CAT, p, seed=5, n=200000)
    freq = np.bincount(x.astype(int), minlength=4) / x.size
    assert np.allclose(freq, p, atol=5e-3)


# ---- fit tiers of tpe_fit.hip: tiny (<= 64, one wave), LDS radix sort
# (<= 10240), global radix sort (> 10240); mixtures in LDS (K <= 4097) or HBM
@pytest.mark.parametrize('n', [2, 63, 64, 65, 1000, 4096, 4097, 10240, 10241, 30000])
@pytest.mark.parametrize('ties', [False, True])
def test_parzen_sort_tiers_bit_exact(eng, n, ties):
    rng = np.random.RandomState(n + ties)
    obs = rng.uniform(-5, 5, n)
    if ties:
        obs = np.round(obs)                          # heavy ties: stable order matters
        obs[::7] = -0.0                              # -0.0 ties +0.0 (numpy order)
    w, mu, sg = eng.parzen_fit(obs, 1.0, 0.25, 10.0)
    ref = O.parzen_fit(obs, 1.0, 0.25, 10.0, kind='stable')
    np.testing.assert_array_equal(mu, ref[1])
    np.testing.assert_array_equal(sg, ref[2])
    np.testing.assert_array_equal(w, ref[0])


@pytest.mark.parametrize('n', [900, 1500, 3000, 4096])
@pytest.mark.parametrize('cluster', [8, 40])
def test_parzen_merge_sort_truncated_key_runs(eng, n, cluster):
    """The merge sorts (<= 1024 and <= 4096 observations) order 32 bits of
    each key: values that differ only below those bits form runs re-ranked by
    their full keys (<= 16), a longer run of distinct full keys falls back to
    the radix sort, a long run of equal keys (quantized ties) stays as is."""
    rng = np.random.RandomState(n + cluster)
    obs = rng.uniform(-5, 5, n)
    base = rng.uniform(-5, 5, 3)
    for j, b in enumerate(base):                      # near-equal clusters, shuffled
        idx = rng.choice(n, cluster, replace=False)
        obs[idx] = b + rng.permutation(cluster) * 1e-13 * (j + 1)
    obs[rng.choice(n, 50, replace=False)] = 2.5       # a long run of equal keys
    w, mu, sg = eng.parzen_fit(obs, 1.0, 0.25, 10.0)
    ref = O.parzen_fit(obs, 1.0, 0.25, 10.0, kind='stable')
    np.testing.assert_array_equal(mu, ref[1])
    np.testing.assert_array_equal(sg, ref[2])
    np.testing.assert_array_equal(w, ref[0])


@pytest.mark.parametrize('n,gamma,cap', [(1000, 0.25, 25), (20000, 0.25, 25), (5000, 2.0, 1000),
                                         (30000, 1.0, 1000), (50, 10.0, 1000)])
def test_split_rounds_and_sort_paths(eng, n, gamma, cap):
    rng = np.random.RandomState(n)
    losses = np.round(rng.rand(n), 3)                # ties
    losses[rng.randint(n, size=5)] = np.inf          # pending trials
    losses[rng.randint(n, size=2)] = np.nan
    mask = eng.split(losses, gamma, gamma_cap=cap)
    good, _ = O.below_tids(np.arange(n), losses, gamma, gamma_cap=cap, kind='stable')
    assert set(np.where(mask)[0].tolist()) == good


@pytest.mark.parametrize('n,upper', [(0, 3), (10, 3), (20000, 7), (5000, 300), (3000, 5000)])
def test_categorical_posterior_sizes(eng, n, upper):
    rng = np.random.RandomState(upper)
    obs = rng.randint(0, min(upper, 40), n)
    p = eng.categorical_posterior(obs, upper, 1.0)
    np.testing.assert_array_equal(p, O.categorical_posterior(obs, upper, 1.0))
    pp = rng.dirichlet(np.ones(upper))
    p = eng.categorical_posterior(obs, upper, 0.5, pp)
    np.testing.assert_array_equal(p, O.categorical_posterior(obs, upper, 0.5, pp))


@pytest.mark.parametrize('q,bounds', [(1, (None, None)), (2, (None, None)), (0.5, (None, None)),
                                      (0.125, (None, None)), (1, (2, 4)), (2, (2, 4)),
                                      (1, (1, 4.1)), (2, (1, 4.1))])
def test_qlgmm_sampler_matches_lpdf(eng, q, bounds):
    """hyperopt/tests/test_tpe.py:424-514 (TestQLGMM1Math) on the device
    sampler: quantized log-GMM draws are multiples of q, inside the
    (log-space) bounds, and their lattice frequencies fit exp(LGMM1_lpdf) --
    chi-square over 20000 draws (lattice points with >= 20 expected hits,
    the rest pooled), plus the reference's own error bounds on the first 20
    lattice points of 1001 draws."""
    from scipy.stats import chisquare
    from hyperopt_amd._engine import LGMM
    w, mu, sg = [.1, .3, .4, .2], [-2.0, 0.0, -3.0, 1.0], [2.1, .4, .8, 2.1]
    low, high = bounds
    for n, seed in ((20000, 11), (1001, 234)):
        s = eng.sample(LGMM, w, mu, sg, low=low, high=high, q=q, seed=seed, n=n) / q
        assert np.all(s == s.astype(int))
        if low is not None:
            assert s.min() * q >= np.round(np.exp(low) / q) * q - 1e-12
            assert s.max() * q <= np.round(np.exp(high) / q) * q + 1e-12
        lo, hi = int(s.min()), int(s.max())
        counts = np.bincount(s.astype(int) - lo)
        xc = np.arange(lo, hi + 1) * q
        with np.errstate(divide='ignore'):
            prob = np.exp(O.lgmm_lpdf(xc, w, mu, sg, low=low, high=high, q=q))
        if n == 1001:
            err = ((prob - counts / float(n)) ** 2)[:20]
            assert np.max(err) < .1 and np.mean(err) < .01 and np.median(err) < .01
            continue
        exp = prob * n
        big = exp >= 20
        obs_b, exp_b = counts[big], exp[big]
        rest_o, rest_e = n - obs_b.sum(), n - exp_b.sum()
        if rest_e >= 20:
            obs_b, exp_b = np.append(obs_b, rest_o), np.append(exp_b, rest_e)
        exp_b = exp_b * obs_b.sum() / exp_b.sum()
        assert chisquare(obs_b, exp_b).pvalue > 1e-4, (q, bounds)


def test_score_argmax_numpy_semantics(eng):
    """broadcast_best's numpy argmax (tpe.py:749-759) through the fused
    operator: the first of tied maxima wins, a NaN score ranks above every
    number (the first NaN wins), across the lanes, waves, tiles and the
    last-tile merge (5000 candidates span several scoring tiles)."""
    from hyperopt_amd._engine import GMM, LGMM
    below = ([0.5, 0.5], [0.5, 2.0], [0.3, 0.4])
    above = ([0.5, 0.5], [-1.0, 4.0], [0.5, 0.6])
    rng = np.random.RandomState(11)
    for fam, lo in ((GMM, -3.0), (LGMM, 0.05)):
        x = rng.uniform(lo, 3.0, 5000) if fam == GMM else np.exp(rng.uniform(-3.0, 1.0, 5000))
        lb, la, bi, bs = eng.score(fam, x, below, above)
        ei = lb - la
        best = int(np.argmax(ei))
        # a copy of the winner later and earlier: the earliest copy wins
        for pos in (best + 3 if best + 3 < x.size else best - 3, 17, 4321):
            y = x.copy()
            y[pos] = x[best]
            _, _, bj, _ = eng.score(fam, y, below, above)
            assert bj == min(pos, best), (fam, pos, best, bj)
        # NaN candidates: the first NaN is numpy's argmax
        y = x.copy()
        y[[2999, 1500, 4100]] = np.nan
        lb2, la2, bj, bs2 = eng.score(fam, y, below, above)
        with np.errstate(invalid='ignore'):
            assert bj == int(np.argmax(lb2 - la2)) == 1500, (fam, bj)
        assert np.isnan(bs2)
