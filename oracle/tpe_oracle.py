"""CPU oracle for the TPE suggestion hot path -- TEST INFRASTRUCTURE ONLY.

This module is a from-scratch numpy/scipy float64 restatement of the
reference's (pminervini/hyperopt v0.0.3.dev) TPE numerics.  It exists to
*check* the HIP engine, never to be the engine: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product path (``hyperopt_amd``) must never import it.

Parity pinning: every function below is checked bit-for-bit (or, where noted,
to float64 round-off) against golden vectors produced by running the reference
itself (converted to Python 3 in /tmp, see ``oracle/setup_reference.sh`` and
``tests/golden/make_golden.py``).  Those fixtures live in ``tests/golden/`` and
are exercised by ``tests/test_oracle_golden.py``.

Citations are ``hyperopt/<file>:<line>`` in the reference tree.
"""
from __future__ import annotations


import numpy as np
from scipy.special import erf

EPS = 1e-12          # hyperopt/tpe.py:25
DEFAULT_LF = 25      # hyperopt/tpe.py:29


# --------------------------------------------------------------------------
# (a2) good/bad split -- hyperopt/tpe.py:613-641 (ap_filter_trials)
# --------------------------------------------------------------------------
def n_below_count(n_trials: int, gamma: float, gamma_cap: int = DEFAULT_LF) -> int:
    """Size of the 'good' set: min(ceil(gamma*sqrt(N)), cap), tpe.py:625."""
    return min(int(np.ceil(gamma * np.sqrt(n_trials))), gamma_cap)


def below_tids(loss_tids, losses, gamma, gamma_cap=DEFAULT_LF, kind=None):
    """Return (below_tid_set, above_tid_set) of the global loss ranking.

    The reference sorts with numpy's default (unstable) argsort, tpe.py:626;
    ``kind='stable'`` gives the tie-break the HIP engine uses (lowest
    position first)."""
    loss_tids = np.asarray(loss_tids)
    losses = np.asarray(losses, dtype=np.float64)
    nb = n_below_count(len(losses), gamma, gamma_cap)
    order = np.argsort(losses, kind=kind) if kind else np.argsort(losses)
    return set(loss_tids[order[:nb]].tolist()), set(loss_tids[order[nb:]].tolist())


def split_observations(o_tids, o_vals, loss_tids, losses, gamma,
                       gamma_cap=DEFAULT_LF, kind=None):
    """ap_filter_trials: observations of one hp split into (below, above),
    each kept in observation (tid) order, tpe.py:629-636."""
    good, bad = below_tids(loss_tids, losses, gamma, gamma_cap, kind)
    o_vals = list(o_vals)
    below = np.asarray([v for t, v in zip(o_tids, o_vals) if t in good])
    above = np.asarray([v for t, v in zip(o_tids, o_vals) if t in bad])
    return below, above


# --------------------------------------------------------------------------
# (a3) linear forgetting -- hyperopt/tpe.py:381-394
# --------------------------------------------------------------------------
def lf_weights(n: int, lf: int = DEFAULT_LF) -> np.ndarray:
    if n == 0:
        return np.zeros(0)
    if n < lf:
        return np.ones(n)
    ramp = np.linspace(1.0 / n, 1.0, num=n - lf)
    return np.concatenate([ramp, np.ones(lf)])


# --------------------------------------------------------------------------
# (a4) adaptive Parzen estimator -- hyperopt/tpe.py:398-475
# --------------------------------------------------------------------------
def parzen_fit(obs, prior_weight, prior_mu, prior_sigma, lf=DEFAULT_LF,
               kind=None, return_order=False):
    """Fit the 1-D Gaussian mixture (weights, mus, sigmas) of one side.

    ``kind`` selects the argsort used for ordering the observations
    (tpe.py:427 uses numpy's default; the engine is stable)."""
    obs = np.asarray(obs, dtype=np.float64).ravel()
    n = obs.size
    order = None
    if n == 0:                                   # tpe.py:410-413
        mus = np.array([prior_mu], dtype=np.float64)
        sig = np.array([prior_sigma], dtype=np.float64)
        pos = 0
    elif n == 1:                                 # tpe.py:414-422
        if prior_mu < obs[0]:
            pos = 0
            mus = np.array([prior_mu, obs[0]])
            sig = np.array([prior_sigma, prior_sigma * .5])
        else:
            pos = 1
            mus = np.array([obs[0], prior_mu])
            sig = np.array([prior_sigma * .5, prior_sigma])
    else:                                        # tpe.py:423-442
        order = np.argsort(obs, kind=kind) if kind else np.argsort(obs)
        sorted_obs = obs[order]
        pos = int(np.searchsorted(sorted_obs, prior_mu))   # side='left'
        mus = np.insert(sorted_obs, pos, prior_mu)
        gaps = np.diff(mus)
        sig = np.empty_like(mus)
        sig[1:-1] = np.maximum(gaps[:-1], gaps[1:])
        sig[0] = gaps[0]
        sig[-1] = gaps[-1]

    if lf and lf < n:                            # tpe.py:444-450
        base = lf_weights(n, lf)
        w = np.insert(base[order], pos, prior_weight)
    else:                                        # tpe.py:452-454
        w = np.ones(mus.size)
        w[pos] = prior_weight

    hi = prior_sigma / 1.0                       # tpe.py:457-462
    lo = prior_sigma / min(100.0, (1.0 + mus.size))
    sig = np.clip(sig, lo, hi)
    sig[pos] = prior_sigma
    w = w / w.sum()
    if return_order:
        return w, mus, sig, order, pos
    return w, mus, sig


# --------------------------------------------------------------------------
# (a9) cdf / lpdf helpers -- hyperopt/tpe.py:96-101, 171-202, 253-256
# --------------------------------------------------------------------------
def normal_cdf(x, mu, sigma):
    z = (x - mu) / np.maximum(np.sqrt(2) * sigma, EPS)
    return 0.5 * (1 + erf(z))


def lognormal_cdf(x, mu, sigma):
    x = np.asarray(x)
    if x.size == 0:
        return np.asarray([])
    if x.min() < 0:
        raise ValueError('negative arg to lognormal_cdf', x)
    with np.errstate(divide='ignore'):
        z = (np.log(np.maximum(x, EPS)) - mu) / np.maximum(np.sqrt(2) * sigma, EPS)
    return .5 + .5 * erf(z)


def lognormal_lpdf(x, mu, sigma):
    sigma = np.maximum(sigma, EPS)
    norm = sigma * x * np.sqrt(2 * np.pi)
    quad = 0.5 * ((np.log(x) - mu) / sigma) ** 2
    return -quad - np.log(norm)


def lse_rows(a):
    m = a.max(axis=1)
    return np.log(np.exp(a - m[:, None]).sum(axis=1)) + m


def _truncation_mass(w, mu, sigma, low, high):
    """p_accept of a (possibly) truncated mixture, tpe.py:130-136/273-276."""
    if low is None and high is None:
        return 1
    return np.sum(w * (normal_cdf(high, mu, sigma) - normal_cdf(low, mu, sigma)))


# --------------------------------------------------------------------------
# (a10) GMM1_lpdf -- hyperopt/tpe.py:104-166
# --------------------------------------------------------------------------
def gmm_lpdf(x, w, mu, sigma, low=None, high=None, q=None):
    x = np.asarray(x, dtype=np.float64)
    w, mu, sigma = (np.asarray(a, dtype=np.float64) for a in (w, mu, sigma))
    if x.size == 0:
        return np.asarray([])
    for a, nm in ((w, 'weights'), (mu, 'mus'), (sigma, 'sigmas')):
        if a.ndim != 1:
            raise TypeError('need vector of %s' % nm, a.shape)
    shape = x.shape
    xs = x.ravel()
    pacc = _truncation_mass(w, mu, sigma, low, high)
    if q is None:
        mahal = ((xs[:, None] - mu) / np.maximum(sigma, EPS)) ** 2
        coef = w / np.sqrt(2 * np.pi * sigma ** 2) / pacc
        out = lse_rows(-0.5 * mahal + np.log(coef))
    else:
        ub = xs + q / 2.0 if high is None else np.minimum(xs + q / 2.0, high)
        lb = xs - q / 2.0 if low is None else np.maximum(xs - q / 2.0, low)
        prob = np.zeros(xs.shape)
        for wk, mk, sk in zip(w, mu, sigma):
            inc = wk * normal_cdf(ub, mk, sk)
            inc -= wk * normal_cdf(lb, mk, sk)
            prob += inc
        out = np.log(prob) - np.log(pacc)
    return out.reshape(shape)


# --------------------------------------------------------------------------
# (a11) LGMM1_lpdf -- hyperopt/tpe.py:259-301
# --------------------------------------------------------------------------
def lgmm_lpdf(x, w, mu, sigma, low=None, high=None, q=None):
    x = np.asarray(x, dtype=np.float64)
    w, mu, sigma = (np.asarray(a, dtype=np.float64) for a in (w, mu, sigma))
    shape = x.shape
    xs = x.ravel()
    pacc = _truncation_mass(w, mu, sigma, low, high)
    if q is None:
        # NB: p_accept is computed but not applied on this branch (tpe.py:278)
        out = lse_rows(lognormal_lpdf(xs[:, None], mu, sigma) + np.log(w))
    else:
        ub = xs + q / 2.0 if high is None else np.minimum(xs + q / 2.0, np.exp(high))
        lb = xs - q / 2.0 if low is None else np.maximum(xs - q / 2.0, np.exp(low))
        lb = np.maximum(0, lb)
        prob = np.zeros(xs.shape)
        for wk, mk, sk in zip(w, mu, sigma):
            inc = wk * lognormal_cdf(ub, mk, sk)
            inc -= wk * lognormal_cdf(lb, mk, sk)
            prob += inc
        out = np.log(prob) - np.log(pacc)
    return out.reshape(shape)


# --------------------------------------------------------------------------
# (a8)/(a12) categorical posterior + lpdf -- tpe.py:50-57, 573-607
# --------------------------------------------------------------------------
def categorical_posterior(obs, upper, prior_weight, p_prior=None, lf=DEFAULT_LF):
    """Posterior probabilities of a randint/choice (p_prior None, tpe.py:573)
    or pchoice (p_prior given, tpe.py:590-607) hyperparameter."""
    obs = np.asarray(obs).astype(np.int64).ravel()
    counts = np.bincount(obs, minlength=upper, weights=lf_weights(obs.size, lf))
    if p_prior is None:
        pseudo = counts + prior_weight
    else:
        pseudo = counts + upper * (prior_weight * np.asarray(p_prior, dtype=np.float64))
    return pseudo / np.sum(pseudo)


def categorical_lpdf(sample, p):
    sample = np.asarray(sample)
    if sample.size == 0:
        return np.asarray([])
    return np.log(np.asarray(p)[sample.astype(np.int64)])


# --------------------------------------------------------------------------
# (a13) EI argmax -- tpe.py:749-759
# --------------------------------------------------------------------------
def best_index(below_llik, above_llik):
    """np.argmax of below-above: first max, first NaN wins."""
    score = np.asarray(below_llik) - np.asarray(above_llik)
    return int(np.argmax(score)), score


# --------------------------------------------------------------------------
# reference RNG streams (numpy RandomState legacy) -- tpe.py:62-93, 216-250,
# pyll/stochastic.py:30-142.  Used to replay the reference's draws exactly.
# --------------------------------------------------------------------------
def gmm_sample(rng, w, mu, sigma, low=None, high=None, q=None, n=1, log_space=False):
    w, mu, sigma = (np.asarray(a, dtype=np.float64) for a in (w, mu, sigma))
    if low is None and high is None:
        comp = np.argmax(rng.multinomial(1, w, (n,)), axis=1)
        draws = rng.normal(loc=mu[comp], scale=sigma[comp])
        out = np.exp(draws) if log_space else draws
    else:
        low, high = float(low), float(high)
        if low >= high:
            raise ValueError('low >= high', (low, high))
        acc = []
        while len(acc) < n:
            k = np.argmax(rng.multinomial(1, w))
            d = rng.normal(loc=mu[k], scale=sigma[k])
            if low <= d < high:
                acc.append(np.exp(d) if log_space else d)
        out = np.asarray(acc, dtype=np.float64).reshape(n)
    out = np.asarray(out, dtype=np.float64).reshape(n)
    if q is not None:
        out = np.round(out / q) * q
    return out


def categorical_sample(rng, p, n):
    """stochastic.categorical with 1-D p, size=(n,) (stochastic.py:104-134)."""
    if n == 0:
        return np.asarray([])
    p = np.asarray(p)
    draws = rng.multinomial(n=1, pvals=p, size=int(n))
    return np.dot(draws, np.arange(len(p)))


def prior_sample(rng, dist, args, n=1):
    """Prior draws of pyll/stochastic.py:30-100 (used by rand.suggest)."""
    if dist == 'uniform':
        return rng.uniform(args[0], args[1], size=n)
    if dist == 'loguniform':
        return np.exp(rng.uniform(args[0], args[1], size=n))
    if dist == 'quniform':
        return np.round(rng.uniform(args[0], args[1], size=n) / args[2]) * args[2]
    if dist == 'qloguniform':
        return np.round(np.exp(rng.uniform(args[0], args[1], size=n)) / args[2]) * args[2]
    if dist == 'normal':
        return rng.normal(args[0], args[1], size=n)
    if dist == 'qnormal':
        return np.round(rng.normal(args[0], args[1], size=n) / args[2]) * args[2]
    if dist == 'lognormal':
        return np.exp(rng.normal(args[0], args[1], size=n))
    if dist == 'qlognormal':
        return np.round(np.exp(rng.normal(args[0], args[1], size=n)) / args[2]) * args[2]
    if dist == 'randint':
        return rng.randint(args[0], size=n)
    if dist == 'categorical':
        return categorical_sample(rng, args[0], n)
    raise ValueError(dist)


# --------------------------------------------------------------------------
# per-hp posterior: observation transform + fit + scorer, tpe.py:485-607
# --------------------------------------------------------------------------
def posterior_spec(dist, args, prior_weight):
    """Return (fit_kind, prior_mu, prior_sigma, lpdf_kind, low, high, q,
    obs_transform) for a prior ``dist(*args)`` (tpe.py:485-568)."""
    if dist in ('uniform', 'quniform', 'loguniform', 'qloguniform'):
        low, high = float(args[0]), float(args[1])
        pm, ps = 0.5 * (high + low), 1.0 * (high - low)
        q = float(args[2]) if dist.startswith('q') else None
        lg = 'log' in dist
        if dist == 'loguniform':
            tr = 'log'
        elif dist == 'qloguniform':
            tr = 'log_clip_explow'
        else:
            tr = None
        return ('lgmm' if lg else 'gmm'), pm, ps, low, high, q, tr
    if dist in ('normal', 'qnormal', 'lognormal', 'qlognormal'):
        pm, ps = float(args[0]), float(args[1])
        q = float(args[2]) if dist.startswith('q') else None
        lg = 'log' in dist
        tr = {'lognormal': 'log', 'qlognormal': 'log_clip_eps'}.get(dist)
        return ('lgmm' if lg else 'gmm'), pm, ps, None, None, q, tr
    raise ValueError(dist)


def transform_obs(obs, tr, low=None):
    obs = np.asarray(obs, dtype=np.float64)
    if tr is None:
        return obs
    if tr == 'log':
        return np.log(obs)
    if tr == 'log_clip_explow':                 # tpe.py:522-533
        return np.log(np.maximum(obs, np.maximum(EPS, np.exp(low))))
    if tr == 'log_clip_eps':                    # tpe.py:564
        return np.log(np.maximum(obs, EPS))
    raise ValueError(tr)


def score_hp(dist, args, below_obs, above_obs, prior_weight, candidates,
             kind=None):
    """Fit both sides for one hp and score ``candidates``.

    Returns dict(below=(w,mu,sigma)|p, above=..., llik_b, llik_a, best)."""
    if dist in ('randint', 'categorical'):
        if dist == 'randint':
            upper, pp = int(args[0]), None
        else:
            pp = np.asarray(args[0], dtype=np.float64)
            upper = len(pp)
        pb = categorical_posterior(below_obs, upper, prior_weight, pp)
        pa = categorical_posterior(above_obs, upper, prior_weight, pp)
        lb = categorical_lpdf(candidates, pb)
        la = categorical_lpdf(candidates, pa)
        best = best_index(lb, la)[0] if len(candidates) else None
        return dict(below=pb, above=pa, llik_b=lb, llik_a=la, best=best)
    fk, pm, ps, low, high, q, tr = posterior_spec(dist, args, prior_weight)
    bo = transform_obs(below_obs, tr, low)
    ao = transform_obs(above_obs, tr, low)
    mb = parzen_fit(bo, prior_weight, pm, ps, kind=kind)
    ma = parzen_fit(ao, prior_weight, pm, ps, kind=kind)
    f = lgmm_lpdf if fk == 'lgmm' else gmm_lpdf
    lb = f(candidates, *mb, low=low, high=high, q=q)
    la = f(candidates, *ma, low=low, high=high, q=q)
    best = best_index(lb, la)[0] if len(candidates) else None
    return dict(below=mb, above=ma, llik_b=lb, llik_a=la, best=best)


def sample_hp(rng, dist, args, below_mix, n):
    """Reference-stream candidate draw from the below posterior of one hp."""
    if dist in ('randint', 'categorical'):
        return categorical_sample(rng, below_mix, n)
    fk, pm, ps, low, high, q, tr = posterior_spec(dist, args, 1.0)
    return gmm_sample(rng, *below_mix, low=low, high=high, q=q, n=n,
                      log_space=(fk == 'lgmm'))


def lpdf_pairs(dist, args, kb, ka, n_cand):
    """Algorithmic work count: (candidate, component) pairs of one hp."""
    if dist in ('randint', 'categorical'):
        return 0
    return n_cand * (kb + ka)




# --------------------------------------------------------------------------
# whole-suggest restatement, reference RNG stream -- tpe.py:804-897
# --------------------------------------------------------------------------
def hp_order(hps):
    """Order in which the reference's pyll interpreter draws hyperparameters.

    ``hps`` maps label -> dict(dist, args, conds) with ``conds`` a tuple of
    (parent_label, branch) pairs.  The stack interpreter (pyll/base.py:852-899)
    visits the sorted label dict last-first, evaluating a hp's condition
    parents before it (observed on the reference, pinned by the suggest
    fixtures)."""
    done, order = set(), []

    def visit(lab):
        if lab in done:
            return
        for path in _paths(hps[lab]):
            for parent, _ in path:
                visit(parent)
        done.add(lab)
        order.append(lab)

    for lab in sorted(hps, reverse=True):
        visit(lab)
    return order


def _paths(h):
    """Alternative condition paths of a hp: ``paths`` (list of tuples of
    (parent, branch)) or the single path ``conds``."""
    if 'paths' in h:
        return h['paths']
    return [h['conds']]


def is_active(h, chosen):
    for path in _paths(h):
        if all(chosen.get(p) is not None and int(chosen[p]) == b for p, b in path):
            return True
    return False


def suggest_reference_stream(hps, loss_tids, losses, obs, seed, n_ei=24,
                             prior_weight=1.0, gamma=0.25, kind=None):
    """Replay one tpe.suggest on an already-assembled history.

    obs: label -> (o_tids, o_vals) in tid order.  Returns (chosen, detail)
    where chosen maps each active label to its value."""
    rng = np.random.RandomState(seed)
    chosen, detail = {}, {}
    for lab in hp_order(hps):
        h = hps[lab]
        active = is_active(h, chosen)
        n = n_ei if active else 0
        o_tids, o_vals = obs[lab]
        bo, ao = split_observations(o_tids, o_vals, loss_tids, losses, gamma, kind=kind)
        if h['dist'] in ('randint', 'categorical'):
            if h['dist'] == 'randint':
                upper, pp = int(h['args'][0]), None
            else:
                pp = np.asarray(h['args'][0], dtype=np.float64)
                upper = len(pp)
            pb = categorical_posterior(bo, upper, prior_weight, pp)
            mix_b = pb
        else:
            fk, pm, ps, low, high, q, tr = posterior_spec(h['dist'], h['args'], prior_weight)
            mix_b = parzen_fit(transform_obs(bo, tr, low), prior_weight, pm, ps, kind=kind)
        cand = sample_hp(rng, h['dist'], h['args'], mix_b, n) if n else np.zeros(0)
        res = score_hp(h['dist'], h['args'], bo, ao, prior_weight, cand, kind=kind)
        detail[lab] = dict(cand=cand, **res)
        if n:
            chosen[lab] = cand[res['best']]
    return chosen, detail
