"""The reference's numpy RandomState draw patterns, for exact stream replay.

hyperopt seeds every suggest call with ``np.random.RandomState(seed)`` and
draws hyperparameters one at a time in its interpreter's order
(space.CompiledSpace.draw_order).  Reproducing those calls -- same numpy
functions, same argument shapes, same order -- reproduces the reference's
suggestions bit for bit.  Used by ``rand.suggest`` (startup trials) and by
``tpe.suggest(..., rng_stream='numpy')``; the default TPE path draws its
candidates on the GPU with counter-based Philox instead.
"""
from __future__ import annotations

import numpy as np


def prior_draw(rng, dist, args, n):
    """Prior samplers of hyperopt/pyll/stochastic.py:30-142 (size=(n,))."""
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
        return multinomial_draw(rng, np.asarray(args[0], dtype=np.float64), n)
    raise ValueError('unknown distribution %r' % dist)


def multinomial_draw(rng, p, n):
    """stochastic.categorical, 1-D p (stochastic.py:118-127)."""
    if n == 0:
        return np.zeros(0, dtype=np.int64)
    one_hot = rng.multinomial(n=1, pvals=p, size=int(n))
    return np.dot(one_hot, np.arange(len(p)))


def posterior_draw(rng, family_log, mixture, low, high, q, n):
    """GMM1 / LGMM1 draw pattern (hyperopt/tpe.py:62-93, 216-250)."""
    w, mu, sigma = (np.asarray(a, dtype=np.float64) for a in mixture)
    if n == 0:
        return np.zeros(0)
    if low is None and high is None:
        comp = np.argmax(rng.multinomial(1, w, (n,)), axis=1)
        out = rng.normal(loc=mu[comp], scale=sigma[comp])
        if family_log:
            out = np.exp(out)
    else:
        low, high = float(low), float(high)
        if low >= high:
            raise ValueError('low >= high', (low, high))
        acc = []
        while len(acc) < n:
            k = np.argmax(rng.multinomial(1, w))
            v = rng.normal(loc=mu[k], scale=sigma[k])
            if low <= v < high:
                acc.append(np.exp(v) if family_log else v)
        out = np.asarray(acc)
    out = np.asarray(out, dtype=np.float64).reshape(n)
    if q is not None:
        out = np.round(out / q) * q
    return out
