"""The reference's test domains (hyperopt/tests/test_domains.py:38-217)
written with hyperopt_amd's hp/scope, as (name, space, settings) for fmin with
a passthrough objective.  Also imported by tests/golden/make_golden.py with
the reference's hp/scope to record the reference trajectories."""
import numpy as np


def build(name, hp, scope, as_apply):
    if name == 'quadratic1':
        return {'loss': (hp.uniform('x', -5, 5) - 3) ** 2, 'status': 'ok'}
    if name == 'q1_lognormal':
        return {'loss': scope.min(0.1 * (hp.lognormal('x', 0, 2) - 10) ** 2, 10),
                'status': 'ok'}
    if name == 'n_arms':
        rng = np.random.RandomState(123)
        x = hp.choice('x', [0, 1])
        mus = as_apply([-1, 0])
        sig = as_apply([1, 1])
        return {'loss': scope.normal(mus[x], sig[x], rng=rng), 'loss_variance': 1.0,
                'status': 'ok'}
    if name == 'distractor':
        x = hp.uniform('x', -15, 15)
        f1 = 1.0 / (1.0 + scope.exp(-x))
        f2 = 2 * scope.exp(-(x + 10) ** 2)
        return {'loss': -f1 - f2, 'status': 'ok'}
    if name == 'gauss_wave':
        x = hp.uniform('x', -20, 20)
        t = hp.choice('curve', [x, x + np.pi])
        f1 = scope.sin(t)
        f2 = 2 * scope.exp(-(t / 5.0) ** 2)
        return {'loss': - (f1 + f2), 'status': 'ok'}
    if name == 'gauss_wave2':
        rng = np.random.RandomState(123)
        var = .1
        x = hp.uniform('x', -20, 20)
        amp = hp.uniform('amp', 0, 1)
        t = (scope.normal(0, var, rng=rng) + 2 * scope.exp(-(x / 5.0) ** 2))
        return {'loss': - hp.choice('hf', [t, t + scope.sin(x) * amp]),
                'loss_variance': var, 'status': 'ok'}
    if name == 'many_dists':
        a = hp.choice('a', [0, 1, 2])
        b = hp.randint('b', 10)
        c = hp.uniform('c', 4, 7)
        d = hp.loguniform('d', -2, 0)
        e = hp.quniform('e', 0, 10, 3)
        f = hp.qloguniform('f', 0, 3, 2)
        g = hp.normal('g', 4, 7)
        h = hp.lognormal('h', -2, 2)
        i = hp.qnormal('i', 0, 10, 2)
        j = hp.qlognormal('j', 0, 2, 1)
        k = hp.pchoice('k', [(.1, 0), (.9, 1)])
        z = a + b + c + d + e + f + g + h + i + j + k
        return {'loss': scope.float(scope.log(1e-12 + z ** 2)), 'status': 'ok'}
    if name == 'branin':
        x = hp.uniform('x', -5., 10.)
        y = hp.uniform('y', 0., 15.)
        pi = float(np.pi)
        loss = ((y - (5.1 / (4 * pi ** 2)) * x ** 2 + 5 * x / pi - 6) ** 2
                + 10 * (1 - 1 / (8 * pi)) * scope.cos(x) + 10)
        return {'loss': loss, 'loss_variance': 0, 'status': 'ok'}
    raise KeyError(name)


# TestOpt settings, hyperopt/tests/test_tpe.py:529-570
THRESH = dict(quadratic1=1e-5, q1_lognormal=0.01, distractor=-1.96, gauss_wave=-2.0,
              gauss_wave2=-2.0, n_arms=-2.5, many_dists=.0005, branin=0.7)
LEN = dict(quadratic1=1000, many_dists=200, distractor=100, q1_lognormal=250,
           gauss_wave2=75, branin=200)
GAMMA = dict(distractor=.05)
PRIOR_WEIGHT = dict(distractor=.01)
N_EI = dict(quadratic1=5, distractor=15)
NAMES = sorted(THRESH)


def settings(name):
    return dict(gamma=GAMMA.get(name, 0.25), prior_weight=PRIOR_WEIGHT.get(name, 1.0),
                n_EI_candidates=N_EI.get(name, 24)), LEN.get(name, 50)
