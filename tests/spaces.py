"""Search-space builders shared by the golden generator (run against the
reference's ``hp``) and the tests (run against ``hyperopt_amd.hp``).

Each builder takes the ``hp`` module to use, so the same space is defined in
both frameworks.  Shapes follow SURVEY.md section 8(d) and the reference's own
test domains (hyperopt/tests/test_domains.py:150-165 for ``many_dists``).
"""
import math


def cfg1_space(hp):
    # config 1: 1-D quadratic, hyperopt/tests/test_domains.py:47-54
    return hp.uniform('x', -5, 5)


def cfg2_space(hp, n_each=5):
    # config 2: 20-D mixed (uniform/loguniform/quniform/choice), SURVEY 8(d)
    s = {}
    for i in range(n_each):
        s['u%d' % i] = hp.uniform('u%d' % i, -5, 5)
        s['lu%d' % i] = hp.loguniform('lu%d' % i, math.log(1e-3), math.log(10))
        s['qu%d' % i] = hp.quniform('qu%d' % i, 0, 100, 1)
        s['c%d' % i] = hp.choice('c%d' % i, [0, 1, 2, 3])
    return s


def many_dists_space(hp):
    # all 11 hp kinds, hyperopt/tests/test_domains.py:150-165
    return {
        'a': hp.choice('a', [0, 1, 2]),
        'b': hp.randint('b', 10),
        'c': hp.uniform('c', 4, 7),
        'd': hp.loguniform('d', -2, 0),
        'e': hp.quniform('e', 0, 10, 3),
        'f': hp.qloguniform('f', 0, 3, 2),
        'g': hp.normal('g', 4, 7),
        'h': hp.lognormal('h', -2, 2),
        'i': hp.qnormal('i', 0, 10, 2),
        'j': hp.qlognormal('j', 0, 2, 1),
        'k': hp.pchoice('k', [(.1, 0), (.9, 1)]),
    }


def cond_space(hp, n_branch=3):
    # config-3-like conditional nesting, small
    branches = []
    for b in range(n_branch):
        branches.append({
            'kind': b,
            'lr%d' % b: hp.loguniform('lr%d' % b, math.log(1e-4), 0),
            'units%d' % b: hp.qloguniform('units%d' % b, 0, math.log(1024), 1),
            'act%d' % b: hp.choice('act%d' % b, ['relu', 'tanh', 'sigmoid']),
            'zz%d' % b: hp.normal('zz%d' % b, 0, 1),
        })
    return {'top': hp.choice('top', branches), 'aa': hp.uniform('aa', 0, 1)}


def cfg3_space(hp, n_branch=7):
    # config 3: exactly 50 hps: top + 7 x (3 loguniform + 3 qloguniform + 1 choice)
    branches = []
    for b in range(n_branch):
        d = {'kind': b}
        for j in range(3):
            d['lr%d_%d' % (b, j)] = hp.loguniform('lr%d_%d' % (b, j), math.log(1e-4), 0)
            d['un%d_%d' % (b, j)] = hp.qloguniform('un%d_%d' % (b, j), 0, math.log(1024), 1)
        d['ch%d' % b] = hp.choice('ch%d' % b, [0, 1, 2])
        branches.append(d)
    return hp.choice('top', branches)


def cfg4_space(hp, d=100):
    # config 4: 100 x uniform(-5, 5)
    return [hp.uniform('x%d' % i, -5, 5) for i in range(d)]


# --------------------------------------------------------------------------
# A recording "hp" so a builder can be described without either framework:
# label -> dict(dist, args, conds); used by the oracle-only tests.
# --------------------------------------------------------------------------
class _Node(object):
    def __init__(self, label, dist, args, options=None):
        self.label, self.dist, self.args, self.options = label, dist, args, options


class RecordingHP(object):
    def uniform(self, l, a, b): return _Node(l, 'uniform', (a, b))
    def quniform(self, l, a, b, q): return _Node(l, 'quniform', (a, b, q))
    def loguniform(self, l, a, b): return _Node(l, 'loguniform', (a, b))
    def qloguniform(self, l, a, b, q): return _Node(l, 'qloguniform', (a, b, q))
    def normal(self, l, a, b): return _Node(l, 'normal', (a, b))
    def qnormal(self, l, a, b, q): return _Node(l, 'qnormal', (a, b, q))
    def lognormal(self, l, a, b): return _Node(l, 'lognormal', (a, b))
    def qlognormal(self, l, a, b, q): return _Node(l, 'qlognormal', (a, b, q))
    def randint(self, l, upper): return _Node(l, 'randint', (upper,))
    def choice(self, l, opts): return _Node(l, 'randint', (len(opts),), list(opts))

    def pchoice(self, l, p_opts):
        p = [float(a) for a, _ in p_opts]
        return _Node(l, 'categorical', (p,), [o for _, o in p_opts])


def describe(space):
    hps = {}

    def walk(x, conds):
        if isinstance(x, _Node):
            hps.setdefault(x.label, dict(dist=x.dist, args=x.args, conds=conds))
            for i, o in enumerate(x.options or []):
                walk(o, conds + ((x.label, i),))
        elif isinstance(x, dict):
            for k in sorted(x):
                walk(x[k], conds)
        elif isinstance(x, (list, tuple)):
            for v in x:
                walk(v, conds)
    walk(space, ())
    return hps
