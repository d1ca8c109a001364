"""hp.* search-space constructors (hyperopt/hp.py, hyperopt/pyll_utils.py:24-116).

Same names, argument order and meaning as the reference.  Each returns an
``expr.HP`` node; ``choice``/``pchoice`` carry their options so conditional
sub-spaces are discovered by ``space.compile_space``.
"""
from .expr import HP


def _label(label):
    if not isinstance(label, str):
        raise TypeError('require string label')
    return label


def choice(label, options):
    options = list(options)
    return HP(_label(label), 'randint', (len(options),), options=options, as_float=False)


def pchoice(label, p_options):
    p, options = zip(*p_options)
    return HP(_label(label), 'categorical', (tuple(float(x) for x in p),),
              options=list(options), as_float=False)


def randint(label, upper):
    return HP(_label(label), 'randint', (int(upper),), as_float=False)


def uniform(label, low, high):
    return HP(_label(label), 'uniform', (float(low), float(high)))


def quniform(label, low, high, q):
    return HP(_label(label), 'quniform', (float(low), float(high), float(q)))


def loguniform(label, low, high):
    return HP(_label(label), 'loguniform', (float(low), float(high)))


def qloguniform(label, low, high, q):
    return HP(_label(label), 'qloguniform', (float(low), float(high), float(q)))


def normal(label, mu, sigma):
    return HP(_label(label), 'normal', (float(mu), float(sigma)))


def qnormal(label, mu, sigma, q):
    return HP(_label(label), 'qnormal', (float(mu), float(sigma), float(q)))


def lognormal(label, mu, sigma):
    return HP(_label(label), 'lognormal', (float(mu), float(sigma)))


def qlognormal(label, mu, sigma, q):
    return HP(_label(label), 'qlognormal', (float(mu), float(sigma), float(q)))
