"""Search-space expressions: a small eager-evaluated replacement for pyll.

The reference builds spaces as pyll graphs (hyperopt/pyll/base.py) and
interprets them with ``rec_eval``.  Here a space is any nesting of dict /
list / tuple containing ``HP`` nodes (hp.* calls) and ``Apply`` nodes
(arithmetic or ``scope.*`` functions on them).  The TPE engine only needs the
hyperparameter descriptors, which ``space.compile_space`` extracts once; the
expression is evaluated per trial by ``evaluate`` (used by Domain.evaluate and
space_eval, hyperopt/fmin.py:324-342).
"""
from __future__ import annotations

import math
import operator

import numpy as np


class Expr(object):
    """Base of lazily evaluated space expressions (supports arithmetic)."""

    def _ap(self, fn, *args):
        return Apply(fn, (self,) + args)

    def __add__(self, o): return Apply(operator.add, (self, o))
    def __radd__(self, o): return Apply(operator.add, (o, self))
    def __sub__(self, o): return Apply(operator.sub, (self, o))
    def __rsub__(self, o): return Apply(operator.sub, (o, self))
    def __mul__(self, o): return Apply(operator.mul, (self, o))
    def __rmul__(self, o): return Apply(operator.mul, (o, self))
    def __truediv__(self, o): return Apply(operator.truediv, (self, o))
    def __rtruediv__(self, o): return Apply(operator.truediv, (o, self))
    def __floordiv__(self, o): return Apply(operator.floordiv, (self, o))
    def __pow__(self, o): return Apply(operator.pow, (self, o))
    def __rpow__(self, o): return Apply(operator.pow, (o, self))
    def __neg__(self): return Apply(operator.neg, (self,))
    def __pos__(self): return self
    def __abs__(self): return Apply(abs, (self,))
    def __getitem__(self, i): return Apply(operator.getitem, (self, i))
    def __lt__(self, o): return Apply(operator.lt, (self, o))
    def __le__(self, o): return Apply(operator.le, (self, o))
    def __gt__(self, o): return Apply(operator.gt, (self, o))
    def __ge__(self, o): return Apply(operator.ge, (self, o))

    def __hash__(self):
        return id(self)


class Apply(Expr):
    """fn(*args) evaluated after its arguments."""

    def __init__(self, fn, args, kwargs=None):
        self.fn = fn
        self.args = tuple(args)
        self.kwargs = dict(kwargs or {})

    def __repr__(self):
        return 'Apply(%s)' % getattr(self.fn, '__name__', self.fn)


class HP(Expr):
    """One hyperparameter: ``hyperopt_param(label, <dist>(*args))``
    (hyperopt/pyll_utils.py:24-116).  ``options`` is set for choice/pchoice,
    whose value selects one option (the pyll ``switch``)."""

    def __init__(self, label, dist, args, options=None, as_float=True):
        if not isinstance(label, str):
            raise TypeError('require string label')
        self.label = label
        self.dist = dist
        self.args = tuple(args)
        self.options = None if options is None else list(options)
        self.as_float = as_float

    def __repr__(self):
        return 'HP(%r, %s%r)' % (self.label, self.dist, self.args)


class Literal(Expr):
    """A constant wrapped as an expression (pyll ``as_apply`` of a value)."""

    def __init__(self, obj):
        self.obj = obj

    def __repr__(self):
        return 'Literal(%r)' % (self.obj,)


def as_apply(obj):
    """Wrap a constant so it can be indexed/combined with hyperparameters."""
    return obj if isinstance(obj, Expr) else Literal(obj)


def _walk_eval(x, assignment, memo):
    if isinstance(x, Literal):
        return x.obj
    if isinstance(x, HP):
        if x.label not in assignment:
            raise KeyError('no value for hyperparameter %r' % x.label)
        v = assignment[x.label]
        if x.options is not None:
            return evaluate(x.options[int(v)], assignment, memo)
        return float(v) if x.as_float else v
    if isinstance(x, Apply):
        key = id(x)
        if key in memo:
            return memo[key]
        args = [evaluate(a, assignment, memo) for a in x.args]
        kw = {k: evaluate(v, assignment, memo) for k, v in x.kwargs.items()}
        r = x.fn(*args, **kw)
        memo[key] = r
        return r
    if isinstance(x, dict):
        return {k: evaluate(v, assignment, memo) for k, v in x.items()}
    if isinstance(x, list):
        return [evaluate(v, assignment, memo) for v in x]
    if isinstance(x, tuple):
        return tuple(evaluate(v, assignment, memo) for v in x)
    return x


def evaluate(x, assignment, memo=None):
    """Value of space ``x`` under ``assignment`` {label: value}."""
    return _walk_eval(x, assignment, {} if memo is None else memo)


class _Scope(object):
    """The handful of pyll ``scope`` functions spaces commonly use."""

    @staticmethod
    def _f(fn, name):
        def g(*args, **kw):
            return Apply(fn, args, kw)
        g.__name__ = name
        return g

    def __init__(self):
        table = {
            'exp': np.exp, 'log': np.log, 'sqrt': np.sqrt, 'sin': np.sin, 'cos': np.cos,
            'tan': np.tan, 'abs': abs, 'float': float, 'int': int, 'min': min, 'max': max,
            'maximum': np.maximum, 'minimum': np.minimum, 'sum': sum, 'len': len,
            'round': round, 'floor': math.floor, 'ceil': math.ceil,
        }
        for k, v in table.items():
            setattr(self, k, self._f(v, k))

    def normal(self, mu, sigma, rng=None):
        """A draw at evaluation time (pyll/stochastic.py:59 with a fixed rng)."""
        return Apply(lambda m, s, r: r.normal(m, s), (mu, sigma, rng))

    def uniform(self, low, high, rng=None):
        return Apply(lambda a, b, r: r.uniform(a, b), (low, high, rng))

    def switch(self, index, *options):
        return Apply(lambda i, *o: o[int(i)], (index,) + options)

    def define(self, fn):
        """Register a user function so ``scope.<name>(...)`` builds an Apply."""
        setattr(self, fn.__name__, self._f(fn, fn.__name__))
        return fn


scope = _Scope()
