"""Compile a search space once into flat per-hyperparameter descriptors.

Replaces, for the TPE hot path, what the reference rebuilds on every suggest:
``Domain``'s vectorized pyll graph (hyperopt/base.py:723-816,
vectorize.py:211-437) and ``tpe_transform``/``build_posterior``
(hyperopt/tpe.py:644-801).  Output:

* ``labels``     -- sorted hyperparameter labels (hp index = position);
* ``hps``        -- per hp: dist, args, condition alternatives;
* ``engine_hps`` -- ``TpeHp`` structs for the C ABI (tpe_engine.h);
* ``draw_order`` -- the order in which the reference's stack interpreter
  draws hyperparameters (reverse-sorted labels, condition parents first),
  needed to replay its RandomState stream exactly.
"""
from __future__ import annotations

import math

import numpy as np

from . import _engine as E
from .expr import HP, Apply

EPS = 1e-12


class DuplicateLabel(Exception):
    """Two different hyperparameters share a label (hyperopt/exceptions.py)."""


class HPDesc(object):
    __slots__ = ('label', 'dist', 'args', 'node', 'paths', 'index')

    def __init__(self, label, dist, args, node):
        self.label, self.dist, self.args, self.node = label, dist, args, node
        self.paths = []     # list of condition tuples ((parent_label, branch), ...)
        self.index = -1

    @property
    def is_categorical(self):
        return self.dist in ('randint', 'categorical')

    @property
    def upper(self):
        return int(self.args[0]) if self.dist == 'randint' else len(self.args[0])

    def conds(self):
        """Immediate (parent, branch) alternatives; () = unconditional."""
        if any(len(p) == 0 for p in self.paths):
            return ()
        alts = []
        for p in self.paths:
            c = p[-1]
            if c not in alts:
                alts.append(c)
        return tuple(alts)

    def parents(self):
        ps = []
        for p in self.paths:
            for lab, _ in p:
                if lab not in ps:
                    ps.append(lab)
        return ps

    def __repr__(self):
        return 'HPDesc(%r, %s%r)' % (self.label, self.dist, self.args)


class CompiledSpace(object):
    def __init__(self, expr):
        self.expr = expr
        found = {}
        self._walk(expr, (), found)
        self.labels = sorted(found)
        self.hps = [found[l] for l in self.labels]
        for i, h in enumerate(self.hps):
            h.index = i
        self.by_label = {h.label: h for h in self.hps}
        # (label, engine index, categorical?) of every hp: tpe.suggest's
        # record -> value conversion
        self.pick_order = [(h.label, h.index, h.is_categorical) for h in self.hps]
        self.draw_order = self._draw_order()
        self._engine_tables = None

    # -- discovery (hyperopt/pyll_utils.py:144-195 expr_to_config) ---------
    def _walk(self, x, conds, found, seen=None):
        if seen is None:
            seen = set()
        if isinstance(x, HP):
            h = found.get(x.label)
            if h is None:
                h = found[x.label] = HPDesc(x.label, x.dist, x.args, x)
            elif h.node is not x:
                raise DuplicateLabel(x.label)
            if conds not in h.paths:
                h.paths.append(conds)
            key = (id(x), conds)
            if key in seen:
                return
            seen.add(key)
            for i, o in enumerate(x.options or []):
                self._walk(o, conds + ((x.label, i),), found, seen)
        elif isinstance(x, Apply):
            for a in x.args:
                self._walk(a, conds, found, seen)
            for a in x.kwargs.values():
                self._walk(a, conds, found, seen)
        elif isinstance(x, dict):
            for k in sorted(x, key=str):
                self._walk(x[k], conds, found, seen)
        elif isinstance(x, (list, tuple)):
            for v in x:
                self._walk(v, conds, found, seen)

    def _draw_order(self):
        done, order = set(), []

        def visit(lab):
            if lab in done:
                return
            done.add(lab)
            for p in self.by_label[lab].parents():
                visit(p)
            order.append(lab)

        for lab in sorted(self.labels, reverse=True):
            visit(lab)
        return order

    def is_active(self, label, chosen):
        """Whether ``label`` participates given the values chosen so far."""
        h = self.by_label[label]
        if not h.paths or any(len(p) == 0 for p in h.paths):
            return True
        for p in h.paths:
            if all(chosen.get(lab) is not None and int(chosen[lab]) == b for lab, b in p):
                return True
        return False

    # -- engine descriptors (hyperopt/tpe.py:485-607) ------------------------
    def engine_tables(self):
        if self._engine_tables is None:
            self._engine_tables = _engine_tables(self)
        return self._engine_tables


def _engine_tables(cs):
    hps, conds, pprior = [], [], []
    for h in cs.hps:
        t = E.TpeHp()
        a = h.args
        d = h.dist
        t.obs_transform = E.OBS_IDENT
        if d in ('uniform', 'quniform', 'loguniform', 'qloguniform'):
            low, high = float(a[0]), float(a[1])
            t.family = E.LGMM if 'log' in d else E.GMM
            t.prior_mu = 0.5 * (high + low)
            t.prior_sigma = 1.0 * (high - low)
            t.low, t.high = low, high
            t.flags = E.HAS_LOW | E.HAS_HIGH
            if d.startswith('q'):
                t.flags |= E.HAS_Q
                t.q = float(a[2])
            if d == 'loguniform':
                t.obs_transform = E.OBS_LOG
            elif d == 'qloguniform':
                t.obs_transform = E.OBS_LOG_CLIP_EXPLOW
        elif d in ('normal', 'qnormal', 'lognormal', 'qlognormal'):
            t.family = E.LGMM if 'log' in d else E.GMM
            t.prior_mu, t.prior_sigma = float(a[0]), float(a[1])
            t.flags = 0
            if d.startswith('q'):
                t.flags |= E.HAS_Q
                t.q = float(a[2])
            if d == 'lognormal':
                t.obs_transform = E.OBS_LOG
            elif d == 'qlognormal':
                t.obs_transform = E.OBS_LOG_CLIP_EPS
        elif d == 'randint':
            t.family = E.CAT
            t.upper = int(a[0])
            t.flags = 0
        elif d == 'categorical':
            t.family = E.CAT
            t.upper = len(a[0])
            t.flags = E.PCHOICE
            t.pprior_begin = len(pprior)
            pprior.extend(float(v) for v in a[0])
        else:
            raise ValueError('unsupported distribution %r' % d)
        c = h.conds()
        t.cond_begin = len(conds)
        t.cond_count = len(c)
        for lab, b in c:
            conds.append((cs.by_label[lab].index, int(b)))
        hps.append(t)
    return hps, conds, np.asarray(pprior, dtype=np.float64)


def compile_space(expr):
    return CompiledSpace(expr)
