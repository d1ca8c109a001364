"""hyperopt.base namespace: trial store, domain, status constants and the
misc (idxs / vals) codec of trial documents.

The store (``trials.py``) is columnar with a change journal; the Domain
compiles its space once (``domain.py``).  The functions here convert between
a list of trial miscs and the per-label columns {label: [tid...]} /
{label: [value...]} the reference's algorithms exchange
(hyperopt/base.py:156-214).
"""
from __future__ import annotations

from .status import *  # noqa: F401,F403
from .status import STATUS_STRINGS, JOB_STATES  # noqa: F401
from .trials import (Trials, TrialDoc, trials_from_docs, InvalidTrial, SONify,  # noqa: F401
                     coarse_utcnow, pmin_sampled)
from .domain import Domain, Ctrl, InvalidResultStatus, InvalidLoss  # noqa: F401
from .space import compile_space, DuplicateLabel  # noqa: F401


def miscs_update_idxs_vals(miscs, idxs, vals, assert_all_vals_used=True, idxs_map=None):
    """Write per-label columns into the miscs they address.

    ``idxs[label]`` lists tids and ``vals[label]`` the matching values; each
    misc first gets empty idxs/vals for every label, then every (tid, value)
    pair -- tids renamed through ``idxs_map`` -- lands as ``[tid]`` /
    ``[value]`` in that tid's misc.  Pairs for tids without a misc raise
    KeyError unless ``assert_all_vals_used`` is False, then they are dropped
    (tpe.suggest keeps only its first fake id this way, tpe.py:891-893).
    """
    if set(idxs) != set(vals):
        raise AssertionError('idxs and vals name different labels')
    rename = idxs_map or {}
    labels = list(idxs)
    by_tid = {}
    for m in miscs:
        by_tid[m['tid']] = m
        m['idxs'] = {lab: [] for lab in labels}
        m['vals'] = {lab: [] for lab in labels}
    for lab in labels:
        col_t, col_v = idxs[lab], vals[lab]
        if len(col_t) != len(col_v):
            raise AssertionError('label %r: %d tids, %d values' % (lab, len(col_t), len(col_v)))
        for t, v in zip(col_t, col_v):
            t = rename.get(t, t)
            m = by_tid.get(t)
            if m is None:
                if assert_all_vals_used:
                    raise KeyError(t)
                continue
            m['idxs'][lab] = [t]
            m['vals'][lab] = [v]
    return miscs


def miscs_to_idxs_vals(miscs, keys=None):
    """The inverse: per-label columns of tids and values over ``miscs``, in
    misc order.  ``keys`` defaults to the first misc's labels."""
    if keys is None:
        if not miscs:
            raise ValueError('cannot infer keys from empty miscs')
        keys = list(miscs[0]['idxs'])
    for m in miscs:
        for k in keys:
            ti, tv = m['idxs'][k], m['vals'][k]
            if len(ti) != len(tv) or (ti and ti != [m['tid']]):
                raise AssertionError('misc %r: inconsistent idxs/vals for %r' % (m['tid'], k))
    idxs = {k: [t for m in miscs for t in m['idxs'][k]] for k in keys}
    vals = {k: [v for m in miscs for v in m['vals'][k]] for k in keys}
    return idxs, vals


def spec_from_misc(misc):
    """{label: value} of a trial's active hyperparameters."""
    spec = {}
    for k, v in misc['vals'].items():
        if len(v) > 1:
            raise NotImplementedError('multiple values', (k, v))
        if v:
            spec[k] = v[0]
    return spec
