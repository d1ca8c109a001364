"""Random search / TPE startup (hyperopt/rand.py).

``rng_stream='numpy'`` (default): host-side prior sampling with the
reference's RandomState stream, so random search and the first
``n_startup_jobs`` trials of a TPE run are identical to the reference's.
``rng_stream='philox'``: the same priors drawn on the device
(``tpe_plan_sample_prior``), all ids of the call in one launch.
"""
from __future__ import annotations

import numpy as np

from . import rstream
from .base import miscs_update_idxs_vals


def _value(h, v):
    return int(v) if h.is_categorical else v


def suggest(new_ids, domain, trials, seed, rng_stream='numpy'):
    """hyperopt/rand.py:14-33: one pass over the space per new id."""
    if rng_stream == 'philox':
        return _suggest_device(new_ids, domain, trials, seed)
    if rng_stream != 'numpy':
        raise ValueError('rng_stream must be "numpy" or "philox"')
    cs = domain.space
    rng = np.random.RandomState(seed)
    rval = []
    for new_id in new_ids:
        chosen = {}
        idxs, vals = {lab: [] for lab in cs.labels}, {lab: [] for lab in cs.labels}
        for lab in cs.draw_order:
            if not cs.is_active(lab, chosen):
                continue
            h = cs.by_label[lab]
            v = _value(h, rstream.prior_draw(rng, h.dist, h.args, 1)[0])
            chosen[lab] = v
            idxs[lab] = [new_id]
            vals[lab] = [v]
        misc = dict(tid=new_id, cmd=domain.cmd, workdir=domain.workdir)
        miscs_update_idxs_vals([misc], idxs, vals)
        rval.extend(trials.new_trial_docs([new_id], [None], [domain.new_result()], [misc]))
    return rval


def suggest_batch(new_ids, domain, trials, seed):
    """hyperopt/rand.py:36-46: all ids drawn per hyperparameter at once."""
    cs = domain.space
    rng = np.random.RandomState(seed)
    chosen = {i: {} for i in new_ids}
    idxs, vals = {lab: [] for lab in cs.labels}, {lab: [] for lab in cs.labels}
    for lab in cs.draw_order:
        h = cs.by_label[lab]
        ids = [i for i in new_ids if cs.is_active(lab, chosen[i])]
        draws = rstream.prior_draw(rng, h.dist, h.args, len(ids))
        for i, v in zip(ids, draws):
            v = _value(h, v)
            chosen[i][lab] = v
            idxs[lab].append(i)
            vals[lab].append(v)
    return idxs, vals


def _suggest_device(new_ids, domain, trials, seed):
    """Prior draws on the GPU: suggestion i keyed by tpe.batch_seeds(seed)[i]."""
    from . import tpe
    new_ids = list(new_ids)
    if not new_ids:
        return []
    cs = domain.space
    st = tpe._state(domain)
    with st.lock:
        plan = st.plan_for(domain, 1, tpe.E.default_engine())
        res = plan.sample_prior(tpe.batch_seeds(seed, len(new_ids)))
    out = []
    for s, new_id in enumerate(new_ids):
        chosen = {h.label: _value(h, float(res[s, h.index]['value']))
                  for h in cs.hps if res[s, h.index]['active']}
        out.append(tpe._new_doc(domain, trials, cs, new_id, chosen))
    return out
