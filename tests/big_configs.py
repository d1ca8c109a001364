"""Configs 3 and 4 at BASELINE size, rebuilt deterministically on any host
(the GPU box has no reference): the same histories tests/golden/make_golden.py
fed the reference for suggest_cfg4.npz / suggest_cfg3_full.npz."""
import numpy as np

import spaces

CFG4_N, CFG4_D = 10000, 100


def cfg4_columns():
    """obs RandomState(1).uniform(-5, 5, (1e4, 100)),
    losses RandomState(2).rand(1e4); hp i is label 'x%d' % i."""
    U = np.random.RandomState(1).uniform(-5, 5, (CFG4_N, CFG4_D))
    L = np.random.RandomState(2).rand(CFG4_N)
    return U, L


def cfg4_domain_history(hp, Domain):
    """(domain, losses[n], vals[P, n], active[P, n]) in the domain's label order."""
    dom = Domain(lambda x: 0.0, spaces.cfg4_space(hp, CFG4_D))
    U, L = cfg4_columns()
    idx = [int(lab[1:]) for lab in dom.space.labels]
    vals = np.ascontiguousarray(U.T[idx])
    return dom, L, vals, np.ones_like(vals, dtype=np.uint8)


def cfg3_trials(hp, Domain, Trials, rand, n=10000):
    dom = Domain(lambda x: 0.0, spaces.cfg3_space(hp))
    t = Trials()
    docs = rand.suggest(list(range(n)), dom, t, 1)
    for d, l in zip(docs, np.random.RandomState(2).rand(n)):
        d['state'] = 2
        d['result'] = {'status': 'ok', 'loss': float(l)}
    t._insert_trial_docs(docs)
    t.refresh()
    return dom, t
