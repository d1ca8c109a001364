#!/usr/bin/env python3
"""Diagnostic: one config-4 1e7-candidate suggest, winners (index, value,
score) of every hp saved to a .npy for comparing two library builds."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import big_configs  # noqa: E402
from hyperopt_amd import hp, _engine as E  # noqa: E402
from hyperopt_amd.base import Domain  # noqa: E402

dom, losses, vals, active = big_configs.cfg4_domain_history(hp, Domain)
hps, conds, pprior = dom.space.engine_tables()
eng = E.Engine(0)
plan = E.Plan(eng, hps, conds, pprior, max_trials=losses.size)
plan.set_history(losses, vals, active)
plan.fit()
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
r = plan.suggest([7], n)
np.save(sys.argv[1], r)
print('saved', sys.argv[1], r['index'][0, :8], r['value'][0, :8])
