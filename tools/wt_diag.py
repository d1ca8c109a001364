#!/usr/bin/env python3
"""Diagnostic: a 2^18-candidate cfg2 suggest on the sorted (pruned) path vs
the unsorted one-per-thread path merged from two chunks; prints the per-hp
winners and scores where they differ, and the engine's lpdfs of both
winning candidates (operator path) for those hps."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import torch  # noqa: E402
import test_gpu_suggest as T  # noqa: E402
from hyperopt_amd import tpe  # noqa: E402

meta, d, dom, trials = T._fixture_trials('cfg2')
tpe.suggest([meta['new_id']], dom, trials, 7, n_EI_candidates=64)
plan = dom._tpe_state.plan
n, cut = 1 << 18, 100_000
full = plan.suggest([13], n)
parts = [plan.suggest([13], cut, cand_begin=0), plan.suggest([13], n - cut, cand_begin=cut)]
raw = torch.from_numpy(np.stack(parts).view(np.uint8).reshape(-1).copy()).cuda()
merged = plan.merge(raw.data_ptr(), world=2, level=0)
torch.cuda.synchronize()
print(full.dtype.names)
for j, lab in enumerate(dom.space.labels):
    a, b = full[0, j], merged[0, j]
    flag = '' if a['index'] == b['index'] else '   <-- differ'
    print('%-6s full idx %7d score %.17g value %.17g | merged idx %7d score %.17g value %.17g%s' % (
        lab, a['index'], a['score'], a['value'], b['index'], b['score'], b['value'], flag))
