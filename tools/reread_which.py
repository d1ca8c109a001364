#!/usr/bin/env python3
"""Diagnostic (round 4, make -C hyperopt_amd/csrc dbg5: the winner's value
taken from a plain finalize re-read of its slot): for the winners whose
value is not the draw at their index, the index whose draw the value is
(all 1e7 draws of the hp regenerated).  Diagnostic only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ['TPE_ENGINE_LIB'] = os.path.join(ROOT, 'hyperopt_amd', 'libtpe_engine_dbg5.so')
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    import big_configs
    from hyperopt_amd import hp, _engine as E
    from hyperopt_amd.base import Domain
    from test_gpu_shifted import _regen
    dom, L, vals, act = big_configs.cfg4_domain_history(hp, Domain)
    hps, conds, pprior = dom.space.engine_tables()
    eng = E.default_engine()
    plan = E.Plan(eng, hps, conds, pprior, max_trials=L.size)
    plan.set_history(L, vals, act)
    plan.fit()
    n, seed = 10_000_000, 7
    r = plan.suggest([seed], n)[0]
    off = sum(1 for i in range(len(hps)) if _regen(plan, hps, i, seed, r['index'][i]) != r['value'][i])
    print('config 4 seed %d: %d of %d winners off the draw at their index' % (seed, off, len(hps)))
    shown = 0
    for i in range(len(hps)):
        d = _regen(plan, hps, i, seed, r['index'][i])
        if d == r['value'][i]:
            continue
        t = hps[i]
        w, mu, sg = plan.mixture(i, 0)
        allx = eng.sample(t.family, w, mu, sg, t.low, t.high, None, seed=seed, stream=i, offset=0, n=n)
        hit = np.flatnonzero(allx == r['value'][i])
        lb, la, _, _ = plan.score_candidates(i, np.array([r['value'][i], d]))
        print('hp %2d winner index %8d draw %.9f | reported %.9f = draw of index %s | EI(reported) %.9f EI(draw) %.9f score %.9f'
              % (i, r['index'][i], d, r['value'][i], hit[:4].tolist(), lb[0] - la[0], lb[1] - la[1], r['score'][i]))
        shown += 1
        if shown >= 8:
            break


if __name__ == '__main__':
    main()
