#!/usr/bin/env python3
"""GPU diagnostics: config-4 hp x0's reference candidates through the
production form (prune mode 3) against the oracle lliks, with the census;
run twice (TPE_MOMENT=1 / 0) to separate the moment form."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    import bench
    from hyperopt_amd import _engine as E
    from golden_io import load, load_json, unpack
    dom, losses, vals, active = bench.build_workload('cfg4')
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.default_engine(0), hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, active)
    plan.fit()
    meta = load_json('suggest_big_meta.json')['cfg4']
    d = load('suggest_cfg4.npz')
    for k, lab in enumerate(meta['labels'][:3]):
        h = dom.space.by_label[lab]
        x = unpack(d, 'samples', k)
        rb, ra = unpack(d, 'llik_b', k), unpack(d, 'llik_a', k)
        plan.census(True)
        lb, la, bi, bs = plan.score_candidates(h.index, x, sorted_mode=3)
        c = plan.census(False, n=10)
        err = np.abs(la - ra) / np.maximum(1, np.abs(ra))
        bad = ~(err <= 1e-6)
        print(lab, 'moment', os.environ.get('TPE_MOMENT'), 'above max rel %.3g bad %d' % (np.nanmax(err), bad.sum()),
              'census', c)
        if bad.any():
            i = np.where(bad)[0][:6]
            print('  idx', i, 'x', x[i], 'got', la[i], 'want', ra[i])


if __name__ == '__main__':
    main()
