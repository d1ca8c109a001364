#!/usr/bin/env python3
"""GPU diagnostics: the moment table (CoefM) of a config-4 slot written by
k_fit, against the numpy restatement of tools/moment_error.py."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import moment_error as ME  # noqa: E402

MOM = np.dtype([('center', '<f8'), ('base', '<f4'), ('cm', '<f4'), ('gam', '<f4'),
                ('m', '<f4', (10,)), ('xh', '<f4')])


def main():
    import bench
    from hyperopt_amd import _engine as E
    dom, losses, vals, active = bench.build_workload('cfg4')
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.default_engine(0), hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, active)
    plan.fit()
    hp = dom.space.by_label['x0'].index
    w, mu, sg = plan.mixture(hp, 1)
    t = plan.table(hp, 1, 2).view(MOM)
    B = ME.tables(w, mu, sg, -5.0, 5.0, 0.0)
    n = B['cen'].size
    print('chunks', n, 'table entries', t.size, 'K', w.size)
    for f, g in (('center', B['cen']), ('xh', B['xh']), ('base', B['base']), ('cm', B['cm']),
                 ('gam', B['gam'])):
        a = t[f][:n].astype(np.float64)
        b = np.asarray(g, np.float64)
        fin = np.isfinite(b)
        d = np.abs(a[fin] - b[fin])
        print(f, 'max |d| %.3g' % d.max(), 'nonfinite dev %d ref %d' % ((~np.isfinite(a)).sum(), (~fin).sum()),
              'ex', a[:3], b[:3])
    mm = t['m'][:n].astype(np.float64)
    rel = np.abs(mm - B['mom']) / np.maximum(1e-30, np.abs(B['mom']))
    print('moments max rel %.3g' % np.nanmax(np.where(np.isfinite(B['xh'])[:, None], rel, 0)))
    print('ex m dev', mm[5], '\nex m ref', B['mom'][5])


if __name__ == '__main__':
    main()
