"""A/B of the log-sum-exp modes (tpe_plan_set_prune: 2 skip + one exponent
per wave, 1 skip, 0 every pair) on a BASELINE config (time per suggest,
census of evaluated pairs, max |delta score| vs mode 0).  Diagnostic: python tools/ab_prune.py cfg4"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

import numpy as np  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else 'cfg4'
    n_cand = int(sys.argv[2]) if len(sys.argv) > 2 else {'cfg4': 10_000_000, 'cfg2': 4096,
                                                         'cfg3': 100_000, 'cfg5': 1_000_000}[cfg]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    import bench
    from hyperopt_amd import _engine as E
    dom, losses, vals, active = bench.build_workload('cfg2' if cfg == 'cfg5' else cfg)
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, active)
    seeds = [7] if cfg != 'cfg5' else list(range(16))
    out = {}
    res = {}
    for mode in (2, 1, 0):
        plan.set_prune(mode)
        plan.fit_suggest(seeds, n_cand)            # warm
        t0 = time.perf_counter()
        for i in range(reps):
            r = plan.fit_suggest([s + 100 * i for s in seeds], n_cand)
        dt = (time.perf_counter() - t0) / reps
        plan.census(True)
        res[mode] = plan.fit_suggest(seeds, n_cand)
        c = plan.census(False)
        out['mode%d' % mode] = dict(ms=1e3 * dt, census=c, lse_eval_frac=c[5] / max(1, c[3]))
        print(json.dumps({'mode%d' % mode: out['mode%d' % mode]}), flush=True)
    for mode in (2, 1):
        a, b = res[mode], res[0]
        out['mode%d' % mode].update(
            speedup=out['mode0']['ms'] / out['mode%d' % mode]['ms'],
            index_diff=int((a['index'] != b['index']).sum()),
            max_abs_dscore=float(np.nanmax(np.abs(a['score'] - b['score']))))
    print(json.dumps(out))


if __name__ == '__main__':
    main()
