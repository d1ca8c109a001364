#!/usr/bin/env python3
"""Host-side cost per step of the eager fit()+suggest() path and of the
graph-replayed fit_suggest(): enqueue time of N back-to-back steps (no sync)
against their total time.  Diagnostic only."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main(n=200):
    import torch
    torch.cuda.set_device(0)
    from hyperopt_amd import _engine as E
    eng = E.Engine(0)
    dom, losses, vals, active = bench.build_workload('cfg2')
    n_cand = bench.CONFIGS['cfg2']['n_cand']
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(eng, hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, active)

    def eager(i):
        plan.fit()
        plan.suggest([i], n_cand, fetch=False)

    def graph(i):
        plan.fit_suggest([i], n_cand, fetch=False)

    for name, f in (('eager', eager), ('graph', graph), ('eager', eager), ('graph', graph)):
        for i in range(5):
            f(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            f(i)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print('%-6s enqueue %7.1f us/step  total %7.1f us/step' %
              (name, 1e6 * (t1 - t0) / n, 1e6 * (t2 - t0) / n), flush=True)
    # raw ctypes call floor
    t0 = time.perf_counter()
    for i in range(n):
        eng.lib.tpe_plan_num_levels(plan.p, None)
    print('ctypes call floor %.2f us' % (1e6 * (time.perf_counter() - t0) / n))


if __name__ == '__main__':
    main()
