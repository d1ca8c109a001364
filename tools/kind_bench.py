#!/usr/bin/env python3
"""Scoring-kernel throughput per lpdf kind: a space of N hps all of one kind
(config-2 ranges), a 1000-trial rand.suggest history and 4096 candidates; the
k_score launch time (HIP events) against the register-only pair peaks of
_engine.microbench.  Diagnostic only."""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def space(hp, kind, n):
    mk = {'u': lambda l: hp.uniform(l, -5, 5),
          'lu': lambda l: hp.loguniform(l, math.log(1e-3), math.log(10)),
          'qu': lambda l: hp.quniform(l, 0, 100, 1),
          'qlu': lambda l: hp.qloguniform(l, math.log(1e-3), math.log(100), 0.01),
          'c': lambda l: hp.choice(l, [0, 1, 2, 3])}[kind]
    return {'%s%d' % (kind, i): mk('%s%d' % (kind, i)) for i in range(n)}


def workload(kind, n_hp=15, n_hist=1000):
    """(domain, losses, vals, active) of a one-kind space with a rand history."""
    from hyperopt_amd import hp, rand, Trials, trials_from_docs
    from hyperopt_amd.base import Domain
    from hyperopt_amd.tpe import build_history
    dom = Domain(lambda x: 0.0, space(hp, kind, n_hp))
    losses = np.random.RandomState(2).rand(n_hist)
    docs = rand.suggest(list(range(n_hist)), dom, Trials(), 1)
    for d, l in zip(docs, losses):
        d['state'] = 2
        d['result'] = {'status': 'ok', 'loss': float(l)}
    t = trials_from_docs(docs, validate=False)
    _, losses, vals, active = build_history(dom, t, dom.space.labels)
    return dom, losses, vals, active


def main(kinds, n_hp, n_cand, n_hist, n_sug=1):
    import torch
    torch.cuda.set_device(0)
    from hyperopt_amd import _engine as E
    eng = E.Engine(0)
    lse_peak, erf_peak = eng.microbench(3), eng.microbench(4)
    print('peaks: lse %.0f Gpair/s, erf %.1f Gpair/s; %d hps x %d candidates x %d suggestions'
          % (lse_peak / 1e9, erf_peak / 1e9, n_hp, n_cand, n_sug))
    for kind in kinds:
        dom, losses, vals, active = workload(kind, n_hp, n_hist)
        hps, conds, pprior = dom.space.engine_tables()
        plan = E.Plan(eng, hps, conds, pprior, max_trials=losses.size)
        plan.set_history(losses, vals, active)

        def step(i):
            plan.fit(gamma=0.25, prior_weight=1.0, lf=25)
            plan.suggest([7 + i + 1000 * s for s in range(n_sug)], n_cand, fetch=False)
        for i in range(5):
            step(i)
        plan.profile(20)
        for i in range(20):
            step(100 + i)
        torch.cuda.synchronize()
        ms, pairs = 0.0, 0.0
        for k in range(len(E.KIND_NAMES)):
            m, n, p = plan.profile_read(k)
            ms = m
            pairs += p
        plan.profile(0)
        plan.census(True)
        for i in range(5):
            step(200 + i)
        cen = plan.census(False)
        ex = cen[2] / 5 if cen[0] else 0.0
        lse_ex = cen[5] / (5 * max(1, n) / 20) if cen[3] else 0.0   # evaluated LSE pairs per launch
        if kind in ('qu', 'qlu'):
            t_peak = ex / erf_peak
            extra = 'evaluated %.2fM of %.2fM pairs (live %.2fM)' % (ex / 1e6, pairs / 1e6,
                                                                       cen[1] / 5 / 1e6)
        else:
            t_peak = pairs / lse_peak if kind != 'c' else 0.0
            extra = 'evaluated LSE pairs %.3g per launch (%.1f%%)' % (
                lse_ex, 100.0 * lse_ex / pairs if pairs else 0.0)
        print('%-4s launch %7.1f us  pairs %6.2fM  %7.0f Gpair/s  t_peak %6.1f us  frac %.2f  %s'
              % (kind, ms * 1e3, pairs / 1e6, pairs / (ms * 1e-3) / 1e9 if ms else 0,
                 t_peak * 1e6, t_peak / (ms * 1e-3) if ms else 0, extra))


if __name__ == '__main__':
    ks = sys.argv[1].split(',') if len(sys.argv) > 1 else ['u', 'lu', 'qu', 'qlu', 'c']
    main(ks, int(sys.argv[2]) if len(sys.argv) > 2 else 15,
         int(sys.argv[3]) if len(sys.argv) > 3 else 4096,
         int(sys.argv[4]) if len(sys.argv) > 4 else 1000,
         int(sys.argv[5]) if len(sys.argv) > 5 else 1)
