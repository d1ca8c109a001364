#!/usr/bin/env python3
"""Diagnostic (round 4, make -C hyperopt_amd/csrc dbg4): at the finalize of
every valid wave-tile row, the candidate the tile scored (kept in registers
since the tile read it) against a plain and a volatile re-read of the same
bucketed slot, for config-4 suggests (one device, 1e7 candidates in 4
chunks; its two unaligned candidate shards), and every winner's value
against tpe_sample(index).  Diagnostic only."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ['TPE_ENGINE_LIB'] = os.path.join(ROOT, 'hyperopt_amd', 'libtpe_engine_dbg4.so')
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
    f = eng.lib.tpe_debug_reread2
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    cnt = np.zeros(4, np.uint64)
    ex = np.zeros((64, 8))
    n, seed, cut = 10_000_000, 7, 4321987
    for mode in (3, 2):
        plan.set_prune(mode)
        for name, (b, m) in {'full': (0, n), 'part0': (0, cut), 'part1': (cut, n - cut)}.items():
            eng.synchronize()
            assert f(cnt.ctypes.data, ex.ctypes.data, 1) == 0
            r = plan.suggest([seed], m, cand_begin=b)[0]
            eng.synchronize()
            assert f(cnt.ctypes.data, ex.ctypes.data, 0) == 0
            bad = sum(1 for i in range(len(hps)) if _regen(plan, hps, i, seed, r['index'][i]) != r['value'][i])
            print('mode %d %-5s rows %d  plain re-read differs %d  volatile differs %d  winners off their draw %d'
                  % (mode, name, cnt[0], cnt[1], cnt[2], bad))
            for e in ex[:min(int(cnt[3]), 4)]:
                print('   li %d cpos %d  x %.9f plain %.9f volatile %.9f  begin %d n %d hp %d' % tuple(
                    [int(e[0]), int(e[1]), e[2], e[3], e[4], int(e[5]), int(e[6]), int(e[7])]))
    plan.set_prune(3)


if __name__ == '__main__':
    main()
