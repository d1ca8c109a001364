#!/usr/bin/env python3
"""Per-phase timing of k_fit from the TPE_STAMPS diagnostic build
(make -C hyperopt_amd/csrc dbg): for each (hp, side) slot of the last fit,
the time (us from the slot's start) at which each phase ended.  Diagnostic
only; the product library has no stamps."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ['TPE_ENGINE_LIB'] = os.path.join(
    ROOT, 'hyperopt_amd', os.environ.get('TPE_STAMPS_LIB', 'libtpe_engine_dbg.so'))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from hyperopt_amd import _engine as E  # noqa: E402

PH = {11: 'keys', 12: 'd1', 13: 'd2', 14: 'd3', 15: 'd4', 1: 'split', 2: 'gather', 3: 'sort', 4: 'place', 5: 'sigma/bins', 6: 'norm', 7: 'wsum',
      8: 'pacc', 10: 'end'}


def main(cfg, slots):
    import torch
    torch.cuda.set_device(0)
    eng = E.Engine(0)
    if cfg == 'cfg1':  # one uniform hp, 50 finished trials (the config-1 fmin's mid point)
        from hyperopt_amd import hp, rand, Trials
        from hyperopt_amd.base import Domain
        from hyperopt_amd.tpe import build_history
        dom, t = Domain(lambda x: 0.0, hp.uniform('x', -5, 5)), Trials()
        docs = rand.suggest(list(range(50)), dom, t, 1)
        for d, l in zip(docs, np.random.RandomState(2).rand(50)):
            d['state'] = 2
            d['result'] = {'status': 'ok', 'loss': float(l)}
        t._insert_trial_docs(docs)
        t.refresh()
        _, losses, vals, active = build_history(dom, t, dom.space.labels)
    else:
        dom, losses, vals, active = bench.build_workload(cfg)
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(eng, hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, active)
    for _ in range(3):
        plan.fit()
    eng.lib.tpe_synchronize(eng.h)
    buf = (C.c_ulonglong * (512 * 48))()
    assert eng.lib.tpe_debug_stamps(buf) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(512, 48).astype(np.int64)
    P = len(dom.space.labels)
    t0 = st[:2 * P, 0].min()
    print(cfg, 'P=%d N=%d' % (P, losses.size))
    order = range(min(2 * P, slots))
    if 'TPE_STAMPS_SLOTS' in os.environ:  # the slowest slots, slowest last
        order = sorted(np.argsort(st[:2 * P, 10] - t0)[-slots:], key=lambda s: st[s, 10])
    for slot in order:
        row = st[slot]
        h = dom.space.hps[slot // 2]
        marks = ['%s=%.1f' % (PH[i], (row[i] - row[0]) / 100.0) for i in [11, 12, 13, 14, 15] + sorted(k for k in PH if k < 11)
                 if row[i] >= row[0]]
        print('%-8s %-10s side=%d start=%5.1f ' % (h.label[:8], h.dist[:10], slot % 2,
                                                   (row[0] - t0) / 100.0) + ' '.join(marks))
    print('kernel span: %.1f us' % ((st[:2 * P, 10].max() - t0) / 100.0))
    sub = {16: 'sd.zero', 17: 'sd.hist', 18: 'sd.bar1', 19: 'sd.scan', 20: 'sd.bar2',
           21: 'ms.load', 22: 'ms.bitonic64', 23: 'ms.bar|L64', 24: 'ms.L64|256', 25: 'ms.L128|1024',
           26: 'ms.L256|fix', 27: 'ms.L512|or', 28: 'np.plan', 29: 'np.leaves', 30: 'np.end',
           31: 'k.zero', 32: 'k.load', 33: 'k.wred', 34: 'k.bar', 35: 'g.load', 36: 'g.scan', 37: 'g.write',
           38: 'rs.init', 39: 'rs.pass', 40: 'cat.seg', 41: 'cat.lfw'}
    slowest = int(np.argmax(st[:2 * P, 10] - st[:2 * P, 0]))
    extra = {int(v) for v in os.environ.get('TPE_STAMPS_DETAIL', '').split(',') if v}
    for slot in sorted(set(range(min(2 * P, 4))) | {slowest} | {e for e in extra if e < 2 * P}):
        row = st[slot]
        print('slot %d last sub-phase stamps (us from slot start): ' % slot + ' '.join(
            '%s=%.2f' % (nm, (row[i] - row[0]) / 100.0) for i, nm in sub.items() if row[i] >= row[0]))
    wall = (st[:2 * P, 10] - st[:2 * P, 0]) / 100e6
    print('shader clock during the fit: %.0f MHz (median over slots)' %
          np.median(st[:2 * P, 9] / np.maximum(wall, 1e-9) / 1e6))


if __name__ == '__main__':
    # usage: fit_stamps.py [config ...]; TPE_STAMPS_SLOTS=n prints the n slowest slots
    for c in sys.argv[1:] or ['cfg2']:
        main(c, int(os.environ.get('TPE_STAMPS_SLOTS', '40')))
