#!/usr/bin/env python3
"""Per-phase timing of k_fit from the TPE_STAMPS debug build
(make -C hyperopt_amd/csrc dbg).  Prints, per (hp, side) slot, the µs spent
in each phase of the last fit.  Diagnostic only."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ['TPE_ENGINE_LIB'] = os.path.join(ROOT, 'hyperopt_amd', 'libtpe_engine_dbg.so')
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from hyperopt_amd import _engine as E  # noqa: E402

PH = ['split', 'gather', 'lds', 'sort/bincount', 'sigma', 'normalise', 'wsum', 'pacc', 'end_cat',
      'end']


def main(cfg):
    import torch
    torch.cuda.set_device(0)
    eng = E.Engine(0)
    dom, losses, vals, active, n_cand = bench.build_workload(cfg)
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(eng, hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, active)
    for _ in range(3):
        plan.fit()
    eng.lib.tpe_synchronize(eng.h)
    buf = (C.c_ulonglong * (512 * 16))()
    assert eng.lib.tpe_debug_stamps(buf) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(512, 16).astype(np.int64)
    P = len(dom.space.labels)
    t0 = st[:2 * P, 0].min()
    print(cfg, 'P=%d N=%d' % (P, losses.size))
    for slot in range(2 * P):
        row = st[slot]
        h = dom.space.hps[slot // 2]
        marks = [(PH[i - 1], (row[i] - row[0]) / 100.0) for i in range(1, 11) if row[i] >= row[0]]
        print('%-8s %-10s side=%d start=%6.1fus ' % (h.label[:8], h.dist[:10], slot % 2,
                                                     (row[0] - t0) / 100.0) +
              ' '.join('%s=%.1f' % m for m in marks))
    end = max(st[s, 10] if st[s, 10] else st[s, 9] for s in range(2 * P))
    print('kernel span (first start -> last end): %.1f us' % ((end - t0) / 100.0))


if __name__ == '__main__':
    for c in sys.argv[1:] or ['cfg2']:
        main(c)
