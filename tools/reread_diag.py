#!/usr/bin/env python3
"""Finalize-time re-read of every winner's candidate (TPE_REREAD build,
``make -C hyperopt_amd/csrc dbg3``): for the full 1e7-candidate config-4
suggest (seed 7) in prune modes 2 and 3, each hp's reported (value, index)
next to the draw regenerated at that index (tpe_sample) and what a re-read
finds at each candidate address a finalize could take:

  slot   cand[li]            the winner's bucketed slot, carried through the
                             wave and block argmax reductions
  pos    cand[index - begin] the global index taken as a slot (bucketed
                             arrays are not in index order)
  (w0, the slot not carried through the block argmax of the wave tiles, was
  a round-4 column: wave tiles publish per-wave records since, no block argmax)
  own0   cand[lane 0's li]   the slot not carried through the wave argmax
  row    cand[li ^ 64]       the same lane's other candidate row

Diagnostic only; the product library has no re-read."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ['TPE_ENGINE_LIB'] = os.path.join(ROOT, 'hyperopt_amd', 'libtpe_engine_dbg3.so')
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from hyperopt_amd import hp, _engine as E  # noqa: E402
from hyperopt_amd.base import Domain  # noqa: E402
import big_configs  # noqa: E402


def regen(plan, t, i, seed, index):
    w, mu, sg = plan.mixture(i, 0)
    lo = t.low if t.flags & E.HAS_LOW else None
    hi = t.high if t.flags & E.HAS_HIGH else None
    q = t.q if t.flags & E.HAS_Q else None
    return plan.engine.sample(t.family, w, mu, sg, lo, hi, q, seed=seed, stream=i,
                              offset=int(index), n=1)[0]


def main():
    import torch
    torch.cuda.set_device(0)
    dom, L, vals, act = big_configs.cfg4_domain_history(hp, Domain)
    hps, conds, pprior = dom.space.engine_tables()
    eng = E.Engine(0)
    plan = E.Plan(eng, hps, conds, pprior, max_trials=L.size)
    plan.set_history(L, vals, act)
    plan.fit()
    n, seed = 10_000_000, 7
    buf = (C.c_double * (512 * 20))()
    for mode in (2, 3):
        plan.set_prune(mode)
        res = plan.suggest([seed], n)[0]
        eng.lib.tpe_synchronize(eng.h)
        assert eng.lib.tpe_debug_reread(buf) == 0
        d = np.frombuffer(buf, dtype=np.float64).reshape(512, 20)
        bad = {'reported': 0, 'slot': 0, 'pos': 0, 'own0': 0, 'row': 0, 'cpos': 0}
        near = []  # |other row - draw|: the row variant's values sit in the wave's window
        rows = []
        for h in dom.space.hps:
            i = h.index
            r = res[i]
            g = regen(plan, hps[i], i, seed, r['index'])
            fv, fi, lt, v_slot, cp, v_pos, v_w0, v_own, beg = d[i, :9]
            assert fv == r['value'] and int(fi) == int(r['index']), (h.label, d[i], r)
            bad['reported'] += fv != g
            bad['slot'] += v_slot != g
            bad['pos'] += v_pos != g
            bad['own0'] += v_own != g
            bad['row'] += d[i, 16] != g
            near.append(abs(d[i, 16] - g))
            bad['cpos'] += int(cp) + int(beg) != int(fi)
            rows.append((h.label, int(fi), int(beg), int(lt), int(cp), g, fv, v_slot, v_pos, v_w0, v_own,
                         d[i, 16]))
        print('mode %d: hps whose re-read differs from the regenerated draw: %s (of %d)' %
              (mode, bad, len(rows)))
        for row in rows:
            if row[0] in ('x10', 'x0', 'x1') or row[6] != row[5]:
                print('  %-4s index %8d begin %8d slot %7d cpos %7d | draw %.12f reported %.12f '
                      'slot %.12f pos %.12f w0 %.12f own0 %.12f row %.12f' % row)
        print('  other-row values: median |row - draw| %.4f, max %.4f' %
              (float(np.median(near)), float(np.max(near))))
        cand_ptr, part_ptr, ncand, cpos_ptr = d[0, 12], d[0, 13], d[0, 14], d[0, 15]
        print('  cand %#x (+%d B / slot) partial %#x cpos %#x' %
              (int(cand_ptr), int(ncand) * 8, int(part_ptr), int(cpos_ptr)))
    plan.set_prune(3)


if __name__ == '__main__':
    main()
