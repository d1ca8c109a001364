#!/usr/bin/env python3
"""Per-block timeline of the last k_score launch from the TPE_STAMPS
diagnostic build (make -C hyperopt_amd/csrc dbg): for every block of
suggestion 0, its start, the end of its component loop and its end (us from
the launch's first block start), grouped by lpdf kind, plus the CU / XCD
spread.  Diagnostic only; the product library has no stamps."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ['TPE_ENGINE_LIB'] = os.path.join(ROOT, 'hyperopt_amd', 'libtpe_engine_dbg.so')
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from hyperopt_amd import _engine as E  # noqa: E402


def main(cfg, n_cand):
    import torch
    torch.cuda.set_device(0)
    eng = E.Engine(0)
    if cfg.startswith('kind:'):  # one-kind space of tools/kind_bench.py
        sys.path.insert(0, os.path.join(ROOT, 'tools'))
        import kind_bench
        dom, losses, vals, active = kind_bench.workload(cfg[5:])
        nc = 4096
    else:
        dom, losses, vals, active = bench.build_workload(cfg)
        nc = bench.CONFIGS[cfg]['n_cand']
    n_cand = n_cand or nc
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(eng, hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, active)
    lv = int(os.environ.get('TPE_STAMPS_LEVEL', '-1'))
    for i in range(5):
        plan.fit(gamma=0.25, prior_weight=1.0, lf=25)
        # TPE_STAMPS_LEVEL=l: levels 0 .. l, one call each (level l's launch
        # is the last one: its stamps are the ones read)
        if lv < 0:
            plan.suggest([7 + i], n_cand, fetch=False)
        else:
            for l in range(lv + 1):
                if i == 4 and l == lv and hasattr(eng.lib, 'tpe_debug_wave_info_clear'):
                    eng.lib.tpe_synchronize(eng.h)
                    assert eng.lib.tpe_debug_wave_info_clear() == 0
                plan.suggest([7 + i], n_cand, level=l, fetch=False)
    eng.lib.tpe_synchronize(eng.h)
    buf = (C.c_ulonglong * (8192 * 4))()
    assert eng.lib.tpe_debug_score_stamps(buf) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 4)
    st = st.astype(np.int64)
    nb = int((st[:, 0] > 0).sum())
    t = st[:nb, :3]
    rel = (t - t[:, 0].min()) / 100.0  # 100 MHz -> us
    meta = st[:nb, 3]
    slot = (meta >> 48) & 0xffff
    tile = (meta >> 32) & 0xffff
    xcc = (meta >> 16) & 0xf
    cu = (meta >> 8) & 0xf
    se = (meta >> 13) & 0x3
    print('%s n_cand=%d blocks=%d; launch span %.1f us' % (cfg, n_cand, nb, rel[:, 2].max()))
    for sl in np.unique(slot):
        r = rel[slot == sl]
        print('%2d tiles %3d  start %6.1f..%6.1f  loop %6.1f (max %6.1f)  tail %5.1f  end max %6.1f' %
              (sl, (slot == sl).sum(), r[:, 0].min(), r[:, 0].max(), (r[:, 1] - r[:, 0]).mean(),
               (r[:, 1] - r[:, 0]).max(), (r[:, 2] - r[:, 1]).mean(), r[:, 2].max()))
    # per wave (wave tiles): component-loop durations and the block ends
    NS = 10  # tpe_score.hip kWaveStamps
    wb = (C.c_ulonglong * (8192 * 8 * NS))()
    if hasattr(eng.lib, 'tpe_debug_wave_stamps') and eng.lib.tpe_debug_wave_stamps(wb) == 0:
        ws = np.frombuffer(wb, dtype=np.uint64).reshape(8192, 8, NS).astype(np.int64)[:nb]
        okw = (ws[:, :, 0] > 0) & (ws[:, :, 1] >= ws[:, :, 0])
        if okw.any():
            t0 = t[:, 0].min()
            dur = (ws[:, :, 1] - ws[:, :, 0]) / 100.0
            start = (ws[:, :, 0] - t0) / 100.0
            end = (ws[:, :, 1] - t0) / 100.0
            d = dur[okw]
            print('wave loops: %d waves, mean %.1f us, p50 %.1f, p90 %.1f, max %.1f; wave starts '
                  '%.1f..%.1f, loop ends max %.1f us' % (d.size, d.mean(), np.median(d),
                                                          np.quantile(d, 0.9), d.max(),
                                                          start[okw].min(), start[okw].max(),
                                                          end[okw].max()))
            # block start (wave 0 entry) to each wave's start after the staging barrier
            bst = rel[:, 0]
            wst = np.where(okw, start, np.nan)
            dl = wst - bst[:, None]
            print('barrier delay (wave start - block entry): p50 %.1f p90 %.1f max %.1f us; '
                  'block entries p50 %.1f max %.1f' % (np.nanmedian(dl), np.nanquantile(dl, 0.9),
                                                       np.nanmax(dl), np.median(bst), bst.max()))
            key0 = xcc * 64 + se * 16 + cu
            bl = np.nanmax(dl, axis=1)
            for b in np.argsort(np.nan_to_num(bl, nan=-1))[::-1][:8]:
                same = np.where(key0 == key0[b])[0]
                print('  block %4d delay %5.1f us entry %5.1f  cu-mates %s entries %s ends %s' % (
                    b, bl[b], bst[b], same.tolist(), np.round(bst[same], 1).tolist(),
                    np.round(np.where(okw[same], end[same], -1).max(axis=1), 1).tolist()))
            bend = np.where(okw, end, -1).max(axis=1)
            sel = bend >= 0
            print('block ends (last wave loop): mean %.1f us, max %.1f us (max / mean %.2f)' %
                  (bend[sel].mean(), bend[sel].max(), bend[sel].max() / bend[sel].mean()))
            # loop time by the wave's place in its sort block
            # (dense value windows), from the tile mapping of tpe_score.hip
            if (ws[:, :, 2:4] > 0).all(axis=2)[okw].any():
                ok4 = okw & (ws[:, :, 2] > 0) & (ws[:, :, 3] > 0)
                ph = [(ws[:, :, 2] - ws[:, :, 0]), (ws[:, :, 3] - ws[:, :, 2]),
                      (ws[:, :, 1] - ws[:, :, 3])]
                for nm, a in zip(['candidates', 'below mixture', 'above mixture'], ph):
                    a = a[ok4] / 100.0
                    print('  %-14s mean %6.2f us  p50 %6.2f  p90 %6.2f  max %6.2f' %
                          (nm, a.mean(), np.median(a), np.quantile(a, 0.9), a.max()))
                # the above mixture's one-exponent loop by phase (waves that
                # stamped every point: the shifted loop ran and passed)
                okf = ok4 & (ws[:, :, 4:9] > 0).all(axis=2)
                if okf.any():
                    seq = [(3, 4, 'above: window'), (4, 5, 'above: pass 1'),
                           (5, 6, 'above: tightening'), (6, 7, 'above: pass 2 + guard'),
                           (7, 1, 'above: to loop end'), (1, 8, 'finalize (wave argmax)')]
                    print('  above-mixture phases over %d waves (us):' % okf.sum())
                    for a0, a1, nm in seq:
                        a = (ws[:, :, a1] - ws[:, :, a0])[okf] / 100.0
                        print('    %-24s mean %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f' %
                              (nm, a.mean(), np.median(a), np.quantile(a, 0.9), a.max()))
            if hasattr(eng.lib, 'tpe_debug_wave_info') and lv >= 0:
                ib = (C.c_uint * (8192 * 8 * 4))()
                assert eng.lib.tpe_debug_wave_info(ib) == 0
                wi = np.frombuffer(ib, dtype=np.uint32).reshape(8192, 8, 4)[:nb].astype(np.int64)
                dd = np.where(okw, dur, -1.0)
                order = np.argsort(dd.ravel())[::-1]
                print('per-wave work [shifted blocks, attempts, fallbacks, exact blocks] by loop time:')
                for q, nm in [(0.5, 'p50'), (0.9, 'p90')]:
                    sel = okw & (dur >= np.quantile(d, q - 0.05)) & (dur <= np.quantile(d, q + 0.05))
                    print('  %s band: mean %s' % (nm, np.round(wi[sel].mean(axis=0), 1).tolist()))
                for f in order[:12]:
                    b, w = divmod(int(f), 8)
                    print('  block %4d wave %d  %6.1f us  %s  phases %s' % (
                        b, w, dur[b, w], wi[b, w].tolist(),
                        np.round((ws[b, w, [2, 3, 1]] - ws[b, w, [0, 2, 3]]) / 100.0, 1).tolist()))
            hist = np.histogram(d, bins=[0, 2, 5, 10, 20, 40, 80, 1e9])[0]
            print('wave loop histogram (us: 0-2,2-5,5-10,10-20,20-40,40-80,80+):', hist.tolist())
    key = xcc * 64 + se * 16 + cu
    u, c = np.unique(key, return_counts=True)
    print('distinct (xcd, se, cu) ids: %d; blocks per id min/max %d/%d; per xcd %s' %
          (u.size, c.min(), c.max(), np.bincount(xcc, minlength=8).tolist()))


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'cfg2',
         int(sys.argv[2]) if len(sys.argv) > 2 else 0)
