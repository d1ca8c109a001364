"""Host-side split of one config-2 (or config-1) tpe.suggest call on the GPU
box: history sync, row upload, the engine call and the Python around it,
medians over an fmin-like loop (each call sees one more finished trial).
Diagnostic only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import numpy as np  # noqa: E402


def main(cfg='cfg2', n=200):
    import spaces
    from hyperopt_amd import hp, rand, tpe, Trials
    from hyperopt_amd import tpe as T
    from hyperopt_amd.base import Domain
    if cfg == 'cfg1':
        dom = Domain(lambda x: 0.0, hp.uniform('x', -5, 5))
        n_hist, n_c = 50, 24
    else:
        dom = Domain(lambda x: 0.0, spaces.cfg2_space(hp))
        n_hist, n_c = 1000, 4096
    t = Trials()
    docs = rand.suggest(list(range(n_hist)), dom, t, 1)
    for d, l in zip(docs, np.random.RandomState(2).rand(n_hist)):
        d['state'] = 2
        d['result'] = {'status': 'ok', 'loss': float(l)}
    t._insert_trial_docs(docs)
    t.refresh()
    tpe.suggest(t.new_trial_ids(1), dom, t, 1, n_EI_candidates=n_c)
    st = dom._tpe_state
    # wrap the engine call to time it apart
    plan_cls = type(st.plan)
    orig = plan_cls.fit_suggest
    tc = []

    def timed(self, *a, **k):
        t0 = time.perf_counter()
        r = orig(self, *a, **k)
        tc.append(time.perf_counter() - t0)
        return r
    plan_cls.fit_suggest = timed
    rows = []
    for i in range(n):
        ids = t.new_trial_ids(1)
        t0 = time.perf_counter()
        h = st.histories[t].sync(t)
        t1 = time.perf_counter()
        h.push(st.plan_for(dom, h.n, st.plan.engine))
        t2 = time.perf_counter()
        out = tpe.suggest(ids, dom, t, 100 + i, n_EI_candidates=n_c)
        t3 = time.perf_counter()
        rows.append((t1 - t0, t2 - t1, t3 - t2, tc[-1]))
        t.insert_trial_docs(out)
        t.refresh()
        t.trials[-1]['result'] = {'status': 'ok', 'loss': float(np.random.rand())}
        t.trials[-1]['state'] = 2
    r = 1e6 * np.median(np.asarray(rows[10:]), axis=0)
    print('%s us medians: sync %.1f  push %.1f  tpe.suggest %.1f (engine call %.1f, rest %.1f)  '
          'total %.1f' % (cfg, r[0], r[1], r[2], r[3], r[2] - r[3], r[0] + r[1] + r[2]))


if __name__ == '__main__':
    for c in sys.argv[1:] or ['cfg2']:
        main(c)
