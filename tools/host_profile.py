"""cProfile of tpe.suggest's host side in an fmin-like loop (config 2 or 3):
where the time between the host call and the returned document goes."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import numpy as np  # noqa: E402


def main(cfg='cfg2', n=200):
    import bench
    from hyperopt_amd import tpe
    r = bench.e2e_latency(cfg, 5)      # builds + warms (plan, mirror)
    print(r)
    import spaces
    from hyperopt_amd import hp, rand, Trials
    from hyperopt_amd.base import Domain
    dom = Domain(lambda x: 0.0, spaces.cfg2_space(hp))
    t = Trials()
    docs = rand.suggest(list(range(1000)), dom, t, 1)
    for d, l in zip(docs, np.random.RandomState(2).rand(1000)):
        d['state'] = 2
        d['result'] = {'status': 'ok', 'loss': float(l)}
    t._insert_trial_docs(docs)
    t.refresh()
    tpe.suggest(t.new_trial_ids(1), dom, t, 1, n_EI_candidates=4096)

    def loop():
        for i in range(n):
            ids = t.new_trial_ids(1)
            out = tpe.suggest(ids, dom, t, 100 + i, n_EI_candidates=4096)
            t.insert_trial_docs(out)
            t.refresh()
            t.trials[-1]['result'] = {'status': 'ok', 'loss': 0.5}
            t.trials[-1]['state'] = 2
    t0 = time.perf_counter()
    cProfile.runctx('loop()', globals(), locals(), '/tmp/host.prof')
    print('per iteration ms (profiled)', 1e3 * (time.perf_counter() - t0) / n)
    pstats.Stats('/tmp/host.prof').sort_stats('tottime').print_stats(25)
    pstats.Stats('/tmp/host.prof').sort_stats('cumulative').print_stats(40)


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else "cfg2", int(sys.argv[2]) if len(sys.argv) > 2 else 200)
