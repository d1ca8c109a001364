#!/usr/bin/env python3
"""Pass rates of the reference's quality thresholds (tests/domains.py) for
the device Philox stream and the reference RandomState stream over many fmin
seeds.  Diagnostic only."""
import functools
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main(names, seeds):
    import domains
    import hyperopt_amd as H
    from hyperopt_amd import fmin, tpe, Trials, hp
    from hyperopt_amd.expr import as_apply
    for name in names:
        kw, n = domains.settings(name)
        out = {}
        for stream in ('philox', 'numpy'):
            wins = 0
            for seed in range(seeds):
                t = Trials()
                fmin(lambda x: x, domains.build(name, hp, H.scope, as_apply),
                     algo=functools.partial(tpe.suggest, rng_stream=stream, **kw), max_evals=n,
                     trials=t, rstate=np.random.RandomState(123 + seed))
                wins += min(t.losses()) < domains.THRESH[name]
            out[stream] = wins
        print(name, out, 'of', seeds, flush=True)


if __name__ == '__main__':
    main(sys.argv[1].split(','), int(sys.argv[2]) if len(sys.argv) > 2 else 20)
