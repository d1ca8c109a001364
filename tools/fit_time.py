#!/usr/bin/env python3
"""Device time of one plan.fit() (split + every hp's two Parzen fits + lpdf
constants) on the bench workloads, HIP events on the launch stream."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from hyperopt_amd import _engine as E  # noqa: E402


def main(cfgs):
    import torch
    torch.cuda.set_device(0)
    eng = E.Engine(0)
    st = torch.cuda.Stream()
    for cfg in cfgs:
        dom, losses, vals, active = bench.build_workload(cfg)
        hps, conds, pprior = dom.space.engine_tables()
        plan = E.Plan(eng, hps, conds, pprior, max_trials=losses.size)
        plan.set_history(losses, vals, active)
        for _ in range(3):
            plan.fit(stream=st.cuda_stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        a.record(st)
        for _ in range(reps):
            plan.fit(stream=st.cuda_stream)
        b.record(st)
        b.synchronize()
        print('%s: P=%d N=%d fit %.1f us' % (cfg, len(hps), losses.size,
                                             1e3 * a.elapsed_time(b) / reps), flush=True)


if __name__ == '__main__':
    main(sys.argv[1:] or ['cfg2', 'cfg3', 'cfg4'])
