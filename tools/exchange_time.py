"""Time the multi-GPU exchange of a sharded suggest on ONE GPU (verdict r4 item 5).

The exchange replaces the cross-GPU half of broadcast_best (reference
hyperopt/tpe.py:749-759): per conditional level, an RCCL all-gather of the
G x S x P x 32-byte records and the device max-loc merge (k_merge).  At one
rank the all-gather moves no data over xGMI, so this measures the fixed part
(RCCL launch + its kernel, k_merge, the stream hand-offs), per suggest.

Prints one JSON line:
  single_ms      plan.fit_suggest (one device, no exchange)
  sharded_ms     ShardedSuggest.fit + suggest at world 1 (levels + exchange)
  exchange_us    per suggest: n_levels x (all_gather_into_tensor + merge),
                 timed alone on the sharded stream with HIP events
  fit_ms         plan.fit alone (every rank repeats it)
usage: python tools/exchange_time.py --config cfg2|cfg3|cfg4 [--reps N]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='cfg2')
    ap.add_argument('--reps', type=int, default=50)
    args = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(bench._free_port()),
                      RANK='0', WORLD_SIZE='1')
    torch.cuda.set_device(0)
    with bench._StdoutToStderr():
        dist.init_process_group('nccl', device_id=torch.device('cuda', 0))
        dist.barrier()
    from hyperopt_amd import _engine as E
    from hyperopt_amd import parallel
    eng = E.default_engine(0)
    dom, losses, vals, active = bench.build_workload(args.config)
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(eng, hps, conds, pprior, max_trials=losses.size)
    plan.set_history(losses, vals, active)
    n_cand = bench.CONFIGS[args.config]['n_cand']
    reps = args.reps if args.config != 'cfg4' else max(2, min(args.reps, 5))
    sh = parallel.ShardedSuggest(plan)

    def timed(fn, n):
        fn(0)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        import time
        t0 = time.perf_counter()
        for i in range(n):
            fn(i + 1)
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / n

    single = timed(lambda i: plan.fit_suggest([7 + i], n_cand, fetch=False), reps)

    def sharded(i):
        sh.fit()
        sh.suggest([7 + i], n_cand, fetch=False)
    sharded_ms = timed(sharded, reps)
    fit_ms = timed(lambda i: plan.fit(), reps)

    # the exchange alone, on the sharded stream, events on that stream
    S, P = 1, plan.n_hp
    local = torch.empty(S * P * parallel.RECORD_BYTES, dtype=torch.uint8, device='cuda')
    sh.suggest([7], n_cand, fetch=False)
    torch.cuda.synchronize()
    nx = 200
    with torch.cuda.stream(sh.stream):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        for warm in (True, False):
            if not warm:
                a.record(sh.stream)
            for _ in range(5 if warm else nx):
                for level in range(plan.n_levels):
                    g = sh.gather(local)
                    plan.merge(g.data_ptr(), sh.world, level, out=local.data_ptr(),
                               stream=sh.stream.cuda_stream, n_suggest=S)
            if not warm:
                b.record(sh.stream)
    torch.cuda.synchronize()
    exch_us = 1e3 * a.elapsed_time(b) / nx
    print(json.dumps(dict(config=args.config, n_cand=n_cand, n_levels=plan.n_levels, n_hp=P,
                          record_bytes_per_rank=S * P * parallel.RECORD_BYTES,
                          single_ms=single, sharded_ms=sharded_ms, fit_ms=fit_ms,
                          exchange_us_per_suggest=exch_us,
                          note='world 1 over RCCL: the fixed part of the exchange '
                               '(collective launch + kernel, k_merge), no xGMI transfer')))
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
