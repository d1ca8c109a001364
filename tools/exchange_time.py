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
                 timed alone on the sharded stream with HIP events, issued
                 back to back (bound by the host's issue when that is longer)
  exchange_device_us  the same on a stream held by a sleep kernel while the
                 host queues them: the device time of the exchange alone
  exchange_host_issue_us  the host's issue time per suggest (perf_counter)
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
    gbuf = torch.empty(sh.world * local.numel(), dtype=torch.uint8, device='cuda')
    sh.suggest([7], n_cand, fetch=False)
    torch.cuda.synchronize()
    nx = 200

    # (the product path: the all-gather reads the plan's own records, the
    # merge stores the merged slots in place -- ShardedSuggest.suggest;
    # TPE_EXCHANGE_COPY=1: the round-6 path with a copy launch on each side)
    copy_path = os.environ.get('TPE_EXCHANGE_COPY') == '1'
    mine = sh._plan_records(S * P * parallel.RECORD_BYTES)

    def exchange_loop(n):
        for _ in range(n):
            for level in range(plan.n_levels):
                if mine is None:
                    plan.get_results(out=local.data_ptr(), stream=sh.stream.cuda_stream)
                src = local if mine is None else mine
                if sh._rccl and not copy_path:   # (ShardedSuggest.suggest's issue)
                    sh._all_gather(gbuf, src, group=sh.group)
                    g = gbuf
                else:
                    g = sh.gather(src, gbuf)
                plan.merge(g.data_ptr(), sh.world, level, out=local.data_ptr(),
                           stream=sh.stream.cuda_stream, n_suggest=S, in_place=not copy_path)

    with torch.cuda.stream(sh.stream):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        exchange_loop(5)
        # (1) back to back as the host issues them (host-issue-bound when
        # the device work is shorter than the issue)
        a.record(sh.stream)
        exchange_loop(nx)
        b.record(sh.stream)
        torch.cuda.synchronize()
        exch_us = 1e3 * a.elapsed_time(b) / nx
        # (2) device time alone: the stream is held by a sleep kernel while
        # the host queues the exchanges, so the events see them back to back
        # on the device (what a level costs when its suggest's kernels keep
        # the device busy while the host issues the exchange, configs 3-5)
        torch.cuda._sleep(int(2e8))
        a.record(sh.stream)
        import time
        t0 = time.perf_counter()
        exchange_loop(nx)
        host_us = 1e6 * (time.perf_counter() - t0) / nx
        b.record(sh.stream)
        torch.cuda.synchronize()
        dev_us = 1e3 * a.elapsed_time(b) / nx
    print(json.dumps(dict(config=args.config, n_cand=n_cand, n_levels=plan.n_levels, n_hp=P,
                          record_bytes_per_rank=S * P * parallel.RECORD_BYTES,
                          single_ms=single, sharded_ms=sharded_ms, fit_ms=fit_ms,
                          exchange_us_per_suggest=exch_us,
                          exchange_device_us_per_suggest=dev_us,
                          exchange_host_issue_us_per_suggest=host_us,
                          plan_view=mine is not None, copy_path=copy_path,
                          note='world 1 over RCCL: the fixed part of the exchange '
                               '(collective launch + kernel, k_merge), no xGMI transfer')))
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
