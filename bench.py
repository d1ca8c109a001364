#!/usr/bin/env python3
"""bench.py -- TPE candidate-scoring throughput of the MI355X engine.

Metric (BASELINE.json): "EI candidates scored/sec (x components)" = (candidate,
mixture-component) lpdf pairs per second, plus tpe.suggest latency.

One *step* = one whole device-side ``tpe.suggest`` posterior pass over the
config's synthetic history, resident in HBM: good/bad split, both Parzen fits
of every hyperparameter, Philox candidate draws, below/above lpdf of every
candidate against every component, EI argmax.  Default workload: BASELINE
configs[1] = config 2 (20-D mixed space, 1000-trial history, 4096 candidates).

--config cfg5 (BASELINE configs[4]: batched asynchronous suggestions x 1e6
candidates, config 2's space and history): one step = one batch of --batch
suggestions per rank in one engine call.

Multi-GPU (torch.distributed.run, one rank per GPU): weak scaling, each rank
serves its own asynchronous suggestions (distinct seeds) on the shared
history, no collective inside the timed region (batched suggestions shard
with no data exchange; the in-suggest candidate sharding + RCCL max-loc path
is hyperopt_amd/parallel.py:ShardedSuggest, covered by tests/test_parallel.py).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def build_workload(cfg):
    """(domain, losses, vals, active, n_cand, description)."""
    import spaces
    from hyperopt_amd import hp, rand, Trials
    from hyperopt_amd.base import Domain
    from hyperopt_amd.tpe import build_history
    if cfg in ('cfg2', 'cfg5'):
        dom = Domain(lambda x: 0.0, spaces.cfg2_space(hp))
        n_hist, n_cand = 1000, (4096 if cfg == 'cfg2' else 1_000_000)
    elif cfg == 'cfg3':
        dom = Domain(lambda x: 0.0, spaces.cfg3_space(hp))
        n_hist, n_cand = 10000, 100000
    elif cfg == 'cfg4':
        dom = Domain(lambda x: 0.0, spaces.cfg4_space(hp))
        n_hist, n_cand = 10000, 10_000_000
    else:
        raise ValueError(cfg)
    losses = np.random.RandomState(2).rand(n_hist)
    if cfg == 'cfg4':   # obs RandomState(1).uniform(-5,5,(1e4,100))
        vals = np.random.RandomState(1).uniform(-5, 5, (n_hist, 100)).T.copy()
        idx = np.array([int(l[1:]) for l in dom.space.labels])   # labels sort as strings
        vals = np.ascontiguousarray(vals[idx])
        active = np.ones_like(vals, dtype=np.uint8)
    else:
        docs = rand.suggest(list(range(n_hist)), dom, Trials(), 1)
        for d, l in zip(docs, losses):
            d['state'] = 2
            d['result'] = {'status': 'ok', 'loss': float(l)}
        from hyperopt_amd import trials_from_docs
        t = trials_from_docs(docs, validate=False)
        _, losses, vals, active = build_history(dom, t, dom.space.labels)
    return dom, losses, vals, active, n_cand


def cpu_baseline(dom, losses, vals, active, n_cand, budget_s):
    """The oracle (numpy restatement, pinned to the reference) timed on one
    host core over whole suggests of the bench's own space and history, with a
    bounded candidate count (the reference path holds 8*n_c*K-byte temporaries,
    so configs 3-5 cannot run at full n_c on the host); pairs as the GPU counts
    them."""
    os.environ.setdefault('OPENBLAS_NUM_THREADS', '1')
    from oracle import tpe_oracle as O
    import spaces
    cs = dom.space
    hps = {h.label: dict(dist=h.dist, args=h.args,
                         conds=tuple(p for p in (h.paths[0] if h.paths else ()))) for h in cs.hps}
    tids = np.arange(losses.size)
    obs = {h.label: (tids[active[h.index] == 1], vals[h.index][active[h.index] == 1])
           for h in cs.hps}
    runs, t_total, pairs = 0, 0.0, 0.0
    with np.errstate(all='ignore'):
        while t_total < budget_s or runs == 0:
            t0 = time.perf_counter()
            chosen, det = O.suggest_reference_stream(hps, tids, losses, obs, 7 + runs,
                                                     n_ei=n_cand)
            t_total += time.perf_counter() - t0
            runs += 1
            for lab, dd in det.items():
                if cs.by_label[lab].is_categorical or len(dd['cand']) == 0:
                    continue
                pairs += len(dd['cand']) * (len(dd['below'][0]) + len(dd['above'][0]))
    return dict(value=pairs / t_total, unit='pairs/s', cores=1, kind='port',
                sample='%d whole suggests of this config (%d candidates each) through the '
                       'oracle (numpy/scipy float64 restatement of tpe.py, bit-equal to '
                       'reference fixtures), single thread, %.1f s' % (runs, n_cand, t_total),
                suggest_s=t_total / runs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--config', default='cfg2', choices=['cfg2', 'cfg3', 'cfg4', 'cfg5'])
    ap.add_argument('--batch', type=int, default=0,
                    help='suggestions per rank per step (default 1; cfg5: 16)')
    ap.add_argument('--cpu-seconds', type=float, default=12.0)
    ap.add_argument('--n-cand', type=int, default=0,
                    help='override candidates per suggest (secondary measurements only)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--traffic-json', default=os.path.join(ROOT, 'profiles', 'traffic.json'))
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))

    from hyperopt_amd import _engine as E
    eng = E.Engine(local)
    dom, losses, vals, active, n_cand = build_workload(args.config)
    if args.n_cand:
        n_cand = args.n_cand
    batch = args.batch or (16 if args.config == 'cfg5' else 1)
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(eng, hps, conds, pprior, max_trials=losses.size)
    # history resident in HBM before the timed region
    d_losses = torch.from_numpy(np.ascontiguousarray(losses)).cuda()
    d_vals = torch.from_numpy(np.ascontiguousarray(vals)).cuda()
    d_act = torch.from_numpy(np.ascontiguousarray(active)).cuda()
    torch.cuda.synchronize()
    plan.set_history_device(d_losses.data_ptr(), d_vals.data_ptr(), d_act.data_ptr(),
                            losses.size)

    def step(i):
        # fit + suggest in one engine call (a replayed hipGraph after the first
        # call of this shape); results stay device-resident in the plan
        seeds = [1_000_003 * rank + 4099 * i + 17 * b + 7 for b in range(batch)]
        plan.fit_suggest(seeds, n_cand, gamma=0.25, prior_weight=1.0, lf=25, fetch=False)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device='cuda')
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    _, pairs_step = plan.last_stats()
    value = world * pairs_step * args.steps / elapsed

    # ---- profiled pass (after the timed region): HIP events on the engine
    # stream around every scoring launch, and the quantized-pair census
    n_prof = max(1, min(args.steps, 20))
    plan.profile(n_prof * 64)   # event ring: every scoring launch of every profiled step
    for i in range(n_prof):
        step(args.warmup + args.steps + i)
    kinds = {}
    score_ms, launches = 0.0, 0
    for kind, name in enumerate(E.KIND_NAMES):
        ms, n, pairs = plan.profile_read(kind)
        score_ms, launches = ms, n
        if pairs:
            kinds[name] = pairs
    lat_ms, lat_launches, lat_pairs = plan.profile_read(5)
    plan.profile(0)
    # A/B: the same steps with every quantized candidate scored on its own
    # (no value lattice), timed like the main region
    no_lat = None
    if lat_launches and args.config == "cfg2":
        plan.set_lattice(False)
        for i in range(max(1, args.warmup)):
            step(i)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        t1 = time.perf_counter()
        for i in range(args.steps):
            step(args.warmup + i)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        e1 = time.perf_counter() - t1
        t = torch.tensor([e1], dtype=torch.float64, device='cuda')
        if dist:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        e1 = float(t.item())
        no_lat = dict(value=world * pairs_step * args.steps / e1, ms_per_step=1e3 * e1 / args.steps)
        plan.set_lattice(True)
    # census pass (its counting variant of the kernel is not timed)
    plan.census(True)
    for i in range(n_prof):
        step(args.warmup + args.steps + n_prof + i)
    census = plan.census(False)

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    # ---- roofline of the dominant kernel, k_score (every lpdf kind of the
    # level in one launch).  Work is priced at the measured register-only
    # rate of exactly its pair arithmetic: log-sum-exp pairs (2 FMA + max +
    # exp2 + fp64 sum) and evaluated quantized pairs (2 fp64 erf); quantized
    # pairs that are exact zeros for the whole wave are skipped by the
    # algorithm and cost no erf.
    lse_peak = eng.microbench(3)
    erf_peak = eng.microbench(4)
    lse_pairs = kinds.get('lse_gmm', 0.0) + kinds.get('lse_lgmm', 0.0)
    erf_pairs = kinds.get('erf_gmm', 0.0) + kinds.get('erf_lgmm', 0.0)
    per_launch = max(1, launches)
    erf_exec = census[2] / per_launch
    t_kernel = score_ms * 1e-3
    t_peak = lse_pairs / lse_peak + erf_exec / erf_peak
    achieved = (lse_pairs + erf_exec * lse_peak / erf_peak) / t_kernel if t_kernel else 0.0
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                traffic = json.load(f).get(args.config, {}).get('score')
        except Exception:
            traffic = None
    roof = dict(bound='valu', unit='Gpair/s', achieved=achieved / 1e9, peak=lse_peak / 1e9,
                frac=(t_peak / t_kernel) if t_kernel else None, traffic=traffic,
                kernel='k_score (all lpdf kinds of a level, one launch)',
                avg_launch_ms=score_ms, launches_per_step=launches / n_prof,
                note='unit = log-sum-exp-pair equivalents: achieved = (LSE pairs + evaluated '
                     'quantized pairs x lse_peak/erf_peak) / launch time; peaks are '
                     'register-only microkernels of exactly the pair arithmetic (LSE pair: 2 '
                     'fp64 FMA + max + v_exp_f32 + fp64 sum, SURVEY 8d "1 exp + 6 flops"; '
                     'quantized pair: 2 OCML fp64 erf + 8 flops)',
                lse_pairs_per_launch=lse_pairs, erf_pairs_per_launch=erf_pairs,
                erf_live_pairs_per_launch=census[1] / per_launch,
                erf_evaluated_pairs_per_launch=erf_exec,
                lse_pair_peak_per_s=lse_peak, erf_pair_peak_per_s=erf_peak,
                fp64_fma_peak_flops=eng.microbench(1), exp_f32_peak_per_s=eng.microbench(0),
                erf_f64_peak_per_s=eng.microbench(2))

    if lat_launches and args.config == "cfg2":
        roof['lattice'] = dict(
            kernel='k_lattice (bounded quantized hps: every lattice value j*q scored once per '
                   'suggest call, candidates look their lpdfs up in k_score; bit-identical; for '
                   'small draws the launch also carries the candidate-draw blocks, timed with it)',
            avg_launch_ms=lat_ms, launches_per_step=lat_launches / n_prof,
            pairs_per_launch=lat_pairs,
            erf_pair_rate_per_s=lat_pairs / (lat_ms * 1e-3) if lat_ms else None,
            frac_of_erf_pair_peak=(lat_pairs / (lat_ms * 1e-3)) / erf_peak if lat_ms else None)
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        n_cpu = {'cfg2': n_cand, 'cfg3': 4096, 'cfg4': 128, 'cfg5': 4096}[args.config]
        cpu = cpu_baseline(dom, losses, vals, active, n_cpu, args.cpu_seconds)
        if n_cpu != n_cand:
            cpu['sample'] += ' (bounded sample: %d of %d candidates per suggest)' % (n_cpu, n_cand)

    line = {
        'metric': 'EI candidates scored/sec (x components)',
        'value': value,
        'unit': 'pairs/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': 1e3 * elapsed / args.steps,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f64',
        'data': 'synthetic (rand.suggest startup history, RandomState(2) losses)',
        'config': {
            'workload': {'cfg2': 'config 2: 20-D mixed space, 1000-trial history, 4096 '
                                 'candidates/suggest', 'cfg3': 'config 3: 50-hp conditional, '
                                 '1e4 history, 1e5 candidates', 'cfg4': 'config 4: 100-D, 1e4 '
                                 'history, 1e7 candidates',
                         'cfg5': 'config 5: batched asynchronous suggestions x 1e6 candidates '
                                 '(config 2 space + 1000-trial history), %d suggestions per GPU '
                                 'per step' % batch}[args.config],
            'suggestions_per_step_per_gpu': batch,
            'candidates_per_suggest': n_cand,
            'pairs_per_step': pairs_step,
            'pairs_per_suggest': pairs_step / batch,
            'suggest_latency_ms': 1e3 * elapsed / args.steps / batch,
            'parallelism': 'replicas' if world > 1 else 'single',
        },
        'roofline': roof,
        'per_candidate_quantized': no_lat,
        'cpu_baseline': cpu,
    }
    print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
