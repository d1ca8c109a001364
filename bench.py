#!/usr/bin/env python3
"""bench.py -- TPE candidate-scoring throughput of the MI355X engine.

Metric (BASELINE.json): "EI candidates scored/sec (x components) +
tpe.suggest latency".  ``value`` = (candidate, mixture-component) lpdf pairs
of the whole job per second: for every active hyperparameter, candidates x
(K_below + K_above), the work the reference's GMM1_lpdf / LGMM1_lpdf calls do
(tpe.py:104-166, 259-301).  This is a reference-equivalent rate: pairs the
engine skips are credited (their lpdf is produced) but not evaluated --
log-sum-exp component blocks whose terms are bounded-negligible (each below
2^-(27 + log2 K) of the candidate's largest term, <= 2^-26 relative on the
lpdf), quantized terms that are exact zeros (both erf saturated), and
candidates that read their lpdf off a value lattice.
``evaluated_pairs_per_s`` reports the pairs actually computed, side by side
with ``evaluated_fraction``.

One *step* = one whole device-side ``tpe.suggest`` posterior pass over the
config's synthetic history, resident in HBM: good/bad split, both Parzen fits
of every hyperparameter, Philox candidate draws, below/above lpdf of every
candidate, EI argmax.  Default workload: config 4 (BASELINE configs[3],
100-D uniform space, 1e4-trial history, 1e7 candidates per hyperparameter),
the largest single-GPU config.  --config cfg2 / cfg3 / cfg5 select the others.

Multi-GPU (one process per GPU; ``--gpus N`` without torchrun re-launches
itself under torch.distributed.run before touching a GPU):
* cfg4: the suggestion's candidates are sharded over ranks
  (parallel.ShardedSuggest: per level an RCCL all-gather of 32-B records and
  the device max-loc merge) -- strong scaling, fixed work per step;
* cfg5: the batch of 1024 suggestions is split over ranks, no exchange --
  strong scaling;
* cfg2 / cfg3: each rank serves its own suggestion (replicas) -- weak.

Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

CONFIGS = {
    'cfg2': dict(n_cand=4096, batch=1, mode='replicas',
                 desc='config 2: 20-D mixed space (uniform/loguniform/quniform/choice), '
                      '1000-trial history, 4096 candidates/suggest'),
    'cfg3': dict(n_cand=100_000, batch=1, mode='replicas',
                 desc='config 3: 50-hp conditional space (nested choice, LGMM1 + '
                      'categorical), 1e4-trial history, 1e5 candidates/suggest'),
    'cfg4': dict(n_cand=10_000_000, batch=1, mode='sharded',
                 desc='config 4: 100-D uniform space, 1e4-trial history, 1e7 '
                      'candidates/suggest (lpdf roofline stress)'),
    'cfg5': dict(n_cand=1_000_000, batch=1024, mode='batch',
                 desc='config 5: 1024 batched asynchronous suggestions x 1e6 candidates '
                      '(config 2 space + 1000-trial history)'),
}


# ----------------------------------------------------------------------------
# workloads (host only)
# ----------------------------------------------------------------------------
def build_workload(cfg):
    """(domain, losses, vals[P, n], active[P, n])."""
    import spaces
    import big_configs
    from hyperopt_amd import hp, rand, Trials
    from hyperopt_amd.base import Domain
    from hyperopt_amd.tpe import build_history
    if cfg == 'cfg4':
        return big_configs.cfg4_domain_history(hp, Domain)
    if cfg == 'cfg3':
        dom, t = big_configs.cfg3_trials(hp, Domain, Trials, rand)
    else:
        dom = Domain(lambda x: 0.0, spaces.cfg2_space(hp))
        t = Trials()
        docs = rand.suggest(list(range(1000)), dom, t, 1)
        for d, l in zip(docs, np.random.RandomState(2).rand(1000)):
            d['state'] = 2
            d['result'] = {'status': 'ok', 'loss': float(l)}
        t._insert_trial_docs(docs)
        t.refresh()
    _, losses, vals, active = build_history(dom, t, dom.space.labels)
    return dom, losses, vals, active


# ----------------------------------------------------------------------------
# CPU baseline: the oracle (numpy restatement pinned to the reference)
# ----------------------------------------------------------------------------
_CPU_CAND = {'cfg2': 4096, 'cfg3': 4096, 'cfg4': 128, 'cfg5': 4096}


def _cpu_worker(args):
    """Whole oracle suggests of the config's own space and history for
    ``budget`` seconds (one process, one thread); returns (pairs, seconds,
    suggests)."""
    cfg, seed0, budget = args
    os.environ['OPENBLAS_NUM_THREADS'] = '1'
    from oracle import tpe_oracle as O
    dom, losses, vals, active = build_workload('cfg2' if cfg == 'cfg5' else cfg)
    cs = dom.space
    hps = {h.label: dict(dist=h.dist, args=h.args, paths=[tuple(p) for p in h.paths])
           for h in cs.hps}
    tids = np.arange(losses.size)
    obs = {h.label: (tids[active[h.index] == 1], vals[h.index][active[h.index] == 1])
           for h in cs.hps}
    n_c = _CPU_CAND[cfg]
    runs, busy, pairs = 0, 0.0, 0.0
    with np.errstate(all='ignore'):
        while busy < budget or runs == 0:
            t0 = time.perf_counter()
            _, det = O.suggest_reference_stream(hps, tids, losses, obs, seed0 + runs, n_ei=n_c)
            busy += time.perf_counter() - t0
            runs += 1
            for lab, dd in det.items():
                if cs.by_label[lab].is_categorical or len(dd['cand']) == 0:
                    continue
                pairs += len(dd['cand']) * (len(dd['below'][0]) + len(dd['above'][0]))
    return pairs, busy, runs


def cpu_baseline(cfg, n_cand, budget_s, cores):
    """One core, then ``cores`` processes at once (independent suggests);
    runs before any GPU call (spawned workers)."""
    import multiprocessing as mp
    one = _cpu_worker((cfg, 7, budget_s))
    agg = None
    if cores > 1:
        ctx = mp.get_context('spawn')
        t0 = time.perf_counter()
        with ctx.Pool(cores) as pool:
            res = pool.map(_cpu_worker, [(cfg, 1000 * (i + 1), budget_s) for i in range(cores)])
        wall = time.perf_counter() - t0
        # aggregate over the span every worker was computing (startup excluded)
        span = max(r[1] for r in res)
        agg = dict(pairs_per_s=sum(r[0] for r in res) / span, wall_s=wall,
                   suggests=sum(r[2] for r in res))
    n_c = _CPU_CAND[cfg]
    sample = ('%d whole oracle suggests of this config\'s space and history (%d candidates '
              'each%s); oracle = numpy/scipy float64 restatement of tpe.py, bit-equal to the '
              'reference on the committed fixtures' % (
                  one[2], n_c, '' if n_c == n_cand else ', a bounded sample of the %d' % n_cand))
    out = dict(unit='pairs/s', kind='port', single_core=dict(value=one[0] / one[1], cores=1,
                                                               suggest_s=one[1] / one[2]))
    if agg is not None:
        out.update(value=agg['pairs_per_s'], cores=cores,
                   sample=sample + '; %d single-thread processes at once, %.0f s each, %d '
                   'suggests in total' % (cores, budget_s, agg['suggests']))
    else:
        out.update(value=one[0] / one[1], cores=1, sample=sample)
    return out


def host_cores():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))      # the GPU box's CPU share is 16


# ----------------------------------------------------------------------------
# end-to-end tpe.suggest latency (host call -> returned trial document)
# ----------------------------------------------------------------------------
def e2e_latency(cfg, n_calls):
    """tpe.suggest through a real Trials in an fmin-like loop: each call sees
    one more finished trial (incremental columnar history + one engine
    call); returns median / p90 ms and the host share."""
    import spaces
    import big_configs
    from hyperopt_amd import hp, rand, tpe, Trials
    from hyperopt_amd.base import Domain
    if cfg == 'cfg3':
        dom, t = big_configs.cfg3_trials(hp, Domain, Trials, rand)
        n_c = CONFIGS['cfg3']['n_cand']
    else:
        dom = Domain(lambda x: 0.0, spaces.cfg2_space(hp))
        t = Trials()
        docs = rand.suggest(list(range(1000)), dom, t, 1)
        for d, l in zip(docs, np.random.RandomState(2).rand(1000)):
            d['state'] = 2
            d['result'] = {'status': 'ok', 'loss': float(l)}
        t._insert_trial_docs(docs)
        t.refresh()
        n_c = CONFIGS['cfg2']['n_cand']
    rng = np.random.RandomState(5)
    tpe.suggest(t.new_trial_ids(1), dom, t, 1, n_EI_candidates=n_c)   # builds plan + mirror
    st = dom._tpe_state
    lat, host = [], []
    for i in range(n_calls):
        ids = t.new_trial_ids(1)
        # the call's history work (sync of the new trial + its row upload),
        # done here so it can be timed apart; the suggest below then finds
        # nothing new
        t0 = time.perf_counter()
        h = st.histories[t].sync(t)
        h.push(st.plan_for(dom, h.n, st.plan.engine))   # (grows the plan as tpe.suggest does)
        t1 = time.perf_counter()
        docs = tpe.suggest(ids, dom, t, 100 + i, n_EI_candidates=n_c)
        t2 = time.perf_counter()
        lat.append(t2 - t0)
        host.append(t1 - t0)
        t.insert_trial_docs(docs)
        t.refresh()
        t.trials[-1]['result'] = {'status': 'ok', 'loss': float(rng.rand())}
        t.trials[-1]['state'] = 2
    lat = 1e3 * np.asarray(lat)
    return dict(tpe_suggest_ms_median=float(np.median(lat)),
                tpe_suggest_ms_p90=float(np.percentile(lat, 90)),
                history_sync_push_ms_median=float(1e3 * np.median(host)),
                calls=n_calls, candidates=n_c, history=len(t.trials) - n_calls,
                note='hyperopt_amd.tpe.suggest on a real Trials, host call to returned doc, '
                     'one new finished trial between calls (tpe.py:804-897 boundary, '
                     'fmin.py:155-156)')


def e2e_cfg1(reps=3):
    """BASELINE configs[0]: fmin(lambda x: (x - 3) ** 2, hp.uniform('x', -5, 5),
    algo=tpe.suggest, max_evals=100, n_EI_candidates=24) -- the whole fmin
    (20 startup draws + 80 TPE suggests) on this framework, and the time of
    each tpe.suggest call (host call -> returned doc).  The first fmin builds
    the plan (cold); the others reuse nothing but the process."""
    from hyperopt_amd import hp, tpe, fmin, Trials
    tpe_s = []

    def algo(new_ids, domain, trials, seed):
        t0 = time.perf_counter()
        out = tpe.suggest(new_ids, domain, trials, seed)
        if len(trials.trials) >= 20:          # a TPE call (not the startup fallback)
            tpe_s.append(time.perf_counter() - t0)
        return out

    runs = []
    best = None
    for r in range(reps + 1):
        t = Trials()
        del tpe_s[:]
        t0 = time.perf_counter()
        best = fmin(lambda x: (x - 3) ** 2, hp.uniform('x', -5, 5), algo=algo, max_evals=100,
                    trials=t, rstate=np.random.RandomState(r))
        runs.append((time.perf_counter() - t0, 1e6 * np.median(tpe_s), len(tpe_s)))
    warm = runs[1:]
    return dict(fmin_s_median=float(np.median([w[0] for w in warm])), fmin_s_cold=runs[0][0],
                tpe_suggest_us_median=float(np.median([w[1] for w in warm])),
                tpe_calls_per_fmin=warm[0][2], best_x_last=float(best['x']),
                note='config 1 (BASELINE configs[0]): 100-eval fmin of (x-3)^2, '
                     'n_EI_candidates=24; warm fmins of a fresh Trials each')


def cpu_cfg1(reps=3):
    """The same fmin with the oracle as ``algo`` (the reference's tpe.suggest
    numerics restated in numpy; tests/oracle_algo.py): the CPU path the
    reference runs for config 1 (0.093 s in the survey
    container)."""
    from hyperopt_amd import hp, fmin, Trials
    from oracle_algo import oracle_suggest
    out = []
    for r in range(reps):
        t0 = time.perf_counter()
        fmin(lambda x: (x - 3) ** 2, hp.uniform('x', -5, 5), algo=oracle_suggest,
             max_evals=100, trials=Trials(), rstate=np.random.RandomState(r))
        out.append(time.perf_counter() - t0)
    return dict(fmin_s_median=float(np.median(out)), cores=1, kind='port',
                sample='%d 100-eval fmins, oracle algo (reference numerics), 1 thread' % reps)


# ----------------------------------------------------------------------------
class _StdoutToStderr(object):
    """fd-level redirect of stdout to stderr (RCCL prints its version banner
    on stdout when a communicator comes up; the bench's stdout is one JSON
    line)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _launch_ranks(n):
    """Re-launch under torch.distributed.run (child process; no GPU touched yet)."""
    port = _free_port()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node=%d' % n, '--master-addr=127.0.0.1', '--master-port=%d' % port,
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--config', default='cfg4', choices=sorted(CONFIGS))
    ap.add_argument('--batch', type=int, default=32,
                    help='cfg5: suggestions per engine call')
    ap.add_argument('--n-cand', type=int, default=0,
                    help='override candidates per suggest (secondary measurements only)')
    ap.add_argument('--cpu-seconds', type=float, default=10.0)
    ap.add_argument('--prune', type=int, default=3, choices=[0, 1, 2, 3],
                    help='log-sum-exp prune mode of large draws (tpe_plan_set_prune; A/B)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-e2e', action='store_true')
    ap.add_argument('--parallelism', default='auto', choices=['auto', 'single', 'sharded'],
                    help="auto: the config's multi-GPU mode when N > 1; 'sharded' forces the "
                         "candidate-sharded path (RCCL all-gather + device merge) even at N = 1")
    ap.add_argument('--traffic-json', default=os.path.join(ROOT, 'traffic.json'))
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        sys.exit(_launch_ranks(args.gpus))
    if world != args.gpus:
        print('bench.py: --gpus %d but WORLD_SIZE=%d' % (args.gpus, world), file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    C = CONFIGS[args.config]
    n_cand = args.n_cand or C['n_cand']

    # CPU baseline first (rank 0, N = 1): host processes only, before any GPU call
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(args.config, n_cand, args.cpu_seconds, host_cores())
        if not args.no_e2e:
            cpu['cfg1'] = cpu_cfg1()

    import torch
    torch.cuda.set_device(local)
    if args.parallelism == 'sharded':
        C = dict(C, mode='sharded')
    dist = None
    if world > 1 or args.parallelism == 'sharded':
        import torch.distributed as dist
        if 'MASTER_ADDR' not in os.environ:     # a one-rank group for --parallelism sharded
            os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_free_port()),
                              RANK='0', WORLD_SIZE='1')
        with _StdoutToStderr():
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
            dist.barrier()          # brings the communicator up (and its banner)
            torch.cuda.synchronize()

    from hyperopt_amd import _engine as E
    from hyperopt_amd import parallel, tpe
    eng = E.default_engine(local)
    dom, losses, vals, active = build_workload(args.config)
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(eng, hps, conds, pprior, max_trials=losses.size)
    plan.set_prune(args.prune)
    # history resident in HBM before the timed region
    d_losses = torch.from_numpy(np.ascontiguousarray(losses)).cuda()
    d_vals = torch.from_numpy(np.ascontiguousarray(vals)).cuda()
    d_act = torch.from_numpy(np.ascontiguousarray(active)).cuda()
    torch.cuda.synchronize()
    plan.set_history_device(d_losses.data_ptr(), d_vals.data_ptr(), d_act.data_ptr(),
                            losses.size)
    plan.engine.synchronize()  # the copies are stream-ordered: done before any fit

    mode = C['mode'] if (world > 1 or args.parallelism == 'sharded') else 'single'
    sharded = parallel.ShardedSuggest(plan) if mode == 'sharded' else None
    if args.config == 'cfg5':
        mine = list(parallel.suggestion_slice(C['batch'], rank, world))
    else:
        mine = [0]

    def step(i):
        if sharded is not None:
            sharded.fit()      # on the sharded stream: ordered before its suggest
            sharded.suggest([7 + 4099 * i], n_cand, fetch=False)
            return
        if args.config == 'cfg5':
            for b0 in range(0, len(mine), args.batch):
                seeds = [1_000_003 * (i + 1) + s for s in mine[b0:b0 + args.batch]]
                plan.fit_suggest(seeds, n_cand, fetch=False)
            return
        plan.fit_suggest([1_000_003 * rank + 4099 * i + 7], n_cand, fetch=False)

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
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    tt = torch.tensor([elapsed], dtype=torch.float64, device='cuda')
    if dist:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = float(tt.item())

    # logical pairs of one suggestion (whole candidate set) from this rank's
    # last engine call: its pairs per candidate x the full candidate count
    _, last_pairs = plan.last_stats()
    per_call_cand = plan_last_cand(plan)
    pairs_suggest = last_pairs / max(1, per_call_cand) * n_cand / max(1, plan._last_nsug)
    if mode == 'replicas':
        sug_step = world
    elif mode == 'batch' or args.config == 'cfg5':
        sug_step = C['batch']
    else:
        sug_step = 1
    pairs_step = pairs_suggest * sug_step
    value = pairs_step * args.steps / elapsed

    # ---- profiled pass (after the timed region): HIP events on the engine
    # stream around every scoring / lattice launch, and the pair census
    n_prof = 1 if args.config in ('cfg4', 'cfg5') else max(1, min(args.steps, 20))
    plan.profile(n_prof * 4096)
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
    plan.census(True)
    for i in range(n_prof):
        step(args.warmup + args.steps + n_prof + i)
    census = plan.census(False, n=12)

    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e:
        e2e = dict(cfg1=e2e_cfg1(), cfg2=e2e_latency('cfg2', 30), cfg3=e2e_latency('cfg3', 10))

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    line = report(args, C, eng, world, mode, elapsed, value, pairs_step, pairs_suggest,
                  sug_step, n_cand, kinds, score_ms, launches, n_prof, lat_ms, lat_launches,
                  lat_pairs, census, cpu, e2e)
    print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


def plan_last_cand(plan):
    """Candidates per suggestion of the plan's last engine call (a shard in
    sharded mode)."""
    return int(getattr(plan, '_last_ncand', 0)) or 1


def report(args, C, eng, world, mode, elapsed, value, pairs_step, pairs_suggest, sug_step,
           n_cand, kinds, score_ms, launches, n_prof, lat_ms, lat_launches, lat_pairs, census,
           cpu, e2e):
    from hyperopt_amd import _engine as E
    # roofline of the dominant kernel, k_score (every lpdf kind of a level
    # in one launch), priced at the measured register-only rate of exactly
    # its pair arithmetic (k_micro): log-sum-exp pairs and evaluated
    # quantized pairs (the per-wave exact-zero skips cost no erf).  LSE pairs
    # are priced at the faster of the two pair sequences k_score has (per
    # group max + lift, or one exponent per wave), whichever each wave ran
    # (one-exponent pairs: fp64 quadratic in prune mode 2, block-local fp32 in 3)
    lse_peak_exact = eng.microbench(3)
    lse_peak_shift = eng.microbench(6 if args.prune == 3 else 5)
    lse_peak_exact32 = eng.microbench(7)   # mode 3's fp32 per-group-lift pair
    lse_peak_mom = eng.microbench(8)       # mode 3's moment form of a 16-component chunk
    lse_peak_mom8 = eng.microbench(9)      # ... of an 8-component block (degree 15)
    lse_peak = max(lse_peak_exact, lse_peak_shift, lse_peak_mom if args.prune == 3 else 0.0)
    erf_peak = eng.microbench(4)
    lse_pairs = kinds.get('lse_gmm', 0.0) + kinds.get('lse_lgmm', 0.0)
    per_launch = max(1, launches)
    lse_exec = census[5] / per_launch if census[3] else lse_pairs
    lse_shift = census[4] / per_launch if census[3] else 0.0   # of which one-exponent form
    lse_exact32 = census[6] / per_launch if census[3] else 0.0  # fp32 per-group-lift form
    lse_mom = census[9] / per_launch if census[3] else 0.0      # of lse_shift: moment form
    lse_mom8 = census[10] / per_launch if census[3] else 0.0    # of lse_mom: the 8-wide form
    lse_momh = census[11] / per_launch if census[3] else 0.0    # of lse_mom: 16-wide degree 15
    erf_exec = census[2] / per_launch
    t_kernel = score_ms * 1e-3
    # each evaluated pair priced at the register-only rate of the arithmetic
    # it ran: per-group-max lift, one wave exponent, or quantized erf
    t_peak = ((lse_exec - lse_shift - lse_exact32) / lse_peak_exact +
              (lse_shift - lse_mom) / lse_peak_shift +
              (lse_mom - lse_mom8 - lse_momh) / lse_peak_mom + lse_mom8 / lse_peak_mom8 +
              lse_momh / (2.0 * lse_peak_mom8) +
              lse_exact32 / lse_peak_exact32 + erf_exec / erf_peak)
    frac = t_peak / t_kernel if t_kernel else None
    achieved = (frac or 0.0) * lse_peak
    # the same launch in literal SURVEY 8(d) units: v_exp_f32 issued (one per
    # evaluated pair, one per moment chunk / block and candidate) against the
    # measured v_exp_f32 peak over the launch time, and VALU instructions
    # (x 64 lanes) per evaluated pair from the committed SQ pass of this config
    exp_peak = eng.microbench(0)
    exp_issued = (lse_exec - lse_mom) + (lse_mom - lse_mom8) / 16.0 + lse_mom8 / 8.0
    exp_issue_frac = exp_issued / (exp_peak * t_kernel) if t_kernel else None
    valu_pp, sq_src = None, None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                sq = json.load(f).get(args.config, {})
            if sq.get('valu_insts_per_launch') and (lse_exec + erf_exec):
                valu_pp = 64.0 * sq['valu_insts_per_launch'] / (lse_exec + erf_exec)
                sq_src = sq.get('_sq_source')
        except Exception:
            valu_pp = None
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                traffic = json.load(f).get(args.config, {}).get('score')
        except Exception:
            traffic = None
    steps_per_launch = launches / n_prof if n_prof else 0
    lat_pairs_step = lat_pairs * (lat_launches / n_prof if n_prof else 0)
    eval_step = (lse_exec + erf_exec) * steps_per_launch + lat_pairs_step
    roof = dict(bound='valu', unit='Gpair/s', achieved=achieved / 1e9, peak=lse_peak / 1e9,
                frac=frac, traffic=traffic,
                kernel='k_score (all lpdf kinds of a level, one launch)',
                avg_launch_ms=score_ms, launches_per_step=steps_per_launch,
                note='frac = (time the evaluated pairs take at the register-only peak of the '
                     'arithmetic each ran: per-group-max LSE pairs, one-wave-exponent LSE pairs, '
                     'quantized erf pairs) / launch time; achieved = frac x peak, in pairs/s of '
                     'the fastest (one-exponent) LSE form; peaks are microkernels of exactly the '
                     'pair arithmetic (LSE pair: 2 fp64 FMA + cvt + v_exp_f32 + fp32/fp64 sum, '
                     'SURVEY 8d "1 exp + 6 flops"; prune mode 3 one-exponent pair: 1 packed '
                     'fp32 FMA pair per 2 components + v_exp_f32 + sums; mode 3 per-group-lift '
                     'pair below the one-exponent size: the same in fp32 with the group max and '
                     'lift; mode 3 moment form of a 16-component equal-sigma chunk: one exp2 + '
                     'a degree-9 packed fp32 polynomial per candidate and chunk, 16 pairs; '
                     '8-wide moment form of a block of 8: the same with a degree-15 polynomial, '
                     '8 pairs (a 16-component chunk in degree 15: the same arithmetic, 16 pairs, '
                     'priced at twice that peak); exp_issue_frac = v_exp_f32 issued / (exp_f32 peak x launch time); '
                     'quantized pair: 2 OCML fp64 erf + 8 flops)',
                lse_evaluated_shifted_pairs_per_launch=lse_shift,
                lse_evaluated_moment_pairs_per_launch=lse_mom,
                lse_evaluated_moment8_pairs_per_launch=lse_mom8,
                lse_evaluated_moment16_deg15_pairs_per_launch=lse_momh,
                lse_pair_moment_peak_per_s=lse_peak_mom,
                lse_pair_moment8_peak_per_s=lse_peak_mom8,
                exp_issue_frac=exp_issue_frac, exp_issued_per_launch=exp_issued,
                valu_per_evaluated_pair=valu_pp,
                valu_per_evaluated_pair_note=('SQ_INSTS_VALU per scoring launch (x 64 lanes) from '
                                              '%s / this run\'s evaluated pairs per launch' % sq_src
                                              if valu_pp else None),
                lse_shifted_retry_pairs_per_launch=census[7] / per_launch,
                lse_shifted_wide_block_pairs_per_launch=census[8] / per_launch,
                lse_evaluated_exact_f32_pairs_per_launch=lse_exact32,
                lse_pair_max_lift_f32_peak_per_s=lse_peak_exact32,
                lse_pairs_per_launch=lse_pairs, lse_evaluated_pairs_per_launch=lse_exec,
                erf_pairs_per_launch=kinds.get('erf_gmm', 0.0) + kinds.get('erf_lgmm', 0.0),
                erf_evaluated_pairs_per_launch=erf_exec,
                lse_pair_peak_per_s=lse_peak, lse_pair_max_lift_peak_per_s=lse_peak_exact,
                lse_pair_wave_exponent_peak_per_s=lse_peak_shift, erf_pair_peak_per_s=erf_peak,
                fp64_fma_peak_flops=eng.microbench(1), exp_f32_peak_per_s=eng.microbench(0),
                erf_f64_peak_per_s=eng.microbench(2))
    if lat_launches:
        roof['lattice'] = dict(
            kernel='k_lattice (bounded quantized hps: every lattice value j*q scored once per '
                   'call; candidates look their lpdfs up in k_score; bit-identical); for small '
                   'draws the launch also carries the candidate-draw rows (k_lattice<true>), '
                   'so its time includes the draw',
            avg_launch_ms=lat_ms, launches_per_step=lat_launches / n_prof,
            pairs_per_launch=lat_pairs)
    ms_step = 1e3 * elapsed / args.steps
    return {
        'metric': 'EI candidates scored/sec (x components)',
        'value': value,
        'unit': 'pairs/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': ms_step,
        'higher_is_better': True,
        'scaling': 'weak' if mode == 'replicas' else 'strong',
        'vs_baseline': None,
        'dtype': ('f64 (log-sum-exp: fp64 accumulation, fp32 exp2 of the shifted term, '
                  'its argument from an fp32 block-local quadratic (mode 3); quantized: fp64 erf)'
                  if args.prune == 3 else
                  'f64 (log-sum-exp: fp64 exponent and accumulation, fp32 exp2 of the '
                  'shifted term; quantized: fp64 erf)'),
        'data': 'synthetic (SURVEY 8(d) histories: RandomState seeds as in tests/big_configs.py)',
        'config': {
            'workload': C['desc'],
            'parallelism': {'single': 'single', 'sharded': 'cand-sharded%d' % world,
                            'batch': 'batch-sharded%d' % world,
                            'replicas': 'replicas%d' % world}[mode],
            'candidates_per_suggest': n_cand,
            'suggestions_per_step': sug_step,
            'pairs_per_step': pairs_step,
            'pairs_per_suggest': pairs_suggest,
            'suggest_latency_ms': ms_step / sug_step if mode != 'replicas' else ms_step,
        },
        # eval_step: this rank's evaluated pairs per step (census per launch x
        # launches per step); every rank does the same share of the job
        'evaluated_pairs_per_s': eval_step * world / (ms_step * 1e-3) if ms_step else None,
        'evaluated_fraction': (eval_step * world / pairs_step) if pairs_step else None,
        'evaluated_pairs_note': 'pairs actually computed per step, all ranks: log-sum-exp pairs '
                                'outside the skipped component blocks (bounded-negligible: every '
                                'skipped term < 2^-(27+log2 K) of the lane maximum, <= 2^-26 '
                                'relative on the lpdf), quantized pairs not skipped as exact '
                                'zeros (both erf saturated), and value-lattice points x '
                                'components; value credits every reference pair',
        'roofline': roof,
        'e2e': e2e,
        'cpu_baseline': cpu,
    }


if __name__ == '__main__':
    main()
