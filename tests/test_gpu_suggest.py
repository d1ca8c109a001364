"""Whole-suggest parity on the GPU: fmin trajectories equal to the reference
(reference RandomState candidate stream, GPU fit + scoring), the reference's
own candidates scored by the GPU plan, and quality/structure of the default
device-Philox path."""
import functools

import numpy as np
import pytest

import hyperopt_amd as H
from hyperopt_amd import hp, tpe, rand, Trials, fmin, trials_from_docs
from hyperopt_amd.base import Domain
from hyperopt_amd.expr import as_apply

from golden_io import load, load_json, unpack
from gpu_util import assert_close, argmax_equiv
import domains
import spaces

pytestmark = pytest.mark.gpu

SPACES = {'cfg2': spaces.cfg2_space, 'many_dists': spaces.many_dists_space,
          'cond': spaces.cond_space, 'cfg3_small': spaces.cfg3_space}


@pytest.mark.parametrize('key', ['0', '123', '123_nei5'])
def test_cfg1_trajectory_equals_reference(key):
    traj = load_json('cfg1_traj.json')[key]
    n_ei = 5 if key.endswith('nei5') else 24
    n = len(traj['xs'])
    algo = functools.partial(tpe.suggest, rng_stream='numpy', n_EI_candidates=n_ei)
    t = Trials()
    best = fmin(lambda x: (x - 3) ** 2, hp.uniform('x', -5, 5), algo=algo, max_evals=n,
                trials=t, rstate=np.random.RandomState(int(key.split('_')[0])))
    xs = [tr['misc']['vals']['x'][0] for tr in t.trials]
    assert xs == traj['xs']
    assert best['x'] == traj['best']


def _fixture_trials(name):
    meta = load_json('suggest_meta.json')[name]
    d = load('suggest_%s.npz' % name)
    dom = Domain(lambda x: 0.0, SPACES[name](hp))
    docs = rand.suggest(list(range(meta['n'])), dom, Trials(), meta['hist_seed'])
    for doc, l in zip(docs, d['losses']):
        doc['state'] = H.JOB_STATE_DONE
        doc['result'] = {'status': 'ok', 'loss': float(l)}
    return meta, d, dom, trials_from_docs(docs)


def _oracle_chosen(name, d, meta, kind):
    from oracle import tpe_oracle as O
    from oracle_algo import oracle_hps
    dom = Domain(lambda x: 0.0, SPACES[name](hp))
    labels = meta['labels']
    tids = np.arange(d['losses'].size)
    obs = {lab: (tids[d['active'][i] == 1], d['vals'][i][d['active'][i] == 1])
           for i, lab in enumerate(labels)}
    with np.errstate(all='ignore'):
        return O.suggest_reference_stream(oracle_hps(dom.space), tids, d['losses'], obs,
                                          meta['suggest_seed'],
                                          n_ei=meta['kw'].get('n_EI_candidates', 24),
                                          kind=kind)


@pytest.mark.parametrize('name', sorted(SPACES))
def test_suggest_numpy_stream_equals_reference(name):
    """Reference RandomState stream, GPU fit + scoring.  Equal to the oracle
    with stable tie order everywhere; equal to the reference itself wherever
    numpy's unstable argsort of tied (quantized) observations does not change
    the Parzen weight/sigma pairing."""
    meta, d, dom, trials = _fixture_trials(name)
    docs = tpe.suggest([meta['new_id']], dom, trials, meta['suggest_seed'], rng_stream='numpy',
                       **meta['kw'])
    vals = docs[0]['misc']['vals']
    stable, _ = _oracle_chosen(name, d, meta, 'stable')
    unstable, _ = _oracle_chosen(name, d, meta, None)
    n_ref = 0
    for i, lab in enumerate(meta['labels']):
        want = [stable[lab]] if lab in stable else []
        assert vals[lab] == want, (lab, vals[lab], want)
        ref = d['chosen'][i]
        if stable.get(lab) == unstable.get(lab):     # tie order irrelevant here
            assert vals[lab] == ([] if np.isnan(ref) else [ref]), (lab, vals[lab], ref)
            n_ref += 1
    assert n_ref >= len(meta['labels']) - 3


@pytest.mark.parametrize('name', sorted(SPACES))
def test_plan_scores_reference_candidates(name):
    """Feed the reference's numpy-sampled candidates (and its history) to the
    GPU plan: lliks within 1e-6 of the reference (of the stable-tie oracle
    for hps whose tied observations numpy pairs differently), argmax
    identical up to 1e-6 EI ties."""
    meta, d, dom, trials = _fixture_trials(name)
    tpe.suggest([meta['new_id']], dom, trials, meta['suggest_seed'], **meta['kw'])
    plan = dom._tpe_state.plan
    cs = dom.space
    _, st = _oracle_chosen(name, d, meta, 'stable')
    _, un = _oracle_chosen(name, d, meta, None)
    from oracle import tpe_oracle as O
    from oracle_algo import oracle_hps
    hps = oracle_hps(cs)
    tids = np.arange(d['losses'].size)
    for k, lab in enumerate(cs.draw_order):
        x = unpack(d, 'samples', k)
        if x.size == 0:
            continue
        lb, la, bi, bs = plan.score_candidates(cs.by_label[lab].index, x)
        i = cs.labels.index(lab)
        o_t, o_v = tids[d['active'][i] == 1], d['vals'][i][d['active'][i] == 1]
        bo, ao = O.split_observations(o_t, o_v, tids, d['losses'], 0.25, kind='stable')
        with np.errstate(all='ignore'):
            r = O.score_hp(hps[lab]['dist'], hps[lab]['args'], bo, ao, 1.0, x, kind='stable')
            ru = O.score_hp(hps[lab]['dist'], hps[lab]['args'], bo, ao, 1.0, x, kind=None)
        assert_close(lb, r['llik_b'], msg='%s/%s below vs oracle' % (name, lab))
        assert_close(la, r['llik_a'], msg='%s/%s above vs oracle' % (name, lab))
        rb, ra = unpack(d, 'llik_b', k), unpack(d, 'llik_a', k)
        if np.array_equal(ru['llik_a'], r['llik_a'], equal_nan=True) and \
                np.array_equal(ru['llik_b'], r['llik_b'], equal_nan=True):
            assert_close(lb, rb, msg='%s/%s below' % (name, lab))
            assert_close(la, ra, msg='%s/%s above' % (name, lab))
        with np.errstate(all='ignore'):
            assert argmax_equiv(r['llik_b'] - r['llik_a'], bi), (name, lab)


@pytest.mark.parametrize('name', domains.NAMES)
def test_testopt_trajectory_equals_reference(name):
    """hyperopt/tests/test_tpe.py:TestOpt replayed with the reference's
    RandomState candidate stream: every trial equals the stable-tie oracle
    run, and equals the reference run itself when no tied-observation
    reordering occurs (7 of the 8 domains)."""
    from oracle_algo import oracle_suggest, trajectory
    ref = load_json('testopt_traj.json')[name]
    kw, n = domains.settings(name)
    t = Trials()
    fmin(lambda x: x, domains.build(name, hp, H.scope, as_apply),
         algo=functools.partial(tpe.suggest, rng_stream='numpy', **kw),
         max_evals=n, trials=t, rstate=np.random.RandomState(123))
    got = trajectory(t)
    o = Trials()
    fmin(lambda x: x, domains.build(name, hp, H.scope, as_apply),
         algo=functools.partial(oracle_suggest, kind='stable', **kw),
         max_evals=n, trials=o, rstate=np.random.RandomState(123))
    want = trajectory(o)
    for i, (g, w) in enumerate(zip(got, want)):
        if g != w:
            # allowed only as an EI near-tie (north star: argmax identical
            # except where the EI gap is below 1e-6): re-run the oracle on
            # the shared history and check the engine's pick is within 1e-6
            _assert_near_tie(name, kw, t, i, g, w)
            break
    else:
        if want == ref['vals']:
            assert got == ref['vals']
    assert min(t.losses()) < domains.THRESH[name]


def _assert_near_tie(name, kw, trials, i, got, want):
    from oracle import tpe_oracle as O
    from oracle_algo import oracle_hps
    from hyperopt_amd.tpe import build_history
    dom = Domain(lambda x: x, domains.build(name, hp, H.scope, as_apply))
    prefix = trials_from_docs([dict(d) for d in trials.trials[:i]], validate=False)
    tids, losses, vals, active = build_history(dom, prefix, dom.space.labels)
    tids = np.asarray(tids)
    obs = {lab: (tids[active[j] == 1], vals[j][active[j] == 1])
           for j, lab in enumerate(dom.space.labels)}
    seed = np.random.RandomState(123)
    for _ in range(i + 1):
        s = seed.randint(2 ** 31 - 1)
    with np.errstate(all='ignore'):
        _, det = O.suggest_reference_stream(oracle_hps(dom.space), tids, losses, obs, s,
                                            n_ei=kw['n_EI_candidates'], gamma=kw['gamma'],
                                            prior_weight=kw['prior_weight'], kind='stable')
    for lab in got:
        if got[lab] == want[lab]:
            continue
        dd = det[lab]
        with np.errstate(all='ignore'):
            score = dd['llik_b'] - dd['llik_a']
        best = np.nanmax(score)
        mine = np.nanmax(np.where(dd['cand'] == got[lab], score, -np.inf))
        assert abs(mine - best) <= 1e-6 * max(1.0, abs(best)), (name, i, lab, mine, best)


@pytest.mark.parametrize('name', domains.NAMES)
def test_testopt_quality_device_philox(name):
    """The reference's quality thresholds with the default on-device Philox
    stream, over 16 fmin seeds: the pass rate must be no worse than the
    reference RandomState stream's on the same seeds minus two runs (at 6
    seeds one stream's 2-run dip is ordinary noise: tools/quality_rates.py
    measured 14/16 vs 15/16 on branin, 15 vs 14 on quadratic1)."""
    kw, n = domains.settings(name)
    rates = {}
    for stream in ('philox', 'numpy'):
        wins = 0
        for seed in range(16):
            t = Trials()
            fmin(lambda x: x, domains.build(name, hp, H.scope, as_apply),
                 algo=functools.partial(tpe.suggest, rng_stream=stream, **kw), max_evals=n,
                 trials=t, rstate=np.random.RandomState(123 + seed))
            assert len(t) == n
            wins += min(t.losses()) < domains.THRESH[name]
        rates[stream] = wins
    assert rates['philox'] >= rates['numpy'] - 2 and rates['philox'] >= 10, rates


def test_philox_suggest_structure_and_determinism():
    meta, d, dom, trials = _fixture_trials('cond')
    a = tpe.suggest([meta['new_id']], dom, trials, 5, n_EI_candidates=256)[0]['misc']['vals']
    b = tpe.suggest([meta['new_id']], dom, trials, 5, n_EI_candidates=256)[0]['misc']['vals']
    c = tpe.suggest([meta['new_id']], dom, trials, 6, n_EI_candidates=256)[0]['misc']['vals']
    assert a == b and a != c
    top = a['top'][0]
    assert isinstance(top, int)
    for lab, v in a.items():
        if lab[:-1] in ('lr', 'units', 'act', 'zz'):
            assert (len(v) == 1) == (int(lab[-1]) == top), (lab, v, top)
    assert len(a['aa']) == 1 and 0 <= a['aa'][0] < 1
    lr = a['lr%d' % top][0]
    assert 1e-4 <= lr <= 1.0
    assert a['units%d' % top][0] == round(a['units%d' % top][0])


def test_candidate_sharding_invariance_and_device_merge():
    """Counter-based draws: any split of [0, n) over devices gives the same
    winner after the max-loc merge (the multi-GPU path, one GPU here)."""
    torch = pytest.importorskip('torch')
    meta, d, dom, trials = _fixture_trials('cfg2')
    tpe.suggest([meta['new_id']], dom, trials, 7, n_EI_candidates=64)
    plan = dom._tpe_state.plan
    n = 4096
    full = plan.suggest([11], n)
    parts = [plan.suggest([11], 1000, cand_begin=0), plan.suggest([11], 3096, cand_begin=1000)]
    gathered = np.stack(parts)                  # [world=2][S=1][P]
    raw = torch.from_numpy(gathered.view(np.uint8).reshape(-1).copy()).cuda()
    merged = plan.merge(raw.data_ptr(), world=2, level=0)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(merged['index'], full['index'])
    np.testing.assert_array_equal(merged['value'], full['value'])
    # in place (out_on_device 2): the merge kernel stores the level's slots
    # into a device buffer that holds the shard's own records -- the same
    # bytes as the copy-out merge
    rec = torch.from_numpy(parts[1].view(np.uint8).reshape(-1).copy()).cuda()
    plan.merge(raw.data_ptr(), world=2, level=0)
    plan.merge(raw.data_ptr(), world=2, level=0, out=rec.data_ptr(), in_place=True)
    torch.cuda.synchronize()
    got = rec.cpu().numpy().view(merged.dtype).reshape(merged.shape)
    np.testing.assert_array_equal(got.view(np.uint8), merged.view(np.uint8))


def test_fit_suggest_graph_replay_matches_eager():
    """tpe_plan_fit_suggest: the first call of a shape runs eagerly, the
    second captures a hipGraph, later ones replay it with the history length
    and seeds patched; every call must equal fit() + suggest() bit for bit,
    across seeds and a growing history."""
    meta, d, dom, trials = _fixture_trials('cfg2')
    tpe.suggest([meta['new_id']], dom, trials, 7, n_EI_candidates=64)
    plan = dom._tpe_state.plan
    from hyperopt_amd.tpe import build_history
    _, losses, vals, active = build_history(dom, trials, dom.space.labels)
    n = losses.size
    for i, (m, seed) in enumerate([(n, 3), (n, 4), (n, 5), (n - 7, 6), (n - 7, 3), (n, 9)]):
        plan.set_history(losses[:m], vals[:, :m], active[:, :m])
        got = plan.fit_suggest([seed], 512)
        plan.fit()
        want = plan.suggest([seed], 512)
        np.testing.assert_array_equal(got.view(np.uint8), want.view(np.uint8), err_msg=str(i))


@pytest.mark.parametrize('name', ['cfg2', 'many_dists', 'cond', 'cfg3_small'])
def test_value_lattice_bitwise_equals_per_candidate(name):
    """Bounded quantized hps scored once per lattice value (k_lattice, the
    default) give the same scores, values and indices, bit for bit, as
    scoring every candidate on its own -- for single and batched suggestions
    and several candidate counts; the lattice launch must actually run."""
    meta, d, dom, trials = _fixture_trials(name)
    tpe.suggest([meta['new_id']], dom, trials, 7, n_EI_candidates=64)
    plan = dom._tpe_state.plan
    ran = 0
    for seeds, n in [([3], 4096), ([4, 5, 6], 2048), ([8], 20000), ([9], 300)]:
        plan.set_lattice(True)
        plan.profile(16)
        got = plan.suggest(seeds, n)
        ran += plan.profile_read(5)[1]
        plan.profile(0)
        plan.set_lattice(False)
        want = plan.suggest(seeds, n)
        np.testing.assert_array_equal(got.view(np.uint8), want.view(np.uint8),
                                      err_msg='%s %s %d' % (name, seeds, n))
    plan.set_lattice(True)
    has_q = any(h.dist in ('quniform', 'qloguniform') for h in dom.space.hps)
    assert (ran > 0) == has_q, (ran, has_q)


@pytest.mark.parametrize('name', ['cfg2', 'many_dists', 'cond', 'cfg3_small'])
def test_fit_suggest_matches_fit_then_suggest(name):
    """tpe_plan_fit_suggest (one engine call) equals fit() + suggest() bit for
    bit on every test space, for single and batched suggestions (up to the 8
    inline seeds) and candidate counts from n_EI=24 to beyond 8192; on
    config 2 also a sorted draw on one-row wave tiles (2^18 candidates, the
    config-3 regime), where both paths read the moment table the fit wrote
    (mom_width: the same table whichever entry point fitted)."""
    meta, d, dom, trials = _fixture_trials(name)
    tpe.suggest([meta['new_id']], dom, trials, 7, n_EI_candidates=64)
    plan = dom._tpe_state.plan
    shapes = [([3], 24), ([4], 4096), ([5, 6, 7], 2000), ([8], 8192), ([9], 8193),
              ([1, 2, 3, 4, 5, 6, 7, 8], 1024)]
    if name == 'cfg2':
        shapes.append(([10], 1 << 18))
    for seeds, n in shapes:
        got = plan.fit_suggest(seeds, n)
        plan.fit()
        want = plan.suggest(seeds, n)
        np.testing.assert_array_equal(got.view(np.uint8), want.view(np.uint8),
                                      err_msg='%s %s %d' % (name, seeds, n))


def test_large_draw_grid_stride_matches_one_per_thread():
    """Large draws (>= 2^22 per launch) come out of k_draw_sorted and score
    on pruned wave tiles; small ones are drawn one per thread and scored
    unpruned on 8-wave tiles.  Candidates are counter-based, so a 2^18-
    candidate suggest equals the merge of two small-draw chunks: the same
    winners, or (the two tile shapes sum in different orders, and the large
    one skips negligible blocks) ties within the scoring tolerance."""
    from gpu_util import assert_winners_match
    torch = pytest.importorskip('torch')
    meta, d, dom, trials = _fixture_trials('cfg2')
    tpe.suggest([meta['new_id']], dom, trials, 7, n_EI_candidates=64)
    plan = dom._tpe_state.plan
    n, cut = 1 << 18, 100_000
    assert n * len(dom.space.labels) >= 1 << 22 and (n - cut) * len(dom.space.labels) < 1 << 22
    full = plan.suggest([13], n)
    parts = [plan.suggest([13], cut, cand_begin=0), plan.suggest([13], n - cut, cand_begin=cut)]
    raw = torch.from_numpy(np.stack(parts).view(np.uint8).reshape(-1).copy()).cuda()
    merged = plan.merge(raw.data_ptr(), world=2, level=0)
    torch.cuda.synchronize()
    # (near the top of 2^18 candidates many EI values lie within the
    # scoring error of each other: swaps are ties, their scores checked)
    assert_winners_match(merged, full, msg='sorted large draw vs small-draw chunks')


def test_graph_replay_in_child_process():
    """The opt-in hipGraph replay (TPE_GRAPH=1, read once per process) with the
    per-call seed patches of the draw nodes -- k_draw, or k_lattice's fused
    draw rows -- equals eager fit() + suggest(), in a child process."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, 'tests'); import test_gpu_suggest as t; "
            "t.test_fit_suggest_graph_replay_matches_eager(); "
            "[t.test_fit_suggest_matches_fit_then_suggest(n) for n in ('cfg2', 'cond')]; print('OK')")
    r = subprocess.run([sys.executable, '-c', code], cwd=root, env=dict(os.environ, TPE_GRAPH='1'),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and 'OK' in r.stdout, (r.stdout[-1000:], r.stderr[-3000:])


def test_batched_suggest_equals_single_seed_suggests():
    """Config 5's path: one batched fit_suggest over S seeds equals S
    single-seed calls bit for bit (suggestion s reads only its own seed), on
    a conditional and a mixed space, for S beyond the 8 inline seeds."""
    for name in ('cfg2', 'cond'):
        meta, d, dom, trials = _fixture_trials(name)
        tpe.suggest([meta['new_id']], dom, trials, 7, n_EI_candidates=64)
        plan = dom._tpe_state.plan
        seeds = tpe.batch_seeds(1234, 11)
        for n in (300, 4096):
            got = plan.fit_suggest(seeds, n)
            for s, sd in enumerate(seeds):
                one = plan.fit_suggest([sd], n)[0]
                np.testing.assert_array_equal(got[s].view(np.uint8), one.view(np.uint8),
                                              err_msg='%s s=%d n=%d' % (name, s, n))


def test_tpe_suggest_batch_of_ids_matches_single_calls():
    """tpe.suggest with several new ids = one engine call; each returned doc
    equals the single-id suggest with that suggestion's batch seed."""
    meta, d, dom, trials = _fixture_trials('cond')
    ids = [meta['new_id'] + i for i in range(5)]
    docs = tpe.suggest(ids, dom, trials, 99, n_EI_candidates=512)
    assert [x['tid'] for x in docs] == ids
    for i, sd in enumerate(tpe.batch_seeds(99, 5)):
        one = tpe.suggest([ids[i]], dom, trials, sd, n_EI_candidates=512)[0]
        assert docs[i]['misc']['vals'] == one['misc']['vals'], i


def test_incremental_device_history_equals_fresh_upload():
    """An fmin run grows the device history row by row (columnar store +
    tpe_plan_update_history); a fresh plan loaded from scratch with the final
    trials must give the same suggestion bit for bit."""
    t = Trials()
    algo = functools.partial(tpe.suggest, n_EI_candidates=256, n_startup_jobs=10)
    space = spaces.cond_space(hp)
    fmin(lambda x: float(np.sin(3 * x['aa'])), space, algo=algo, max_evals=60, trials=t,
         rstate=np.random.RandomState(3))
    dom = Domain(lambda x: 0.0, space)
    a = tpe.suggest([1000], dom, t, 5, n_EI_candidates=256, n_startup_jobs=10)[0]
    hist = dom._tpe_state.histories[t]
    assert hist.n == 60
    for k in range(3):     # incremental steps on the same plan
        (nid,) = t.new_trial_ids(1)
        t.insert_trial_docs(tpe.suggest([nid], dom, t, 11 + k, n_EI_candidates=256,
                                        n_startup_jobs=10))
        t.refresh()
        t.trials[-1]['result'] = {'status': 'ok', 'loss': float(k) - 5.0}
        t.trials[-1]['state'] = H.JOB_STATE_DONE
    inc = tpe.suggest([2000], dom, t, 5, n_EI_candidates=256, n_startup_jobs=10)[0]
    fresh_dom = Domain(lambda x: 0.0, space)
    ref = tpe.suggest([2000], fresh_dom, t, 5, n_EI_candidates=256, n_startup_jobs=10)[0]
    assert inc['misc']['vals'] == ref['misc']['vals']
    assert a['misc']['vals'] != {} and dom._tpe_state.histories[t].n == 63


def test_thread_trials_async_batched_tpe():
    """Asynchronous workers + batched TPE suggestions (max_queue_len > 1):
    completes, every trial evaluated once, reaches the quadratic's optimum."""
    t = H.ThreadTrials(n_workers=4)
    try:
        fmin(lambda x: (x - 3) ** 2, hp.uniform('x', -5, 5),
             algo=functools.partial(tpe.suggest, n_EI_candidates=1024), max_evals=120,
             trials=t, rstate=np.random.RandomState(1), max_queue_len=4)
    finally:
        t.shutdown()
    assert len(t) == 120
    assert all(d['state'] == H.JOB_STATE_DONE for d in t.trials)
    assert min(t.losses()) < 1e-2


@pytest.mark.parametrize('name', ['cfg2', 'cond'])
def test_pruned_lse_equals_full_evaluation(name):
    """Large draws (>= 4M candidate draws) are value-bucketed by the draw and
    log-sum-exp tiles skip the component blocks whose terms are all below
    2^-(27 + log2 K) of every candidate's largest (mode 1): scores agree
    with the unpruned run within 2^-26 relative per lpdf, winners equal up to
    ties within that.  Modes 2 and 3 (default) also give each wave one exponent (fp64 /
    block-local fp32 quadratic): scores within the north-star 1e-6, winners
    equal up to ties within it.  The winner also
    equals the merge of two differently tiled shards."""
    torch = pytest.importorskip('torch')
    from gpu_util import assert_winners_match
    meta, d, dom, trials = _fixture_trials(name)
    tpe.suggest([meta['new_id']], dom, trials, 7, n_EI_candidates=64)
    plan = dom._tpe_state.plan
    n = 1 << 18 if name == 'cfg2' else 1 << 20
    plan.set_prune(1)
    plan.census(True)
    got = plan.suggest([21, 22], n)
    c = plan.census(False)
    plan.set_prune(2)
    shifted64 = plan.suggest([21, 22], n)
    plan.set_prune(3)
    shifted = plan.suggest([21, 22], n)
    plan.set_prune(0)
    want = plan.suggest([21, 22], n)
    plan.set_prune(3)
    assert_winners_match(got, want, rtol=2.0 ** -25, msg='block skip (mode 1)')
    assert_winners_match(shifted64, want, msg='one exponent per wave')
    assert_winners_match(shifted, want, msg='one exponent per wave, block-local fp32')
    assert c[3] > 0 and c[5] < c[3], c          # blocks were skipped
    if name != 'cfg2':
        return                                   # one level: shards merge directly
    cut = 77_777
    parts = [plan.suggest([21], cut, cand_begin=0), plan.suggest([21], n - cut, cand_begin=cut)]
    raw = torch.from_numpy(np.stack(parts).view(np.uint8).reshape(-1).copy()).cuda()
    merged = plan.merge(raw.data_ptr(), world=2, level=0)
    torch.cuda.synchronize()
    assert_winners_match(merged[0], shifted[0], msg='shard merge')


def test_graph_replay_across_fused_draw_threshold():
    """a graph captured while n_below + 1 <= 32 (lattice launch
    carrying the draw rows, 32-entry tables) must not be replayed once n_below
    reaches 32 (gamma_cap = 64): the step key includes the fused-draw choice.
    Child process with TPE_GRAPH=1; every call equals eager fit + suggest."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, 'tests'); import test_gpu_suggest as t; "
            "t._graph_threshold_body(); print('OK')")
    r = subprocess.run([sys.executable, '-c', code], cwd=root, env=dict(os.environ, TPE_GRAPH='1'),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and 'OK' in r.stdout, (r.stdout[-1000:], r.stderr[-3000:])


def _graph_threshold_body():
    meta, d, dom, trials = _fixture_trials('cfg2')
    tpe.suggest([meta['new_id']], dom, trials, 7, n_EI_candidates=64)
    plan = dom._tpe_state.plan
    from hyperopt_amd.tpe import build_history
    _, losses, vals, active = build_history(dom, trials, dom.space.labels)
    # n_below = min(ceil(0.25 sqrt(n)), 64): 500 -> 6, 16000 would be 32;
    # with gamma 1.0: n = 900 -> 30 (fused), n = 1000 -> 32 (not fused)
    for i, (m, seed) in enumerate([(900, 3), (900, 4), (900, 5), (1000, 6), (1000, 7),
                                   (900, 8), (1000, 9)]):
        plan.set_history(losses[:m], vals[:, :m], active[:, :m])
        got = plan.fit_suggest([seed], 512, gamma=1.0, gamma_cap=64)
        plan.fit(gamma=1.0, gamma_cap=64)
        want = plan.suggest([seed], 512)
        assert np.isfinite(got['value'][got['active'] == 1]).all(), i
        np.testing.assert_array_equal(got.view(np.uint8), want.view(np.uint8), err_msg=str(i))


def test_sorted_draw_suggest_is_reproducible():
    """Large draws come out value-bucketed with a stable (thread-timing
    independent) scatter, so the pruned wave tiles see the same candidate
    windows every run: the same suggest twice is identical bit for bit."""
    meta, d, dom, trials = _fixture_trials('cfg2')
    tpe.suggest([meta['new_id']], dom, trials, 7, n_EI_candidates=64)
    plan = dom._tpe_state.plan
    n = 1 << 18                       # 2^18 x 20 hps: the sorted-draw path
    a = plan.suggest([31, 32], n)
    b = plan.suggest([31, 32], n)
    np.testing.assert_array_equal(a.view(np.uint8), b.view(np.uint8))


def test_small_draw_pruning_in_child_process():
    """Opt-in bucketing + block skip of small-draw log-sum-exp slots
    (TPE_SMALL_SORT=1, read once per process): batched suggestions equal the
    single-seed ones bit for bit, and the winners equal the default path's up
    to near-ties (the skip moves an lpdf by <= 2^-26 relative)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, numpy as np; sys.path.insert(0, 'tests'); import test_gpu_suggest as t; "
            "t.test_batched_suggest_equals_single_seed_suggests(); "
            "meta, d, dom, trials = t._fixture_trials('cfg2'); "
            "t.tpe.suggest([meta['new_id']], dom, trials, 7, n_EI_candidates=64); "
            "r = dom._tpe_state.plan.suggest([5, 6], 8192); "
            "np.save(sys.argv[1], r); print('OK')")
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        out = [os.path.join(td, 'on.npy'), os.path.join(td, 'off.npy')]
        for path, flag in zip(out, ('1', '0')):
            r = subprocess.run([sys.executable, '-c', code, path], cwd=root,
                               env=dict(os.environ, TPE_SMALL_SORT=flag),
                               capture_output=True, text=True, timeout=300)
            assert r.returncode == 0 and 'OK' in r.stdout, (r.stdout[-1000:], r.stderr[-3000:])
        on, off = np.load(out[0]), np.load(out[1])
    from gpu_util import assert_winners_match
    assert_winners_match(on, off, msg='small-draw pruning')


def test_deferred_history_patch_identical():
    """Small history updates (a few appended trials: tpe_plan_update_history's
    kernel-argument patch) are deferred into the next fit, whose blocks write
    them before reading the history; two of them in a row (the first goes out
    on its own), then fit+suggest, equal a plan given the whole history at
    once -- byte for byte; a plain fit and a mixture read after a deferred
    update see it too."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from hyperopt_amd import _engine as E
    dom, losses, vals, act = bench.build_workload('cfg2')
    hps, conds, pprior = dom.space.engine_tables()
    n = losses.size
    vals = np.ascontiguousarray(vals, dtype=np.float64)
    act = np.ascontiguousarray(act, dtype=np.uint8)
    eng = E.default_engine()
    full = E.Plan(eng, hps, conds, pprior, max_trials=n)
    full.set_history(losses, vals, act)
    ref = full.fit_suggest([11, 12], 4096)
    part = E.Plan(eng, hps, conds, pprior, max_trials=n)
    m = n - 3
    part.set_history(losses[:m], np.ascontiguousarray(vals[:, :m]), np.ascontiguousarray(act[:, :m]))
    part.fit_suggest([5], 4096)
    part.update_history(n - 1, m, vals, act, n, m, losses)   # two rows (deferred)
    part.update_history(n, n - 1, vals, act, n, n - 1, losses)  # one more (the first flushes)
    got = part.fit_suggest([11, 12], 4096)
    np.testing.assert_array_equal(got.view(np.uint8), ref.view(np.uint8))
    # plain fit after a deferred update: the fitted mixtures match
    part2 = E.Plan(eng, hps, conds, pprior, max_trials=n)
    part2.set_history(losses[:m], np.ascontiguousarray(vals[:, :m]), np.ascontiguousarray(act[:, :m]))
    part2.update_history(n, m, vals, act, n, m, losses)
    part2.fit()
    full.fit()
    for h in range(len(hps)):
        for side in (0, 1):
            a, b = part2.mixture(h, side), full.mixture(h, side)
            for x, y in zip(a, b):
                np.testing.assert_array_equal(x, y)
