"""Generate the golden fixtures in tests/golden/ by running the REFERENCE.

Run in the build container only (the reference never travels to the GPU box):

    oracle/setup_reference.sh /tmp/oracle
    python tests/golden/make_golden.py /tmp/oracle

It imports the mechanically converted reference and
records inputs and outputs of the TPE hot path as plain arrays (npz, no
pickles) plus JSON.  Nothing from the reference's source is stored.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = sys.argv[1] if len(sys.argv) > 1 else '/tmp/oracle'
ONLY = sys.argv[2:]  # optional subset of generator names, e.g. testopt
sys.path.insert(0, REF)
sys.path.insert(0, os.path.dirname(HERE))          # tests/ for spaces.py

import hyperopt                                     # noqa: E402  (reference)
from hyperopt import tpe, rand, hp, Trials, base, fmin   # noqa: E402
from hyperopt.pyll import scope                     # noqa: E402
from hyperopt.pyll import stochastic                # noqa: E402
import spaces                                       # noqa: E402

assert os.path.abspath(os.path.dirname(hyperopt.__file__)).startswith(os.path.abspath(REF))
NONE = np.nan


def pack(d, name, arrays, dtype=np.float64):
    arrays = [np.asarray(a, dtype=dtype).ravel() for a in arrays]
    off = np.zeros(len(arrays) + 1, dtype=np.int64)
    off[1:] = np.cumsum([a.size for a in arrays])
    d[name] = np.concatenate(arrays) if arrays else np.zeros(0, dtype)
    d[name + '_off'] = off


def opt(v):
    return NONE if v is None else float(v)


# ---------------------------------------------------------------- split
def gen_split():
    rng = np.random.RandomState(11)
    d = {}
    cases = []
    for n in (1, 3, 20, 57, 100, 1000, 10000):
        for mode in ('plain', 'ties', 'inf'):
            for gamma in (0.25, 0.05, 1.0):
                tids = np.arange(n) * 2 + 5
                losses = rng.randn(n)
                if mode == 'ties':
                    losses = np.round(losses * 2) / 2
                if mode == 'inf':
                    losses[rng.rand(n) < 0.2] = np.inf
                act = rng.rand(n) < 0.7
                o_tids = tids[act]
                o_vals = rng.uniform(-5, 5, size=o_tids.size)
                below, above = tpe.ap_filter_trials(o_tids, o_vals, tids, losses, gamma)
                cases.append((tids, losses, gamma, o_tids, o_vals, below, above))
    pack(d, 'tids', [c[0] for c in cases], np.int64)
    pack(d, 'losses', [c[1] for c in cases])
    d['gamma'] = np.array([c[2] for c in cases])
    pack(d, 'o_tids', [c[3] for c in cases], np.int64)
    pack(d, 'o_vals', [c[4] for c in cases])
    pack(d, 'below', [c[5] for c in cases])
    pack(d, 'above', [c[6] for c in cases])
    np.savez_compressed(os.path.join(HERE, 'split.npz'), **d)
    print('split cases', len(cases))


# ---------------------------------------------------------------- parzen
def gen_parzen():
    rng = np.random.RandomState(12)
    cases = []
    for n in (0, 1, 2, 3, 10, 24, 25, 26, 27, 100, 1000, 10000):
        for mode in ('plain', 'tied', 'prior_edge'):
            pw = float(rng.choice([1.0, 0.01, 2.5]))
            pm, ps = 0.0, 10.0
            obs = rng.uniform(-5, 5, size=n)
            if mode == 'tied':
                obs = np.round(obs)
            if mode == 'prior_edge' and n:
                obs[0] = pm            # prior mu equal to an observation
                pm, ps = float(obs.max()) + 1.0, 3.0
            w, mu, sig = tpe.adaptive_parzen_normal(obs, pw, pm, ps)
            order = np.argsort(obs) if n >= 2 else np.zeros(0, np.int64)
            cases.append((obs, pw, pm, ps, w, mu, sig, order))
    d = {}
    pack(d, 'obs', [c[0] for c in cases])
    d['prior'] = np.array([[c[1], c[2], c[3]] for c in cases])
    pack(d, 'w', [c[4] for c in cases])
    pack(d, 'mu', [c[5] for c in cases])
    pack(d, 'sigma', [c[6] for c in cases])
    pack(d, 'order', [c[7] for c in cases], np.int64)
    np.savez_compressed(os.path.join(HERE, 'parzen.npz'), **d)
    print('parzen cases', len(cases))


# ---------------------------------------------------------------- lpdf
VARIANTS = [
    # name, sampler, lpdf, low, high, q, obs generator
    ('gmm_unb', 'GMM1', None, None, None),
    ('gmm_bnd', 'GMM1', -5.0, 5.0, None),
    ('gmmq_bnd', 'GMM1', 0.0, 100.0, 1.0),
    ('gmmq_unb', 'GMM1', None, None, 2.0),
    ('gmmq_bnd_half', 'GMM1', 1.01, 10.0, 0.5),
    ('lgmm_bnd', 'LGMM1', np.log(1e-3), np.log(10), None),
    ('lgmm_unb', 'LGMM1', None, None, None),
    ('lgmmq_bnd', 'LGMM1', 0.0, np.log(1024), 1.0),
    ('lgmmq_unb', 'LGMM1', None, None, 0.01),
]


def gen_lpdf():
    rng = np.random.RandomState(13)
    d = {}
    rows = []
    bm, am, cands, lb, la, best, meta = [], [], [], [], [], [], []
    for name, sampler, low, high, q in VARIANTS:
        for (nb, na, nc) in ((2, 10, 24), (8, 992, 4096), (25, 1000, 1000)):
            if low is not None:
                lo_lin, hi_lin = (low, high)
                ps = high - low
                pm = 0.5 * (high + low)
            else:
                pm, ps = (0.0, 2.0) if sampler == 'LGMM1' else (1.0, 5.0)
                lo_lin, hi_lin = pm - 2 * ps, pm + 2 * ps
            ob = rng.uniform(lo_lin, hi_lin, size=nb)
            oa = rng.uniform(lo_lin, hi_lin, size=na)
            if q is not None and sampler == 'GMM1':
                ob, oa = np.round(ob / q) * q, np.round(oa / q) * q
            if q is not None and sampler == 'LGMM1':
                qq = lambda v: np.log(np.maximum(np.round(np.exp(v) / q) * q, max(1e-12, np.exp(low) if low is not None else 1e-12)))
                ob, oa = qq(ob), qq(oa)
            pw = 1.0
            mixb = tpe.adaptive_parzen_normal(ob, pw, pm, ps)
            mixa = tpe.adaptive_parzen_normal(oa, pw, pm, ps)
            srng = np.random.RandomState(1000 + len(rows))
            fn = tpe.GMM1 if sampler == 'GMM1' else tpe.LGMM1
            x = fn(*mixb, low=low, high=high, q=q, rng=srng, size=(nc,))
            x = np.asarray(x, dtype=np.float64)
            # far tail candidates to exercise -inf / NaN paths
            if sampler == 'GMM1':
                tail = np.array([pm + 50 * ps, pm - 50 * ps, pm + 7 * ps])
                if q is not None:
                    tail = np.round(tail / q) * q
            else:
                tail = np.array([np.exp(pm + 30 * ps), np.exp(pm - 30 * ps)])
                if q is not None:
                    tail = np.round(tail / q) * q
            x = np.concatenate([x, tail])
            lpdf = tpe.GMM1_lpdf if sampler == 'GMM1' else tpe.LGMM1_lpdf
            with np.errstate(all='ignore'):
                yb = lpdf(x, *mixb, low=low, high=high, q=q)
                ya = lpdf(x, *mixa, low=low, high=high, q=q)
                bb = tpe.broadcast_best(x, yb, ya)[0]
            best_i = int(np.argmax(yb - ya))
            assert x[best_i] == bb or (np.isnan(x[best_i]) and np.isnan(bb))
            bm.append(np.stack(mixb)); am.append(np.stack(mixa))
            cands.append(x); lb.append(yb); la.append(ya); best.append(best_i)
            meta.append([0 if sampler == 'GMM1' else 1, opt(low), opt(high), opt(q)])
            rows.append(name)
    pack(d, 'mix_b', bm); pack(d, 'mix_a', am)
    pack(d, 'cand', cands); pack(d, 'llik_b', lb); pack(d, 'llik_a', la)
    d['best'] = np.array(best, dtype=np.int64)
    d['meta'] = np.array(meta)
    np.savez_compressed(os.path.join(HERE, 'lpdf.npz'), **d)
    with open(os.path.join(HERE, 'lpdf_names.json'), 'w') as f:
        json.dump(rows, f)
    print('lpdf cases', len(rows))


# ---------------------------------------------------------------- categorical
def gen_categorical():
    rng = np.random.RandomState(14)
    d = {}
    cases = []
    for upper in (2, 3, 4, 10):
        for n in (0, 5, 30, 500):
            for pchoice in (False, True):
                obs = rng.randint(upper, size=n)
                pw = float(rng.choice([1.0, 0.5]))
                lfw = tpe.linear_forgetting_weights(len(obs), 25)
                counts = np.bincount(obs, minlength=upper, weights=lfw)
                if pchoice:
                    pp = rng.dirichlet(np.ones(upper))
                    p = tpe.tpe_cat_pseudocounts(counts, upper, pw, pp, (7,))
                else:
                    pp = np.full(upper, np.nan)
                    pc = counts + pw
                    p = pc / np.sum(pc)
                srng = np.random.RandomState(2000 + len(cases))
                draws = stochastic.categorical(p, upper=upper, rng=srng, size=(64,))
                lp = tpe.categorical_lpdf(draws, p, upper)
                cases.append((obs, upper, pw, pp, p, draws, lp))
    pack(d, 'obs', [c[0] for c in cases], np.int64)
    d['upper'] = np.array([c[1] for c in cases], dtype=np.int64)
    d['pw'] = np.array([c[2] for c in cases])
    pack(d, 'pprior', [c[3] for c in cases])
    pack(d, 'p', [c[4] for c in cases])
    pack(d, 'draws', [c[5] for c in cases], np.int64)
    pack(d, 'lpdf', [c[6] for c in cases])
    np.savez_compressed(os.path.join(HERE, 'categorical.npz'), **d)
    print('categorical cases', len(cases))


# ---------------------------------------------------------------- samplers
def gen_samplers():
    d = {}
    cases = []
    mixes = [([.1, .3, .4, .2], [1.0, 2.0, 3.0, 4.0], [.1, .4, .8, 2.0]),
             ([.5, .5], [0.0, 1.0], [1.0, 0.3])]
    for mi, mix in enumerate(mixes):
        for fn_name in ('GMM1', 'LGMM1'):
            for (low, high, q) in ((None, None, None), (2.5, 3.5, None), (None, None, 0.5),
                                   (0.5, 1.5, 1.0)):
                fn = getattr(tpe, fn_name)
                seed = 300 + len(cases)
                x = fn(*mix, low=low, high=high, q=q, rng=np.random.RandomState(seed), size=(50,))
                cases.append((mi, 0 if fn_name == 'GMM1' else 1, opt(low), opt(high), opt(q), seed, x))
    d['meta'] = np.array([c[:6] for c in cases])
    pack(d, 'x', [c[6] for c in cases])
    np.savez_compressed(os.path.join(HERE, 'samplers.npz'), **d)
    with open(os.path.join(HERE, 'samplers_mixes.json'), 'w') as f:
        json.dump(mixes, f)
    print('sampler cases', len(cases))


# ---------------------------------------------------------------- cfg1 trajectories
def gen_cfg1():
    out = {}
    for seed in (0, 123):
        t = Trials()
        best = fmin(lambda x: (x - 3) ** 2, spaces.cfg1_space(hp), algo=tpe.suggest,
                    max_evals=100, trials=t, rstate=np.random.RandomState(seed))
        xs = [tr['misc']['vals']['x'][0] for tr in t.trials]
        out[str(seed)] = dict(best=best['x'], xs=xs, losses=t.losses())
    # n_EI=5 variant (TestOpt quadratic1 setting) to 60 evals
    from functools import partial
    t = Trials()
    best = fmin(lambda x: (x - 3) ** 2, spaces.cfg1_space(hp),
                algo=partial(tpe.suggest, n_EI_candidates=5),
                max_evals=60, trials=t, rstate=np.random.RandomState(123))
    out['123_nei5'] = dict(best=best['x'], xs=[tr['misc']['vals']['x'][0] for tr in t.trials],
                           losses=t.losses())
    with open(os.path.join(HERE, 'cfg1_traj.json'), 'w') as f:
        json.dump(out, f, indent=0)
    print('cfg1', {k: v['best'] for k, v in out.items()})


# ---------------------------------------------------------------- whole suggest
def history_from_rand(domain, n, seed, loss_seed):
    t = Trials()
    docs = rand.suggest(list(range(n)), domain, t, seed)
    losses = np.random.RandomState(loss_seed).rand(n)
    for doc, l in zip(docs, losses):
        doc['state'] = base.JOB_STATE_DONE
        doc['result'] = {'status': base.STATUS_OK, 'loss': float(l)}
    t.insert_trial_docs(docs)
    t.refresh()
    return t


def capture_suggest(domain, trials, seed, **kw):
    calls = []
    keep = []
    samp = {}

    def wrap(name, kind):
        f = scope._impls[name]

        def g(*a, **k):
            r = f(*a, **k)
            keep.append((a, k, r))
            if kind == 'sampler':
                samp[id(r)] = dict(name=name, args=a, kw=k)
            elif kind == 'lpdf':
                samp.setdefault(id(a[0]), {}).setdefault('lpdf', []).append((a, k, r))
            else:
                calls.append((a[0], a[1], a[2]))
            return r
        scope._impls[name] = g
        return f

    saved = {}
    for nm, kind in (('GMM1', 'sampler'), ('LGMM1', 'sampler'), ('categorical', 'sampler'),
                     ('GMM1_lpdf', 'lpdf'), ('LGMM1_lpdf', 'lpdf'), ('categorical_lpdf', 'lpdf'),
                     ('broadcast_best', 'best')):
        saved[nm] = wrap(nm, kind)
    try:
        docs = tpe.suggest([len(trials.trials)], domain, trials, seed, **kw)
    finally:
        for nm, f in saved.items():
            scope._impls[nm] = f
    per = []
    for (s, yb, ya) in calls:
        rec = samp.get(id(s), {})
        per.append(dict(samples=np.asarray(s, dtype=np.float64).ravel(),
                        llik_b=np.asarray(yb, dtype=np.float64).ravel(),
                        llik_a=np.asarray(ya, dtype=np.float64).ravel()))
    return docs, per


def gen_suggest():
    from hyperopt.pyll_utils import expr_to_config
    cases = {
        'cfg2': (spaces.cfg2_space(hp), 1000, 1, 2, 7, dict(n_EI_candidates=4096)),
        'many_dists': (spaces.many_dists_space(hp), 60, 3, 4, 5, dict()),
        'cond': (spaces.cond_space(hp), 120, 5, 6, 9, dict(n_EI_candidates=64)),
        'cfg3_small': (spaces.cfg3_space(hp), 300, 1, 2, 7, dict(n_EI_candidates=256)),
    }
    meta = {}
    for name, (space, n, hseed, lseed, sseed, kw) in cases.items():
        domain = base.Domain(lambda x: 0.0, space)
        trials = history_from_rand(domain, n, hseed, lseed)
        labels = sorted(domain.params.keys())
        vals = np.full((len(labels), n), np.nan)
        act = np.zeros((len(labels), n), dtype=np.uint8)
        for j, tr in enumerate(trials.trials):
            for i, lab in enumerate(labels):
                v = tr['misc']['vals'][lab]
                if v:
                    vals[i, j] = float(v[0]); act[i, j] = 1
        losses = np.array([tr['result']['loss'] for tr in trials.trials])
        docs, per = capture_suggest(domain, trials, sseed, **kw)
        out_vals = docs[0]['misc']['vals']
        chosen = np.full(len(labels), np.nan)
        for i, lab in enumerate(labels):
            if out_vals[lab]:
                chosen[i] = float(out_vals[lab][0])
        d = dict(vals=vals, active=act, losses=losses, chosen=chosen)
        pack(d, 'samples', [p['samples'] for p in per])
        pack(d, 'llik_b', [p['llik_b'] for p in per])
        pack(d, 'llik_a', [p['llik_a'] for p in per])
        np.savez_compressed(os.path.join(HERE, 'suggest_%s.npz' % name), **d)
        meta[name] = dict(labels=labels, n=n, hist_seed=hseed, loss_seed=lseed,
                          suggest_seed=sseed, kw=kw, new_id=n,
                          n_best_calls=len(per))
        print('suggest', name, 'calls', len(per), 'chosen', dict(zip(labels, chosen.tolist())))
    with open(os.path.join(HERE, 'suggest_meta.json'), 'w') as f:
        json.dump(meta, f, indent=1)


# ---------------------------------------------------------------- configs 3 / 4 at size
def _keep(per, order, picks):
    """The captured calls of the labels in ``picks`` (capture order is the
    reference interpreter's hp order ``order``)."""
    out = []
    for lab in picks:
        k = order.index(lab)
        out.append((lab, per[k]))
    return out


def gen_big():
    """Config 4 (100 x uniform(-5, 5), N = 1e4: K_a ~ 9976) and config 3 (50-hp
    conditional, N = 1e4) at full history size with 4096 reference-drawn
    candidates per hp; only a few hps' candidates / lliks are stored."""
    meta = {}
    # -- config 4: SURVEY 8(d) history, obs RandomState(1), losses RandomState(2)
    n, D = 10000, 100
    U = np.random.RandomState(1).uniform(-5, 5, (n, D))
    L = np.random.RandomState(2).rand(n)
    domain = base.Domain(lambda x: 0.0, spaces.cfg4_space(hp, D))
    labels = ['x%d' % i for i in range(D)]
    t = Trials()
    miscs = [dict(tid=j, cmd=domain.cmd, workdir=None,
                  idxs={lab: [j] for lab in labels},
                  vals={lab: [float(U[j, i])] for i, lab in enumerate(labels)})
             for j in range(n)]
    docs = t.new_trial_docs(list(range(n)), [None] * n,
                            [{'status': base.STATUS_OK, 'loss': float(l)} for l in L], miscs)
    for d in docs:
        d['state'] = base.JOB_STATE_DONE
    t.insert_trial_docs(docs)
    t.refresh()
    docs, per = capture_suggest(domain, t, 7, n_EI_candidates=4096)
    order = sorted(labels, reverse=True)          # the interpreter's hp order here
    assert len(per) == D
    picks = ['x0', 'x7', 'x42', 'x99']
    kept = _keep(per, order, picks)
    d = {}
    pack(d, 'samples', [p['samples'] for _, p in kept])
    pack(d, 'llik_b', [p['llik_b'] for _, p in kept])
    pack(d, 'llik_a', [p['llik_a'] for _, p in kept])
    out_vals = docs[0]['misc']['vals']
    d['chosen'] = np.array([float(out_vals[lab][0]) for lab in picks])
    np.savez_compressed(os.path.join(HERE, 'suggest_cfg4.npz'), **d)
    meta['cfg4'] = dict(labels=picks, n=n, D=D, obs_seed=1, loss_seed=2, suggest_seed=7,
                        kw=dict(n_EI_candidates=4096), new_id=n)
    print('cfg4 kept', picks, d['chosen'])
    # -- config 3: rand.suggest history seed 1, losses RandomState(2)
    domain = base.Domain(lambda x: 0.0, spaces.cfg3_space(hp))
    trials = history_from_rand(domain, 10000, 1, 2)
    docs, per = capture_suggest(domain, trials, 7, n_EI_candidates=4096)
    sizes = [p['samples'].size for p in per]
    live = [k for k, z in enumerate(sizes) if z > 0]
    d = {}
    pack(d, 'samples', [per[k]['samples'] for k in live])
    pack(d, 'llik_b', [per[k]['llik_b'] for k in live])
    pack(d, 'llik_a', [per[k]['llik_a'] for k in live])
    labs = sorted(domain.params.keys())
    out_vals = docs[0]['misc']['vals']
    d['chosen'] = np.array([float(out_vals[lab][0]) if out_vals[lab] else np.nan for lab in labs])
    d['call_index'] = np.array(live, dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, 'suggest_cfg3_full.npz'), **d)
    meta['cfg3_full'] = dict(labels=labs, n=10000, hist_seed=1, loss_seed=2, suggest_seed=7,
                             kw=dict(n_EI_candidates=4096), new_id=10000, n_calls=len(per))
    print('cfg3 full: calls', len(per), 'with candidates', live)
    with open(os.path.join(HERE, 'suggest_big_meta.json'), 'w') as f:
        json.dump(meta, f, indent=1)


# ---------------------------------------------------------------- TestOpt runs
def gen_testopt():
    """fmin trajectories of the reference's TestOpt (test_tpe.py:517-641)."""
    from functools import partial
    from hyperopt.pyll import as_apply
    import domains
    out = {}
    for name in domains.NAMES:
        kw, n = domains.settings(name)
        space = domains.build(name, hp, scope, as_apply)
        old = np.seterr('raise')
        np.seterr(under='ignore')
        try:
            t = Trials()
            fmin(lambda x: x, space=space, algo=partial(tpe.suggest, **kw), trials=t,
                 max_evals=n, rstate=np.random.RandomState(123))
        finally:
            np.seterr(**old)
        vals = [{k: (v[0] if v else None) for k, v in tr['misc']['vals'].items()}
                for tr in t.trials]
        out[name] = dict(vals=vals, losses=t.losses(), min=min(t.losses()))
        print('testopt', name, len(t.trials), min(t.losses()))
    with open(os.path.join(HERE, 'testopt_traj.json'), 'w') as f:
        json.dump(out, f)


if __name__ == '__main__':
    np.seterr(all='ignore')
    gens = dict(split=gen_split, parzen=gen_parzen, lpdf=gen_lpdf, categorical=gen_categorical,
                samplers=gen_samplers, cfg1=gen_cfg1, suggest=gen_suggest, testopt=gen_testopt,
                big=gen_big)
    for name, g in gens.items():
        if not ONLY or name in ONLY:
            g()
