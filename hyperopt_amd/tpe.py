"""TPE suggestion on the MI355X engine -- ``tpe.suggest`` drop-in.

Same call as the reference (hyperopt/tpe.py:804-897)::

    suggest(new_ids, domain, trials, seed, prior_weight=1.0, n_startup_jobs=20,
            n_EI_candidates=24, gamma=0.25, linear_forgetting=25)

Host side (this module): the trial history is a columnar mirror of the
Trials (``history.TrialHistory``: tpe.py:820-848 semantics, synced
incrementally and copied to the device row by row), the startup fallback to
``rand.suggest`` and the write-back of the winning values (tpe.py:887-897).
Device side (libtpe_engine.so, one plan per Domain): the good/bad split,
every hyperparameter's two Parzen fits, candidate draws, below/above lpdf
and the EI argmax, level by level through conditional choices.  There is no
CPU fallback: without the engine this raises.

``new_ids`` may hold several ids (the reference accepts exactly one,
tpe.py:812): the suggestions are served by ONE batched engine call on the
same history, suggestion s drawing its candidates with ``batch_seeds(seed,
S)[s]`` (s = 0 uses ``seed`` itself, so a single suggestion is unchanged).

``rng_stream='numpy'`` replays the reference's RandomState candidate stream
(hyperopt draws in its interpreter order): the fit and the scoring stay on the
GPU, the draws are made on the host with the reference's numpy calls, so the
suggestions equal the reference's (up to 1e-6 EI ties).  The default
``'philox'`` draws candidates on the device (counter-based Philox keyed by
seed, hp and candidate index).
"""
from __future__ import annotations

import logging
import math
import threading
import weakref

import numpy as np

from . import _engine as E
from . import rand, rstream
from .history import TrialHistory

logger = logging.getLogger(__name__)

EPS = 1e-12
DEFAULT_LF = 25

_default_prior_weight = 1.0
_default_n_EI_candidates = 24
_default_gamma = 0.25
_default_n_startup_jobs = 20
_default_linear_forgetting = DEFAULT_LF


def build_history(domain, trials, labels=None):
    """(tids, losses[N], vals[P, N], active[P, N]) of ``trials`` in tid
    order -- the reference's history assembly (tpe.py:820-848), from a
    fresh columnar mirror.  ``labels`` must be the domain's (sorted) labels."""
    h = TrialHistory(domain)
    if labels is not None and list(labels) != h.labels:
        raise ValueError('labels must be the domain space labels')
    return h.sync(trials).columns()


def batch_seeds(seed, n):
    """Per-suggestion Philox keys of a batch: ``seed`` first, then splitmix64
    steps of it (independent streams; deterministic in (seed, position))."""
    out = [int(seed) & (2 ** 64 - 1)]
    z = out[0]
    for _ in range(1, n):
        z = (z + 0x9E3779B97F4A7C15) & (2 ** 64 - 1)
        x = z
        x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & (2 ** 64 - 1)
        x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & (2 ** 64 - 1)
        out.append(x ^ (x >> 31))
    return out


# --------------------------------------------------------------------------
# per-Domain device state: the plan, and one history mirror per Trials
# --------------------------------------------------------------------------
class _State(object):
    def __init__(self):
        self.plan = None
        self.lock = threading.Lock()
        self.histories = weakref.WeakKeyDictionary()

    def history(self, domain, trials):
        h = self.histories.get(trials)
        if h is None:
            h = self.histories[trials] = TrialHistory(domain)
        return h

    def plan_for(self, domain, n, engine):
        p = self.plan
        if p is None or p.max_trials < n or p.engine is not engine:
            cap = max(64, 1 << max(0, int(math.ceil(math.log2(max(n, 1))))))
            hps, conds, pprior = domain.space.engine_tables()
            self.plan = p = E.Plan(engine, hps, conds, pprior, cap)
        return p


def _state(domain):
    st = domain.__dict__.get('_tpe_state')
    if st is None:
        st = domain.__dict__.setdefault('_tpe_state', _State())
    return st


def _domain_plan(domain, n_trials, engine):
    """The domain's plan, sized for ``n_trials`` (tools / tests)."""
    st = _state(domain)
    st.plan_for(domain, n_trials, engine)
    return st


def _fmt(h, v):
    return int(round(v)) if h.is_categorical else float(v)


def _new_doc(domain, trials, cs, new_id, chosen):
    """The returned document (tpe.py:887-897): misc idxs / vals of the one
    new id -- what miscs_update_idxs_vals(idxs_map={fake_ids[0]: new_id})
    leaves in it, built directly (one misc, every label present)."""
    misc = dict(tid=new_id, cmd=domain.cmd, workdir=domain.workdir,
                idxs={lab: ([new_id] if lab in chosen else []) for lab in cs.labels},
                vals={lab: ([chosen[lab]] if lab in chosen else []) for lab in cs.labels})
    return trials.new_trial_docs([new_id], [None], [domain.new_result()], [misc])[0]


def _picks(cs, res):
    """{label: value} of every suggestion's active winners, from the engine's
    [S][P] records (one conversion to Python lists, no per-field numpy
    scalar access)."""
    S = res.shape[0]
    act = res['active'].tolist()
    idx = res['index'].tolist()
    val = res['value'].tolist()
    out = []
    for s in range(S):
        a, i, v = act[s], idx[s], val[s]
        out.append({lab: (int(round(v[j])) if cat else v[j])
                    for lab, j, cat in cs.pick_order if a[j] and i[j] >= 0})
    return out


def suggest(new_ids, domain, trials, seed,
            prior_weight=_default_prior_weight,
            n_startup_jobs=_default_n_startup_jobs,
            n_EI_candidates=_default_n_EI_candidates,
            gamma=_default_gamma,
            linear_forgetting=_default_linear_forgetting,
            rng_stream='philox', startup_stream='numpy', engine=None):
    """hyperopt/tpe.py:804-897 on the GPU, one document per id in
    ``new_ids``.  ``linear_forgetting`` is accepted and, as in the reference
    (tpe.py:809), not used: LF is fixed at 25.  The first ``n_startup_jobs``
    trials come from ``rand.suggest`` with ``startup_stream``: 'numpy' (the
    reference's RandomState stream, default) or 'philox' (device prior
    draws, tpe_plan_sample_prior)."""
    new_ids = list(new_ids)
    if not new_ids:
        return []
    if rng_stream not in ('philox', 'numpy'):
        raise ValueError('rng_stream must be "philox" or "numpy"')
    cs = domain.space
    st = _state(domain)
    with st.lock:
        hist = st.history(domain, trials).sync(trials)
        startup = hist.n < n_startup_jobs
    if startup:
        # the reference's RandomState prior stream (numpy), or device prior
        # draws with the Philox stream (tpe_plan_sample_prior)
        return rand.suggest(new_ids, domain, trials, seed, rng_stream=startup_stream)
    with st.lock:
        engine = engine or E.default_engine()
        plan = st.plan_for(domain, hist.n, engine)
        hist.push(plan)
        seeds = batch_seeds(seed, len(new_ids))
        n_ei = int(n_EI_candidates)
        if rng_stream == 'philox':
            # fit + sample + score + argmax of every suggestion in one call
            res = plan.fit_suggest(seeds, n_ei, gamma=gamma, prior_weight=prior_weight,
                                   lf=DEFAULT_LF)
            picks = _picks(cs, res)
        else:
            plan.fit(gamma=gamma, prior_weight=prior_weight, lf=DEFAULT_LF)
            picks = [_suggest_numpy_stream(cs, plan, sd, n_ei) for sd in seeds]
    return [_new_doc(domain, trials, cs, i, c) for i, c in zip(new_ids, picks)]


def _suggest_numpy_stream(cs, plan, seed, n_ei):
    """Reference RandomState candidate stream; fit + scoring on the GPU."""
    rng = np.random.RandomState(seed)
    chosen = {}
    for lab in cs.draw_order:
        if not cs.is_active(lab, chosen):
            continue
        h = cs.by_label[lab]
        if h.is_categorical:
            p = plan.mixture(h.index, 0)[0]
            cand = rstream.multinomial_draw(rng, p, n_ei).astype(np.float64)
        else:
            t = cs.engine_tables()[0][h.index]
            lg = t.family == E.LGMM
            low = t.low if t.flags & E.HAS_LOW else None
            high = t.high if t.flags & E.HAS_HIGH else None
            q = t.q if t.flags & E.HAS_Q else None
            cand = rstream.posterior_draw(rng, lg, plan.mixture(h.index, 0), low, high, q, n_ei)
        if n_ei == 0:
            continue
        _, _, best, _ = plan.score_candidates(h.index, cand)
        chosen[lab] = _fmt(h, cand[best])
    return chosen


# --------------------------------------------------------------------------
# operator-level drop-ins for the reference's scope functions (GPU-backed)
# --------------------------------------------------------------------------
def _eng():
    return E.default_engine()


def ap_filter_trials(o_idxs, o_vals, l_idxs, l_vals, gamma, gamma_cap=DEFAULT_LF):
    """tpe.py:613-641; ties in the loss ranking broken by position."""
    l_idxs = np.asarray(l_idxs)
    mask = _eng().split(np.asarray(l_vals, dtype=np.float64), gamma, gamma_cap)
    good = set(l_idxs[mask].tolist())
    bad = set(l_idxs[~mask].tolist())
    below = [v for i, v in zip(o_idxs, o_vals) if i in good]
    above = [v for i, v in zip(o_idxs, o_vals) if i in bad]
    return np.asarray(below), np.asarray(above)


def linear_forgetting_weights(N, LF):
    """tpe.py:381-394 (host: trivial)."""
    assert N >= 0 and LF > 0
    if N == 0:
        return np.asarray([])
    if N < LF:
        return np.ones(N)
    return np.concatenate([np.linspace(1.0 / N, 1.0, num=N - LF), np.ones(LF)], axis=0)


def adaptive_parzen_normal(mus, prior_weight, prior_mu, prior_sigma, LF=DEFAULT_LF):
    """tpe.py:398-475 on the GPU (stable sort for tied observations)."""
    mus = np.asarray(mus, dtype=np.float64)
    if mus.ndim != 1:
        raise TypeError('mus must be vector', mus)
    return _eng().parzen_fit(mus, prior_weight, prior_mu, prior_sigma, LF)


def _opt(v):
    return None if v is None else float(v)


def GMM1_lpdf(samples, weights, mus, sigmas, low=None, high=None, q=None):
    """tpe.py:104-166 on the GPU."""
    w, m, s = (np.asarray(a, dtype=np.float64) for a in (weights, mus, sigmas))
    for a, nm in ((w, 'weights'), (m, 'mus'), (s, 'sigmas')):
        if a.ndim != 1:
            raise TypeError('need vector of %s' % nm, a.shape)
    x = np.asarray(samples, dtype=np.float64)
    if x.size == 0:
        return np.asarray([])
    return _eng().lpdf(E.GMM, x, w, m, s, _opt(low), _opt(high), _opt(q))


def LGMM1_lpdf(samples, weights, mus, sigmas, low=None, high=None, q=None):
    """tpe.py:259-301 on the GPU."""
    w, m, s = (np.asarray(a, dtype=np.float64) for a in (weights, mus, sigmas))
    x = np.asarray(samples, dtype=np.float64)
    if x.size == 0:
        return np.asarray([]).reshape(x.shape)
    return _eng().lpdf(E.LGMM, x, w, m, s, _opt(low), _opt(high), _opt(q))


def categorical_lpdf(sample, p, upper=None):
    """tpe.py:50-57 on the GPU."""
    sample = np.asarray(sample)
    if sample.size == 0:
        return np.asarray([])
    p = np.asarray(p, dtype=np.float64)
    return _eng().lpdf(E.CAT, sample.astype(np.float64), p)


def broadcast_best(samples, below_llik, above_llik):
    """tpe.py:749-759 (argmax with numpy semantics)."""
    if len(samples):
        score = np.asarray(below_llik) - np.asarray(above_llik)
        if len(samples) != len(score):
            raise ValueError()
        best = int(np.argmax(score))
        return [samples[best]] * len(samples)
    return []


def GMM1(weights, mus, sigmas, low=None, high=None, q=None, rng=None, size=()):
    """tpe.py:62-93: Philox draws on the GPU, seeded from ``rng``."""
    return _draw(E.GMM, weights, mus, sigmas, low, high, q, rng, size)


def LGMM1(weights, mus, sigmas, low=None, high=None, q=None, rng=None, size=()):
    """tpe.py:216-250: Philox draws on the GPU, seeded from ``rng``."""
    return _draw(E.LGMM, weights, mus, sigmas, low, high, q, rng, size)


def _draw(family, weights, mus, sigmas, low, high, q, rng, size):
    n = int(np.prod(size)) if size != () else 1
    seed = int(rng.randint(2 ** 31 - 1)) if rng is not None else int(np.random.randint(2 ** 31 - 1))
    if (low is None) != (high is None):
        raise TypeError('one-sided truncation is not supported (tpe.py:76)')
    out = _eng().sample(family, weights, mus, sigmas, _opt(low), _opt(high), _opt(q), seed=seed,
                        n=n)
    return out.reshape(size) if size != () else out[0]
