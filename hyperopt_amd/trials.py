"""Columnar trial store behind the reference's ``Trials`` interface.

The reference keeps trials as a list of dicts and every TPE call walks all
of them (hyperopt/base.py:217-650, tpe.py:820-848).  Here the documents are
still dicts (user code reads ``trials.trials[i]['misc']['vals']``), but the
store also keeps, per document, the columns the suggest path needs -- job
state, experiment-key match -- and an append-only *change journal*: every
assignment of ``state``/``result``/``misc``/``exp_key`` on a stored document
is logged.  A consumer (``history.TrialHistory``, one per Domain) replays the
journal since its last cursor, so a suggest touches only the documents that
changed instead of the whole history.

Behaviour (which documents are visible, id allocation, doc layout, errors)
follows the reference; see the cited lines at each method.
"""
from __future__ import annotations

import datetime
import itertools

import numpy as np

from . import status as S

__all__ = ['TrialDoc', 'Trials', 'trials_from_docs', 'InvalidTrial', 'SONify']

# the document fields whose reassignment changes what TPE sees
_TRACKED = frozenset(('state', 'result', 'misc', 'exp_key', 'spec', 'tid'))


class InvalidTrial(ValueError):
    """A document that does not have the trial layout (base.py:372-400)."""


_PLAIN = (str, int, float, bool, type(None), datetime.datetime)


def SONify(arg):
    """numpy scalars / arrays -> plain Python containers and numbers
    (the reference's BSON-friendliness pass, base.py:108-150)."""
    if type(arg) in _PLAIN:  # the common leaves: one exact type test
        return arg
    if isinstance(arg, dict):
        return {SONify(k): SONify(v) for k, v in arg.items()}
    if isinstance(arg, (list, tuple)):
        return type(arg)(SONify(v) for v in arg)
    if isinstance(arg, np.ndarray):
        return SONify(arg.item()) if arg.ndim == 0 else [SONify(v) for v in arg]
    if isinstance(arg, np.bool_):
        return bool(arg)
    if isinstance(arg, np.integer):
        return int(arg)
    if isinstance(arg, np.floating):
        return float(arg)
    return arg


def coarse_utcnow():
    """UTC now at millisecond resolution (what mongo would store)."""
    t = datetime.datetime.utcnow()
    return t.replace(microsecond=1000 * (t.microsecond // 1000))


class _Journal(object):
    """Append-only log of changed documents.  ``gen`` changes when the log is
    compacted or the store is cleared: a consumer holding an older gen must
    rebuild from scratch."""
    __slots__ = ('docs', 'gen')

    def __init__(self):
        self.docs = []
        self.gen = 0

    def reset(self):
        # gen first: a reader snapshots docs, then gen, and rebuilds on a
        # changed gen whichever list it got (history.TrialHistory.sync)
        self.gen += 1
        self.docs = []


class TrialDoc(dict):
    """A stored trial document: a dict that logs reassignments of the tracked
    fields to its store's journal and keeps its state column current."""
    __slots__ = ('_store', '_row')

    def __init__(self, *a, **kw):
        dict.__init__(self, *a, **kw)
        self._store = None
        self._row = -1

    def _changed(self, key):
        st = self._store
        if st is not None and key in _TRACKED:
            st._touch(self, key)

    def __setitem__(self, key, value):
        dict.__setitem__(self, key, value)
        self._changed(key)

    def __delitem__(self, key):
        dict.__delitem__(self, key)
        self._changed(key)

    def update(self, *a, **kw):
        d = dict(*a, **kw)
        dict.update(self, d)
        for k in d:
            self._changed(k)

    def setdefault(self, key, default=None):
        if key in self:
            return self[key]
        self[key] = default
        return default

    def pop(self, key, *default):
        v = dict.pop(self, key, *default)
        self._changed(key)
        return v

    def __reduce__(self):
        # pickles / deep-copies as a detached document
        return (TrialDoc, (dict(self),))

    def __copy__(self):
        return TrialDoc(dict(self))


class _Column(object):
    """A growable 1-D numpy column (amortised doubling)."""
    __slots__ = ('a', 'n')

    def __init__(self, dtype, cap=64):
        self.a = np.zeros(cap, dtype=dtype)
        self.n = 0

    def push(self, v):
        if self.n == self.a.size:
            b = np.zeros(2 * self.a.size, dtype=self.a.dtype)
            b[:self.n] = self.a[:self.n]
            self.a = b
        self.a[self.n] = v
        self.n += 1

    def view(self):
        return self.a[:self.n]

    def clear(self):
        self.n = 0


class _Store(object):
    """Documents in insertion order plus their state / key columns, shared
    by a Trials object and its views (base.py:271-279 share the list)."""

    def __init__(self):
        self.docs = []
        self.state = _Column(np.int8)
        self.keys = []            # exp_key per document
        self.journal = _Journal()
        self.ids = set()          # every tid seen or handed out (base.py:264, 427-431)

    def add(self, doc):
        if not isinstance(doc, TrialDoc):
            doc = TrialDoc(doc)
        if doc._store is not None and doc._store is not self:
            doc = TrialDoc(dict(doc))   # a document lives in one store
        doc._store = self
        doc._row = len(self.docs)
        self.docs.append(doc)
        self.state.push(_state_code(doc.get('state')))
        self.keys.append(doc.get('exp_key'))
        return doc

    def _touch(self, doc, key):
        r = doc._row
        if key == 'state':
            self.state.a[r] = _state_code(doc.get('state'))
        elif key == 'exp_key':
            self.keys[r] = doc.get('exp_key')
        self.journal.docs.append(doc)
        # keep the log proportional to the store
        if len(self.journal.docs) > 8 * len(self.docs) + 4096:
            self.journal.reset()

    def clear(self):
        for d in self.docs:
            d._store = None
        self.docs = []
        self.state.clear()
        self.keys = []
        self.journal.reset()

    def __setstate__(self, state):
        # a pickled / deep-copied store comes back with detached documents
        # (TrialDoc.__reduce__): re-attach them, rebuild the state / key
        # columns from the documents and start a new journal generation, so
        # resuming fmin on an unpickled Trials tracks state changes again
        # (the reference reads states from the documents, base.py:327-338)
        self.__dict__.update(state)
        self.state = _Column(np.int8, max(64, len(self.docs)))
        self.keys = []
        for r, doc in enumerate(self.docs):
            doc._store = self
            doc._row = r
            self.state.push(_state_code(doc.get('state')))
            self.keys.append(doc.get('exp_key'))
        self.journal.reset()


def _state_code(v):
    try:
        return int(v)
    except (TypeError, ValueError):
        return -1


class Trials(object):
    """The trial database of one optimisation (hyperopt/base.py:217-638).

    ``trials`` is the list visible since the last :meth:`refresh` (documents
    in an error state, or of another experiment key, are hidden); documents
    are shared objects, so results written into them are visible at once.
    """

    async_ = False

    def __init__(self, exp_key=None, refresh=True):
        self._store = _Store()
        self._exp_key = exp_key
        self.attachments = {}
        self._trials = []
        self._mask = np.zeros(0, dtype=bool)
        self._epoch = 0           # bumped when a refresh drops an earlier document
        if refresh:
            self.refresh()

    # -- views sharing the store (base.py:271-279) -------------------------
    def view(self, exp_key=None, refresh=True):
        other = object.__new__(self.__class__)
        other._store = self._store
        other._exp_key = exp_key
        other.attachments = self.attachments
        other._trials = []
        other._mask = np.zeros(0, dtype=bool)
        other._epoch = 0
        if refresh:
            other.refresh()
        return other

    @property
    def _dynamic_trials(self):
        """Every stored document, insertion order (reference attribute)."""
        return self._store.docs

    # -- visibility --------------------------------------------------------
    def _visible_mask(self, docs_state, keys):
        m = docs_state != S.JOB_STATE_ERROR
        if self._exp_key is not None:
            m &= np.fromiter((k == self._exp_key for k in keys), dtype=bool, count=len(keys))
        return m

    def refresh(self):
        """Recompute the visible documents (base.py:327-338): every stored
        document not in an error state (and of this exp_key)."""
        st = self._store
        mask = self._visible_mask(st.state.view(), st.keys)
        old = self._mask
        n_old = min(old.size, mask.size)
        if old.size <= mask.size and np.array_equal(mask[:n_old], old):
            # a pure extension (the common case): only the new documents
            # are looked at; the list is a new object as in the reference
            add = list(itertools.compress(st.docs[n_old:], mask[n_old:]))
            st.ids.update(d['tid'] for d in add)
            self._trials = self._trials + add
        else:
            self._epoch += 1      # an earlier document dropped out: consumers rebuild
            # the visible tids join the known ids (the set never shrinks)
            fresh = mask.copy()
            fresh[:n_old] &= ~old[:n_old]
            st.ids.update(d['tid'] for d in itertools.compress(st.docs, fresh))
            self._trials = list(itertools.compress(st.docs, mask))
        self._mask = mask

    @property
    def trials(self):
        return self._trials

    def __iter__(self):
        return iter(self._trials)

    def __len__(self):
        return len(self._trials)

    def __getitem__(self, item):
        # by position or by tid would be ambiguous (base.py:322-325)
        raise NotImplementedError('')

    @property
    def tids(self):
        return [d['tid'] for d in self._trials]

    @property
    def specs(self):
        return [d['spec'] for d in self._trials]

    @property
    def results(self):
        return [d['result'] for d in self._trials]

    @property
    def miscs(self):
        return [d['misc'] for d in self._trials]

    @property
    def idxs_vals(self):
        from .base import miscs_to_idxs_vals
        return miscs_to_idxs_vals(self.miscs)

    @property
    def idxs(self):
        return self.idxs_vals[0]

    @property
    def vals(self):
        return self.idxs_vals[1]

    # -- attachments (base.py:281-306) --------------------------------------
    def aname(self, trial, name):
        return 'ATTACH::%s::%s' % (trial['tid'], name)

    def trial_attachments(self, trial):
        return _TrialAttachments(self, trial)

    # -- insertion ---------------------------------------------------------
    def assert_valid_trial(self, trial):
        """Layout check of one document (base.py:372-400)."""
        if not (hasattr(trial, 'keys') and hasattr(trial, 'values')):
            raise InvalidTrial('trial should be dict-like', trial)
        missing = [k for k in S.TRIAL_KEYS if k not in trial]
        if missing:
            raise InvalidTrial('trial missing key %s', missing[0])
        misc = trial['misc']
        missing = [k for k in S.TRIAL_MISC_KEYS if k not in misc]
        if missing:
            raise InvalidTrial('trial["misc"] missing key', missing[0])
        if trial['tid'] != misc['tid']:
            raise InvalidTrial('tid mismatch between root and misc', trial)
        if trial['exp_key'] != self._exp_key:
            raise InvalidTrial('wrong exp_key', (trial['exp_key'], self._exp_key))
        return trial

    def _insert_trial_docs(self, docs):
        """Store without validation; returns the tids (base.py:402-407)."""
        st = self._store
        return [st.add(d)['tid'] for d in docs]

    def insert_trial_doc(self, doc):
        return self.insert_trial_docs([doc])[0]

    def insert_trial_docs(self, docs):
        """Validate and store; visible after the next refresh."""
        checked = [self.assert_valid_trial(SONify(d)) for d in docs]
        return self._insert_trial_docs(checked)

    def new_trial_ids(self, N):
        """N fresh ids: the count of ids known so far onwards (base.py:427-431)."""
        ids = self._store.ids
        first = len(ids)
        out = list(range(first, first + N))
        ids.update(out)
        return out

    def new_trial_docs(self, tids, specs, results, miscs):
        """Fresh NEW-state documents (base.py:433-449); not inserted."""
        cols = (tids, specs, results, miscs)
        if len(set(map(len, cols))) != 1:
            raise AssertionError('tids/specs/results/miscs differ in length')
        return [TrialDoc(tid=t, spec=s, result=r, misc=m, state=S.JOB_STATE_NEW,
                         exp_key=self._exp_key, owner=None, version=0, book_time=None,
                         refresh_time=None)
                for t, s, r, m in zip(*cols)]

    def source_trial_docs(self, tids, specs, results, miscs, sources):
        """Documents derived from existing trials (Ctrl.inject_results,
        base.py:451-474): misc.from_tid names the source trial."""
        cols = (tids, specs, results, miscs, sources)
        if len(set(map(len, cols))) != 1:
            raise AssertionError('argument lengths differ')
        out = []
        for t, s, r, m, src in zip(*cols):
            for k, v in (('tid', t), ('cmd', None), ('from_tid', src['tid'])):
                if m.setdefault(k, v) != v:
                    raise AssertionError('misc[%r] != %r' % (k, v))
            out.append(TrialDoc(tid=t, spec=s, result=r, misc=m, version=0,
                                state=src['state'], exp_key=src['exp_key'],
                                owner=src['owner'], book_time=src['book_time'],
                                refresh_time=src['refresh_time']))
        return out

    def delete_all(self):
        self._store.clear()
        self.attachments = {}
        self._epoch += 1
        self._mask = np.zeros(0, dtype=bool)
        self._trials = []
        self.refresh()

    # -- state counts (base.py:481-509), on the state column -----------------
    def _count(self, arg, states):
        if isinstance(arg, (int, np.integer)) and arg in S.JOB_STATES:
            want = np.asarray([arg], dtype=np.int8)
        elif hasattr(arg, '__iter__'):
            ss = set(arg)
            if not all(x in S.JOB_STATES for x in ss):
                raise AssertionError('unknown job state in %r' % (arg,))
            want = np.asarray(sorted(ss), dtype=np.int8)
        else:
            raise TypeError(arg)
        return int(np.isin(states, want).sum())

    def count_by_state_synced(self, arg, trials=None):
        if trials is None:
            return self._count(arg, self._store.state.view()[self._mask])
        return self._count(arg, np.fromiter((_state_code(d['state']) for d in trials),
                                            dtype=np.int8, count=len(trials)))

    def count_by_state_unsynced(self, arg):
        st = self._store
        states = st.state.view()
        if self._exp_key is not None:
            keep = np.fromiter((k == self._exp_key for k in st.keys), dtype=bool,
                               count=len(st.keys))
            states = states[keep]
        return self._count(arg, states)

    # -- results ------------------------------------------------------------
    def losses(self, bandit=None):
        if bandit is None:
            return [r.get('loss') for r in self.results]
        return [bandit.loss(r, s) for r, s in zip(self.results, self.specs)]

    def statuses(self, bandit=None):
        if bandit is None:
            return [r.get('status') for r in self.results]
        return [bandit.status(r, s) for r, s in zip(self.results, self.specs)]

    def average_best_error(self, bandit=None):
        """True loss of the best trial, averaged over the probability that
        each near-best trial is the best when losses are noisy
        (base.py:523-573)."""
        rs = self.results
        if bandit is None:
            ok = [r for r in rs if r['status'] == S.STATUS_OK]
            rows = [(r['loss'], r.get('loss_variance', 0), r.get('true_loss', r['loss']))
                    for r in ok]
        else:
            pairs = [(r, s) for r, s in zip(rs, self.specs) if bandit.status(r) == S.STATUS_OK]
            rows = [(bandit.loss(r, s), bandit.loss_variance(r, s), bandit.true_loss(r, s))
                    for r, s in pairs]
            if rows and not np.all(np.isfinite(np.asarray(rows, dtype=float))):
                raise ValueError()
        if not rows:
            raise ValueError('Empty loss vector')
        tab = np.asarray(sorted(rows), dtype=float)
        loss, var, true = tab[:, 0], tab[:, 1], tab[:, 2]
        if not var.any():
            return true[np.argmin(loss)]
        limit = loss[0] + 3 * np.sqrt(var[0])
        n = 0
        while n < len(loss) and loss[n] < limit:
            n += 1
        p = pmin_sampled(loss[:n], var[:n])
        return (p * true[:n]).sum()

    @property
    def best_trial(self):
        """The STATUS_OK trial of lowest loss (first on ties), or None."""
        ok = [d for d in self._trials if d['result']['status'] == S.STATUS_OK]
        if not ok:
            return None
        ls = np.asarray([float(d['result']['loss']) for d in ok])
        if np.isnan(ls).any():
            raise AssertionError('NaN loss among STATUS_OK trials')
        return ok[int(np.argmin(ls))]

    @property
    def argmin(self):
        """{label: value} of the best trial's active hyperparameters."""
        bt = self.best_trial
        if bt is None:
            return {}
        return {k: v[0] for k, v in bt['misc']['vals'].items() if v}

    def fmin(self, fn, space, algo, max_evals, rstate=None, verbose=0,
             pass_expr_memo_ctrl=None, catch_eval_exceptions=False, return_argmin=True,
             max_queue_len=1):
        from .fmin import fmin
        return fmin(fn, space, algo, max_evals, trials=self, rstate=rstate, verbose=verbose,
                    allow_trials_fmin=False, pass_expr_memo_ctrl=pass_expr_memo_ctrl,
                    catch_eval_exceptions=catch_eval_exceptions, return_argmin=return_argmin,
                    max_queue_len=max_queue_len)


class _TrialAttachments(object):
    """attachments[name] of one trial, stored in the Trials' blob dict."""
    __slots__ = ('t', 'doc')

    def __init__(self, t, doc):
        self.t, self.doc = t, doc

    def __contains__(self, name):
        return self.t.aname(self.doc, name) in self.t.attachments

    def __getitem__(self, name):
        return self.t.attachments[self.t.aname(self.doc, name)]

    def __setitem__(self, name, value):
        self.t.attachments[self.t.aname(self.doc, name)] = value

    def __delitem__(self, name):
        del self.t.attachments[self.t.aname(self.doc, name)]


def pmin_sampled(mean, var, n_samples=1000, rng=None):
    """Monte-Carlo probability that each of several noisy losses is the
    smallest (hyperopt/utils.py pmin_sampled)."""
    rng = np.random.RandomState(232342) if rng is None else rng
    draws = rng.randn(n_samples, len(mean)) * np.sqrt(var) + mean
    hits = (draws == draws.min(axis=1)[:, None]).sum(axis=0)
    return hits.astype('float64') / hits.sum()


def trials_from_docs(docs, validate=True, **kwargs):
    """A refreshed Trials holding ``docs`` (base.py:641-650)."""
    t = Trials(**kwargs)
    if validate:
        t.insert_trial_docs(docs)
    else:
        t._insert_trial_docs(docs)
    t.refresh()
    return t
