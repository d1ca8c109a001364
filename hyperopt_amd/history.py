"""Columnar trial history of one (Domain, Trials) pair, synced incrementally
to the engine.

The reference re-assembles the history from every trial document on every
``tpe.suggest`` (tpe.py:820-848 plus ``miscs_to_idxs_vals``, base.py:187-202)
and hands it to numpy.  Here the history is kept as columns -- per-trial
losses, per-hyperparameter values and activity -- that are extended as
trials arrive: a sync reads only the documents appended to the visible list
and the ones the store's change journal names, and ``push`` copies only the
changed rows to the plan's device-resident history
(``tpe_plan_update_history``).

Semantics are the reference's: the loss of a trial is ``domain.loss(result,
spec)`` with None -> +inf; documents sharing a tid (``misc.from_tid``) keep
the one of lowest loss (the later one on ties); a tid whose first document
has a NaN loss is dropped; rows are in tid order; an observation counts for
a trial when its misc idxs entry equals the trial's (from_tid-aware) tid.
A history that is a plain extension (new integer tids in increasing order,
no from_tid) takes the incremental path; anything else rebuilds the columns
from cached per-document rows.
"""
from __future__ import annotations

import math
import numbers
import weakref

import numpy as np

def _loss_of(domain, doc):
    v = domain.loss(doc['result'], doc['spec'])
    return math.inf if v is None else float(v)


def _is_int_tid(t):
    return isinstance(t, numbers.Integral) and not isinstance(t, bool)


class TrialHistory(object):
    """losses[n], vals[P][n], active[P][n] in tid order (host columns with a
    row capacity; ``self.vals[:, :self.n]`` etc. are the live part)."""

    def __init__(self, domain):
        self.domain = domain
        self.labels = list(domain.space.labels)
        self.P = len(self.labels)
        self._cache = {}        # id(doc) -> (doc, tid, vals row, active row)
        self._alloc(64)
        self._forget()

    # -- storage -------------------------------------------------------------
    def _alloc(self, cap):
        self.cap = cap
        self.losses = np.zeros(cap)
        self.vals = np.zeros((self.P, cap))
        self.active = np.zeros((self.P, cap), dtype=np.uint8)

    def _grow(self, need):
        if need <= self.cap:
            return
        cap = self.cap
        while cap < need:
            cap *= 2
        l, v, a = self.losses, self.vals, self.active
        self._alloc(cap)
        self.losses[:self.n] = l[:self.n]
        self.vals[:, :self.n] = v[:, :self.n]
        self.active[:, :self.n] = a[:, :self.n]

    def _forget(self):
        """Drop all rows: the next sync rebuilds from the documents."""
        self.n = 0
        self.tids = []
        self.docs = []          # the document of each row
        self._row = {}          # id(doc) -> row (incremental mode)
        self._dropped = {}      # id(doc) -> (doc, its loss then): visible documents without a row
        self._pending = set()   # rows with loss +inf (new / running / failed)
        self._owner = None      # weakref to the Trials synced
        self._epoch = None
        self._jgen = None
        self._jpos = 0
        self._seen = 0          # visible documents consumed
        self._vals_dirty = 0    # rows >= this differ from the device copy
        self._loss_dirty = 0
        self._dev = None        # weakref to the plan holding the device copy
        self._plain = True      # rows == visible documents, integer tids ascending

    # -- per-document rows -----------------------------------------------------
    def _extract(self, doc):
        """(tid, vals row, active row) of a document, cached per object."""
        key = id(doc)
        hit = self._cache.get(key)
        if hit is not None and hit[0] is doc:
            return hit[1], hit[2], hit[3]
        misc = doc['misc']
        tid = misc.get('from_tid', doc['tid'])
        v = np.zeros(self.P)
        a = np.zeros(self.P, dtype=np.uint8)
        ix, vx = misc['idxs'], misc['vals']
        for i, lab in enumerate(self.labels):
            t = ix[lab]
            if t and t[0] == tid:
                v[i] = float(vx[lab][0])
                a[i] = 1
        self._cache[key] = (doc, tid, v, a)
        return tid, v, a

    def _put_row(self, r, tid, loss, v, a, doc):
        self.losses[r] = loss
        self.vals[:, r] = v
        self.active[:, r] = a
        if r == len(self.docs):
            self.docs.append(doc)
            self.tids.append(tid)
        else:
            self.docs[r] = doc
            self.tids[r] = tid
        if loss == math.inf:
            self._pending.add(r)
        else:
            self._pending.discard(r)

    # -- sync ----------------------------------------------------------------
    def sync(self, trials):
        """Bring the columns up to date with ``trials.trials``."""
        view = trials.trials
        store = getattr(trials, '_store', None)
        journal = store.journal if store is not None else None
        # snapshot the journal (list, then gen: see _Journal.reset); entries
        # logged after the snapshot are read by the next sync
        jdocs = journal.docs if journal is not None else None
        jgen = journal.gen if journal is not None else None
        jlen = len(jdocs) if jdocs is not None else 0
        fresh = jgen is not None and jgen == self._jgen
        changed = jdocs[self._jpos:jlen] if fresh else []
        if fresh:
            for doc in changed:
                self._cache.pop(id(doc), None)  # misc / tid may have changed
        else:
            self._cache.clear()             # unknown changes: nothing cached is trusted
        same = (fresh and self._plain and self._owner is not None and
                self._owner() is trials and
                getattr(trials, '_epoch', None) == self._epoch and len(view) >= self._seen)
        if not (same and self._incremental(view, changed)):
            self._rebuild(view)
        self._owner = weakref.ref(trials)
        self._epoch = getattr(trials, '_epoch', None)
        self._jgen = jgen
        self._jpos = jlen if fresh else 0
        self._seen = len(view)
        return self

    def _incremental(self, view, changed):
        """Apply changed and appended documents; False = needs a rebuild."""
        dom = self.domain
        done = set()
        for doc in changed:
            k = id(doc)
            if k in done:
                continue
            done.add(k)
            if k in self._dropped and self._dropped[k][0] is doc:
                # a visible document the last rebuild left out (a first NaN
                # loss, or a duplicate tid that lost the dedupe) changed: it
                # may belong in the history now
                return False
            r = self._row.get(k)
            if r is None or self.docs[r] is not doc:
                continue                        # not a row (yet): appended below
            tid, v, a = self._extract(doc)
            loss = _loss_of(dom, doc)
            if tid != self.tids[r] or loss != loss:
                return False
            if not (np.array_equal(v, self.vals[:, r]) and np.array_equal(a, self.active[:, r])):
                self._vals_dirty = min(self._vals_dirty, r)
            if loss != self.losses[r]:
                self._loss_dirty = min(self._loss_dirty, r)
            self._put_row(r, tid, loss, v, a, doc)
        # safety net for results mutated in place (no journal entry): the
        # losses of every row still waiting for one (+inf) are re-read, and
        # those of every document the last rebuild left out (a NaN loss that
        # is now a number, a duplicate tid whose loss now wins the dedupe) --
        # all of them, however many: the reference re-reads every document on
        # every call (tpe.py:820-848), so a skipped check would be a silent
        # divergence; the cost is one loss lookup per such document
        for d, l0 in self._dropped.values():
            loss = _loss_of(dom, d)
            if not (loss == l0 or (loss != loss and l0 != l0)):
                return False
        for r in list(self._pending):
            loss = _loss_of(dom, self.docs[r])
            if loss != loss:
                return False
            if loss != math.inf:
                self.losses[r] = loss
                self._pending.discard(r)
                self._loss_dirty = min(self._loss_dirty, r)
        new = view[self._seen:]
        self._grow(self.n + len(new))
        last = self.tids[-1] if self.tids else None
        for doc in new:
            if 'from_tid' in doc['misc']:
                return False
            tid, v, a = self._extract(doc)
            if not _is_int_tid(tid) or (last is not None and tid <= last):
                return False
            loss = _loss_of(dom, doc)
            if loss != loss:
                return False
            r = self.n
            self._put_row(r, tid, loss, v, a, doc)
            self._row[id(doc)] = r
            self.n = r + 1
            last = tid
        return True

    def _rebuild(self, view):
        """Full rebuild with the reference's dedupe and tid sort."""
        dom = self.domain
        dev = self._dev
        self._forget()
        self._dev = dev
        best = {}               # tid -> [loss, doc]
        seen = {}               # id(doc) -> its loss now
        for doc in view:
            tid = doc['misc'].get('from_tid', doc['tid'])
            loss = _loss_of(dom, doc)
            seen[id(doc)] = loss
            cur = best.get(tid)
            if cur is None:
                best[tid] = [loss, doc if loss == loss else None]
            elif loss <= cur[0]:
                cur[0], cur[1] = loss, doc
        rows = sorted(((t, e[0], e[1]) for t, e in best.items() if e[1] is not None),
                      key=lambda z: z[0])
        kept = {id(e[2]) for e in rows}
        self._dropped = {id(d): (d, seen[id(d)]) for d in view if id(d) not in kept}
        self._grow(len(rows))
        plain = True
        for r, (tid, loss, doc) in enumerate(rows):
            _, v, a = self._extract(doc)
            self._put_row(r, tid, loss, v, a, doc)
            self._row[id(doc)] = r
            plain &= 'from_tid' not in doc['misc']
        self.n = len(rows)
        # rows that are not 1:1 documents (merged from_tid results): every
        # later sync rebuilds
        self._plain = plain and all(_is_int_tid(t) for t in self.tids)
        self._vals_dirty = self._loss_dirty = 0

    # -- views ----------------------------------------------------------------
    def columns(self):
        """(tids, losses[n], vals[P, n], active[P, n]) copies."""
        n = self.n
        return (list(self.tids), self.losses[:n].copy(), self.vals[:, :n].copy(),
                self.active[:, :n].copy())

    # -- device copy ------------------------------------------------------------
    def push(self, plan):
        """Copy the rows and losses that changed since the last push into
        ``plan``'s device history."""
        if self._dev is None or self._dev() is not plan or \
                getattr(plan, '_history_owner', None) is not self:
            self._vals_dirty = self._loss_dirty = 0
        r0 = min(self._vals_dirty, self.n)
        l0 = min(self._loss_dirty, r0, self.n)
        plan.update_history(self.n, r0, self.vals, self.active, self.cap, l0, self.losses)
        plan._history_owner = self
        self._dev = weakref.ref(plan)
        self._vals_dirty = self._loss_dirty = self.n
        return self
