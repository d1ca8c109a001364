"""Columnar trial store and incremental history (no GPU): the journal sees
every reassignment, refresh/visibility/id allocation follow the reference,
and the incrementally synced history -- including its row-by-row device copy
-- always equals a from-scratch assembly with the reference's semantics
(tpe.py:820-848)."""
import copy
import math
import pickle

import numpy as np
import pytest

import hyperopt_amd as H
from hyperopt_amd import hp, rand, Trials, trials_from_docs
from hyperopt_amd.base import Domain, miscs_to_idxs_vals, miscs_update_idxs_vals, TrialDoc
from hyperopt_amd.history import TrialHistory


def reference_history(domain, trials):
    """Direct restatement of tpe.py:820-848 + base.py:187-202 on the docs."""
    best_loss, best_doc = {}, {}
    for doc in trials.trials:
        tid = doc['misc'].get('from_tid', doc['tid'])
        loss = domain.loss(doc['result'], doc['spec'])
        loss = float('inf') if loss is None else float(loss)
        best_loss.setdefault(tid, loss)
        if loss <= best_loss[tid]:
            best_loss[tid] = loss
            best_doc[tid] = doc
    tids = sorted(best_doc)
    labels = domain.space.labels
    vals = np.zeros((len(labels), len(tids)))
    act = np.zeros((len(labels), len(tids)), dtype=np.uint8)
    for j, t in enumerate(tids):
        m = best_doc[t]['misc']
        for i, lab in enumerate(labels):
            ix = m['idxs'][lab]
            if ix and ix[0] == t:
                vals[i, j] = m['vals'][lab][0]
                act[i, j] = 1
    return tids, np.array([best_loss[t] for t in tids]), vals, act


class FakePlan(object):
    """Host stand-in for the device history: applies update_history calls."""
    def __init__(self, P, cap):
        self.max_trials = cap
        self.vals = np.full((P, cap), np.nan)
        self.active = np.full((P, cap), 7, dtype=np.uint8)
        self.losses = np.full(cap, np.nan)
        self.n = 0
        self.rows_copied = 0

    def update_history(self, n, row0, vals, active, ld, loss0, losses, stream=None):
        self.vals[:, row0:n] = vals[:, row0:n]
        self.active[:, row0:n] = active[:, row0:n]
        self.losses[loss0:n] = losses[loss0:n]
        self.rows_copied += n - row0
        self.n = n


def check(dom, t, hist, plan=None):
    want = reference_history(dom, t)
    got = hist.sync(t).columns()
    assert got[0] == want[0]
    np.testing.assert_array_equal(got[1], want[1])
    np.testing.assert_array_equal(got[2], want[2])
    np.testing.assert_array_equal(got[3], want[3])
    if plan is not None:
        hist.push(plan)
        n = plan.n
        assert n == len(want[0])
        np.testing.assert_array_equal(plan.losses[:n], want[1])
        np.testing.assert_array_equal(plan.vals[:, :n], want[2])
        np.testing.assert_array_equal(plan.active[:, :n], want[3])


SPACE = {'a': hp.uniform('a', 0, 1), 'c': hp.choice('c', [hp.normal('n', 0, 1), 3]),
         'q': hp.quniform('q', 0, 10, 1)}


def test_journal_records_reassignments():
    t = Trials()
    dom = Domain(lambda x: 0, SPACE)
    docs = rand.suggest([0, 1], dom, t, 0)
    t.insert_trial_docs(docs)
    t.refresh()
    j = t._store.journal
    n0 = len(j.docs)
    d = t.trials[0]
    d['result'] = {'status': 'ok', 'loss': 1.0}
    d['state'] = H.JOB_STATE_DONE
    d['book_time'] = None          # untracked field
    d.update(misc=d['misc'])
    assert [x is d for x in j.docs[n0:]] == [True] * 3
    assert t.count_by_state_unsynced(H.JOB_STATE_DONE) == 1
    assert t.count_by_state_synced([H.JOB_STATE_NEW, H.JOB_STATE_DONE]) == 2


def test_refresh_visibility_ids_and_epoch():
    t = Trials()
    dom = Domain(lambda x: 0, SPACE)
    t.insert_trial_docs(rand.suggest([5, 6, 7], dom, t, 1))
    t.refresh()
    assert t.tids == [5, 6, 7]
    assert t.new_trial_ids(2) == [3, 4]     # len(ids) onwards, as in the reference
    e0 = t._epoch
    t.insert_trial_docs(rand.suggest([8], dom, t, 2))
    t.refresh()
    assert t._epoch == e0 and t.tids == [5, 6, 7, 8]
    t._dynamic_trials[1]['state'] = H.JOB_STATE_ERROR
    t.refresh()
    assert t._epoch != e0 and t.tids == [5, 7, 8]
    v = t.view(exp_key='other')
    assert len(v) == 0


def test_doc_copies_and_pickles_detached():
    t = Trials()
    dom = Domain(lambda x: 0, SPACE)
    t.insert_trial_docs(rand.suggest([0], dom, t, 3))
    t.refresh()
    d = t.trials[0]
    for c in (copy.copy(d), copy.deepcopy(d), pickle.loads(pickle.dumps(d))):
        assert isinstance(c, TrialDoc) and c == d and c._store is None
        c['state'] = 2                # no journal entry in the original store
    assert len(t._store.journal.docs) == 0
    d2 = Domain(abs, SPACE)
    d2._tpe_state = object()
    assert "_tpe_state" not in pickle.loads(pickle.dumps(d2)).__dict__


def test_miscs_codec_roundtrip():
    miscs = [{'tid': i, 'cmd': None} for i in range(3)]
    idxs = {'x': [0, 2], 'y': [1]}
    vals = {'x': [1.5, 2.5], 'y': [7]}
    miscs_update_idxs_vals(miscs, idxs, vals)
    assert miscs[1]['idxs'] == {'x': [], 'y': [1]}
    i2, v2 = miscs_to_idxs_vals(miscs)
    assert i2 == idxs and v2 == vals
    m = [{'tid': 9}]
    miscs_update_idxs_vals(m, {'x': [100, 3]}, {'x': [1.0, 2.0]}, idxs_map={100: 9},
                           assert_all_vals_used=False)
    assert m[0]['vals'] == {'x': [1.0]}
    with pytest.raises(KeyError):
        miscs_update_idxs_vals([{'tid': 0}], {'x': [1]}, {'x': [0.5]})


@pytest.mark.parametrize('seed', range(6))
def test_incremental_history_equals_reference_assembly(seed):
    """Random fmin-like traffic (appends, results, failures, errors, in-place
    result edits, injected from_tid results, NaN losses, out-of-order tids):
    after every step the synced columns and the device copy built from the
    pushed rows equal the reference's assembly."""
    rng = np.random.RandomState(seed)
    dom = Domain(lambda x: 0, SPACE)
    t = Trials()
    hist = TrialHistory(dom)
    plan = FakePlan(len(dom.space.labels), 4096)
    next_id = 0
    for step in range(120):
        op = rng.randint(12)
        if op < 5 or len(t._dynamic_trials) < 3:
            k = 1 + rng.randint(3)
            ids = list(range(next_id, next_id + k))
            next_id += k
            if rng.rand() < 0.05:
                ids = [next_id + 50]     # out of order later
            t.insert_trial_docs(rand.suggest(ids, dom, t, int(rng.randint(1 << 30))))
        elif op < 8:
            new = [d for d in t._dynamic_trials if d['state'] == H.JOB_STATE_NEW]
            if new:
                d = new[rng.randint(len(new))]
                r = rng.rand()
                if r < 0.7:
                    d['result'] = {'status': 'ok', 'loss': float(rng.randint(5))}
                elif r < 0.8:
                    d['result'] = {'status': 'ok', 'loss': float('nan')}
                elif r < 0.9:
                    d['result'] = {'status': 'fail'}
                else:
                    d['state'] = H.JOB_STATE_ERROR
                    continue
                d['state'] = H.JOB_STATE_DONE
        elif op == 8 and t.trials:
            d = t.trials[rng.randint(len(t.trials))]
            d['result']['loss'] = float(rng.rand())     # in place: no journal entry
            if d['state'] == H.JOB_STATE_NEW:
                d['result']['status'] = 'ok'
        elif op == 9 and t.trials:
            src = t.trials[rng.randint(len(t.trials))]
            ctrl = H.Ctrl(t, current_trial=src)
            m = copy.deepcopy(src['misc'])
            for k in ('tid', 'from_tid', 'cmd'):
                m.pop(k, None)
            ctrl.inject_results([None], [{'status': 'ok', 'loss': float(rng.rand())}], [m])
        t.refresh()
        # in-place edits of finished rows are outside the contract (the
        # reference re-reads everything); resync them like a user would
        if op == 8:
            hist = TrialHistory(dom)
        check(dom, t, hist, plan)


def test_incremental_path_copies_only_new_rows():
    dom = Domain(lambda x: 0, SPACE)
    t = Trials()
    hist = TrialHistory(dom)
    plan = FakePlan(len(dom.space.labels), 4096)
    ids = t.new_trial_ids(500)
    t.insert_trial_docs(rand.suggest(ids, dom, t, 4))
    t.refresh()
    for d in t.trials:
        d['result'] = {'status': 'ok', 'loss': 1.0}
        d['state'] = H.JOB_STATE_DONE
    check(dom, t, hist, plan)
    base = plan.rows_copied
    for i in range(20):
        (nid,) = t.new_trial_ids(1)
        t.insert_trial_docs(rand.suggest([nid], dom, t, i))
        t.refresh()
        check(dom, t, hist, plan)
        t.trials[-1]['result'] = {'status': 'ok', 'loss': float(i)}
        t.trials[-1]['state'] = H.JOB_STATE_DONE
    assert plan.rows_copied - base == 20
    assert hist._plain


def test_thread_trials_async_fmin_with_rand():
    """Asynchronous evaluation by worker threads (the Mongo worker protocol in
    process): every trial evaluated once, queue bound respected."""
    seen = []

    def fn(x):
        seen.append(x)
        return (x - 1) ** 2

    t = H.ThreadTrials(n_workers=3)
    try:
        H.fmin(fn, hp.uniform('x', -3, 3), algo=rand.suggest, max_evals=40, trials=t,
               rstate=np.random.RandomState(0), max_queue_len=3)
    finally:
        t.shutdown()
    assert len(t) == 40 and len(seen) == 40
    assert all(d['state'] == H.JOB_STATE_DONE for d in t.trials)
    assert {d['owner'] for d in t.trials} <= {'thread-0', 'thread-1', 'thread-2'}
    assert t.best_trial['result']['loss'] == min(t.losses())


def test_fmin_batched_queue_uses_all_ids():
    """max_queue_len=S: the algorithm gets S ids per call (serial trials)."""
    calls = []

    def algo(new_ids, domain, trials, seed):
        calls.append(len(new_ids))
        return rand.suggest(new_ids, domain, trials, seed)

    t = Trials()
    H.fmin(lambda x: x, hp.uniform('x', 0, 1), algo=algo, max_evals=20, trials=t,
           rstate=np.random.RandomState(0), max_queue_len=4)
    assert len(t) == 20 and calls == [4] * 5


def test_delete_all_and_refresh_cost_shape():
    dom = Domain(lambda x: 0, SPACE)
    t = Trials()
    t.insert_trial_docs(rand.suggest([0, 1, 2], dom, t, 5))
    t.refresh()
    lst = t.trials
    t.insert_trial_docs(rand.suggest([3], dom, t, 6))
    t.refresh()
    assert len(lst) == 3 and len(t.trials) == 4     # a new list per refresh
    t.delete_all()
    assert t.trials == [] and len(t) == 0
    t.insert_trial_docs(rand.suggest([9], dom, t, 7))
    t.refresh()
    assert t.tids == [9]


def test_pickled_trials_resume_with_pending_doc():
    """a Trials pickled with a queued NEW document comes
    back with its documents attached to the store, so a resumed fmin sees
    the evaluated state and finishes (the reference reads states from the
    documents, base.py:327-338)."""
    import signal
    t = Trials()
    H.fmin(lambda x: x ** 2, hp.uniform('x', -1, 1), algo=rand.suggest, max_evals=3, trials=t,
           rstate=np.random.RandomState(0))
    dom = Domain(lambda x: x ** 2, hp.uniform('x', -1, 1))
    t.insert_trial_docs(rand.suggest(t.new_trial_ids(1), dom, t, 9))   # queued, never run
    t.refresh()
    for loaded in (pickle.loads(pickle.dumps(t)), copy.deepcopy(t)):
        st = loaded._store
        assert all(d._store is st and st.docs[d._row] is d for d in st.docs)
        assert list(st.state.view()) == [d['state'] for d in st.docs]
        last = loaded.trials[-1]
        assert last['state'] == H.JOB_STATE_NEW and last._store is st
        old = signal.signal(signal.SIGALRM, lambda *a: (_ for _ in ()).throw(TimeoutError()))
        signal.alarm(30)
        try:
            H.fmin(lambda x: x ** 2, hp.uniform('x', -1, 1), algo=rand.suggest, max_evals=6,
                   trials=loaded, rstate=np.random.RandomState(1))
        finally:
            signal.alarm(0)
            signal.signal(signal.SIGALRM, old)
        assert len(loaded) == 6
        assert all(d['state'] == H.JOB_STATE_DONE for d in loaded.trials)
        assert st.state.view().tolist() == [H.JOB_STATE_DONE] * 6
    assert len(t) == 4 and t.trials[-1]['state'] == H.JOB_STATE_NEW   # original untouched


def test_dropped_document_reassigned_enters_history():
    """a tid dropped by a rebuild (its first loss NaN) whose
    result is later reassigned to a finite loss enters the incrementally
    synced history, as a fresh assembly (the reference's per-call rebuild)
    includes it."""
    dom = Domain(lambda x: 0, SPACE)
    t = Trials()
    hist = TrialHistory(dom)
    plan = FakePlan(len(dom.space.labels), 64)
    t.insert_trial_docs(rand.suggest([0, 1, 2], dom, t, 5))
    t.refresh()
    for i, d in enumerate(t.trials):
        d['result'] = {'status': 'ok', 'loss': float('nan') if i == 1 else float(i)}
        d['state'] = H.JOB_STATE_DONE
    check(dom, t, hist, plan)
    assert hist.tids == [0, 2]
    t.insert_trial_docs(rand.suggest([3], dom, t, 6))
    t.refresh()
    t.trials[3]['result'] = {'status': 'ok', 'loss': 0.5}
    t.trials[3]['state'] = H.JOB_STATE_DONE
    t.trials[1]['result'] = {'status': 'ok', 'loss': 0.25}
    check(dom, t, hist, plan)
    assert hist.tids == [0, 1, 2, 3]


def test_dropped_document_mutated_in_place_enters_history():
    """the same document's loss changed in place
    (doc['result']['loss'] = x, no journal entry) also enters the history:
    the few dropped documents' losses are re-read on every sync."""
    dom = Domain(lambda x: 0, SPACE)
    t = Trials()
    hist = TrialHistory(dom)
    plan = FakePlan(len(dom.space.labels), 64)
    t.insert_trial_docs(rand.suggest([0, 1, 2], dom, t, 5))
    t.refresh()
    for i, d in enumerate(t.trials):
        d['result'] = {'status': 'ok', 'loss': float('nan') if i == 1 else float(i)}
        d['state'] = H.JOB_STATE_DONE
    check(dom, t, hist, plan)
    assert hist.tids == [0, 2]
    t.trials[1]['result']['loss'] = 0.25          # in place: no journal entry
    check(dom, t, hist, plan)
    assert hist.tids == [0, 1, 2]


def test_many_dropped_and_pending_documents_mutated_in_place():
    """more than 64 dropped documents (NaN losses) and more than
    64 pending (+inf) rows, each result then changed in place (no journal
    entry): every one enters the incrementally synced history with its new
    loss, as the reference's per-call reassembly would have it."""
    dom = Domain(lambda x: 0, SPACE)
    t = Trials()
    hist = TrialHistory(dom)
    plan = FakePlan(len(dom.space.labels), 512)
    n = 300
    t.insert_trial_docs(rand.suggest(list(range(n)), dom, t, 5))
    t.refresh()
    for i, d in enumerate(t.trials):
        if i % 3 == 0:
            d['result'] = {'status': 'ok', 'loss': float('nan')}     # dropped (100)
            d['state'] = H.JOB_STATE_DONE
        elif i % 3 == 1:
            d['result'] = {'status': 'ok', 'loss': float(i)}
            d['state'] = H.JOB_STATE_DONE
        # i % 3 == 2: left NEW, loss +inf (pending, 100 rows)
    check(dom, t, hist, plan)
    assert len(hist._dropped) == 100 and len(hist._pending) == 100
    for i, d in enumerate(t.trials):
        if i % 3 != 1:
            d['result']['loss'] = 0.5 * i               # in place: no journal entry
    check(dom, t, hist, plan)
    assert hist.tids == list(range(n))
    assert np.array_equal(hist.losses[:n], [0.5 * i if i % 3 != 1 else float(i)
                                            for i in range(n)])
