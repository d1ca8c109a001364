"""Asynchronous evaluation with a pool of worker threads: batched TPE
suggestions feeding a job queue.

The reference evaluates asynchronously through MongoDB: the driver keeps
``max_queue_len`` NEW jobs queued (hyperopt/fmin.py:131-185) and worker
processes reserve them atomically (mongoexp.py:449-482, 997-1099) while
suggestions are computed one at a time (tpe.py:812).  ``ThreadTrials`` is the
same protocol in one process: the store *is* the queue, ``n_workers``
threads reserve NEW documents (NEW -> RUNNING under the store lock, owner =
the worker), evaluate them with the driver's Domain and write DONE / ERROR
back.  Pending trials carry loss +inf into TPE exactly as pending Mongo jobs
do, and the driver asks ``tpe.suggest`` for every free queue slot at once,
so the GPU serves them as one batched call::

    trials = ThreadTrials(n_workers=8)
    fmin(fn, space, algo=tpe.suggest, max_evals=1000, trials=trials,
         max_queue_len=8)
"""
from __future__ import annotations

import logging
import threading

from . import status as S
from .domain import Ctrl
from .trials import Trials, coarse_utcnow, SONify

logger = logging.getLogger(__name__)


class ThreadTrials(Trials):
    """A Trials whose NEW documents are evaluated by worker threads."""

    async_ = True

    def __init__(self, n_workers=4, exp_key=None, refresh=True, catch_eval_exceptions=True):
        super().__init__(exp_key=exp_key, refresh=refresh)
        self.n_workers = int(n_workers)
        self.catch_eval_exceptions = catch_eval_exceptions
        self.poll_interval_secs = 0.005
        self._cv = threading.Condition()
        self._domain = None
        self._threads = []
        self._stop = False
        self.errors = []

    # -- driver side ---------------------------------------------------------
    def attach_domain(self, domain):
        """Called by FMinIter for asynchronous trials (the reference pickles
        the domain into the attachments for its Mongo workers, fmin.py:70-77)."""
        with self._cv:
            self._domain = domain
            if not self._threads:
                for i in range(self.n_workers):
                    t = threading.Thread(target=self._work, args=('thread-%d' % i,), daemon=True)
                    t.start()
                    self._threads.append(t)

    def _insert_trial_docs(self, docs):
        with self._cv:
            out = super()._insert_trial_docs(docs)
            self._cv.notify_all()
        return out

    def wait_for_progress(self, timeout):
        """Block until a worker finishes a job (or timeout)."""
        with self._cv:
            self._cv.wait(timeout)

    def shutdown(self):
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        for t in self._threads:
            t.join()
        self._threads = []
        self._stop = False

    # -- worker side ------------------------------------------------------------
    def _reserve(self, owner):
        """The oldest NEW document of this experiment, marked RUNNING."""
        st = self._store
        states = st.state.view()
        for r in (states == S.JOB_STATE_NEW).nonzero()[0]:
            doc = st.docs[r]
            if self._exp_key is not None and doc.get('exp_key') != self._exp_key:
                continue
            doc['state'] = S.JOB_STATE_RUNNING
            doc['owner'] = owner
            doc['book_time'] = coarse_utcnow()
            return doc
        return None

    def _work(self, owner):
        while True:
            with self._cv:
                doc = None
                while not self._stop:
                    doc = self._reserve(owner)
                    if doc is not None:
                        break
                    self._cv.wait(0.5)
                if self._stop:
                    return
                domain = self._domain
            spec = {k: v[0] for k, v in doc['misc']['vals'].items() if v}
            try:
                res = domain.evaluate(spec, Ctrl(self, current_trial=doc))
                err = None
            except Exception as e:      # recorded like a failed Mongo job
                res, err = None, e
            with self._cv:
                if err is None:
                    doc['result'] = SONify(res)
                    doc['state'] = S.JOB_STATE_DONE
                else:
                    logger.info('job exception: %s', err)
                    doc['misc']['error'] = (str(type(err)), str(err))
                    doc['state'] = S.JOB_STATE_ERROR
                    self.errors.append(err)
                doc['refresh_time'] = coarse_utcnow()
                self._cv.notify_all()
