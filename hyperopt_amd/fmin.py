"""The optimisation driver: ``fmin`` and its iterator ``FMinIter``.

Same contract as hyperopt/fmin.py:46-342 -- every ``algo`` call receives
``rstate.randint(2 ** 31 - 1)`` as its seed, new trial ids come from
``trials.new_trial_ids`` and evaluation is serial unless the trials object
is asynchronous -- so a reference user's seeds reproduce their runs.

Beyond the reference, ``max_queue_len`` is exposed by ``fmin``: with
``max_queue_len = S > 1`` the algorithm is asked for S suggestions at once
(``tpe.suggest`` then serves them from one batched engine call) and the
batch is evaluated before the next one is requested.
"""
from __future__ import annotations

import functools
import logging
import os
import sys
import time

import numpy as np

from . import base
from . import expr as _expr
from . import status as S

logger = logging.getLogger(__name__)


def fmin_pass_expr_memo_ctrl(f):
    """Mark ``f`` to be called as f(expr=, memo=, ctrl=) by Domain.evaluate."""
    f.fmin_pass_expr_memo_ctrl = True
    return f


def partial(fn, **kwargs):
    """functools.partial that keeps the fmin_pass_expr_memo_ctrl mark."""
    p = functools.partial(fn, **kwargs)
    if hasattr(fn, 'fmin_pass_expr_memo_ctrl'):
        p.fmin_pass_expr_memo_ctrl = fn.fmin_pass_expr_memo_ctrl
    return p


class FMinIter(object):
    """Suggest -> insert -> evaluate loop over one Domain and Trials."""

    catch_eval_exceptions = False

    def __init__(self, algo, domain, trials, rstate, async_=None, max_queue_len=1,
                 poll_interval_secs=1.0, max_evals=sys.maxsize, verbose=0):
        self.algo = algo
        self.domain = domain
        self.trials = trials
        self.rstate = rstate
        self.async_ = getattr(trials, 'async_', False) if async_ is None else async_
        self.max_queue_len = max(1, int(max_queue_len))
        self.poll_interval_secs = poll_interval_secs
        self.max_evals = max_evals
        self.verbose = verbose
        if self.async_:
            # asynchronous trials need the domain on the worker side: in
            # process (ThreadTrials) or pickled into the attachments the way
            # the reference hands it to Mongo workers (fmin.py:70-77)
            attach = getattr(trials, 'attach_domain', None)
            if attach is not None:
                attach(domain)
            else:
                import pickle
                trials.attachments['FMinIter_Domain'] = pickle.dumps(domain, protocol=-1)

    # -- evaluation ----------------------------------------------------------
    def _evaluate(self, doc):
        """Run the objective on one NEW document, writing its outcome back."""
        t = base.coarse_utcnow()
        doc['book_time'] = doc['refresh_time'] = t
        ctrl = base.Ctrl(self.trials, current_trial=doc)
        try:
            result = self.domain.evaluate(base.spec_from_misc(doc['misc']), ctrl)
        except Exception as e:
            logger.info('job exception: %s', e)
            doc['misc']['error'] = (str(type(e)), str(e))
            doc['state'] = S.JOB_STATE_ERROR     # hidden from trials.trials after refresh
            doc['refresh_time'] = base.coarse_utcnow()
            if not self.catch_eval_exceptions:
                self.trials.refresh()
                raise
            return
        doc['result'] = result
        doc['state'] = S.JOB_STATE_DONE
        doc['refresh_time'] = base.coarse_utcnow()

    def serial_evaluate(self, N=-1):
        """Evaluate up to N (all if N < 0) NEW documents in insertion order."""
        todo = [d for d in self.trials._dynamic_trials if d['state'] == S.JOB_STATE_NEW]
        if N >= 0:
            todo = todo[:N]
        for d in todo:
            self._evaluate(d)
        self.trials.refresh()

    def _pause(self):
        """Let asynchronous workers make progress."""
        wait = getattr(self.trials, 'wait_for_progress', None)
        if wait is not None:
            wait(self.poll_interval_secs)
        else:
            time.sleep(self.poll_interval_secs)

    def _wait_for_workers(self):
        busy = [S.JOB_STATE_NEW, S.JOB_STATE_RUNNING]
        while self.trials.count_by_state_unsynced(busy) > 0:
            self._pause()
        self.trials.refresh()

    def block_until_done(self):
        if self.async_:
            self._wait_for_workers()
        else:
            self.serial_evaluate()

    # -- proposing -------------------------------------------------------------
    def _queued(self):
        return self.trials.count_by_state_unsynced(S.JOB_STATE_NEW)

    def _propose(self, n):
        """Ask the algorithm for n suggestions; store what it returns.
        Returns how many it gave (0 = the algorithm is exhausted)."""
        ids = self.trials.new_trial_ids(n)
        self.trials.refresh()
        docs = self.algo(ids, self.domain, self.trials, self.rstate.randint(2 ** 31 - 1))
        if len(docs) > len(ids):
            raise AssertionError('algo returned more trials than ids')
        if docs:
            self.trials.insert_trial_docs(docs)
            self.trials.refresh()
        return len(docs)

    def run(self, N, block_until_done=True):
        """Queue and evaluate N more trials (fewer if the algorithm stops)."""
        left = N
        exhausted = False
        while left > 0 and not exhausted:
            room = self.max_queue_len - self._queued()
            while room > 0 and left > 0:
                got = self._propose(min(room, left))
                if got == 0:
                    exhausted = True
                    break
                left -= got
                room = self.max_queue_len - self._queued()
            if self.async_:
                self._pause()                         # workers fill the results
            else:
                self.serial_evaluate()
        if block_until_done:
            self.block_until_done()
            self.trials.refresh()

    def __iter__(self):
        return self

    def __next__(self):
        self.run(1, block_until_done=self.async_)
        if len(self.trials) >= self.max_evals:
            raise StopIteration()
        return self.trials

    next = __next__

    def exhaust(self):
        self.run(self.max_evals - len(self.trials), block_until_done=self.async_)
        self.trials.refresh()
        return self


def fmin(fn, space, algo, max_evals, trials=None, rstate=None, allow_trials_fmin=True,
         pass_expr_memo_ctrl=None, catch_eval_exceptions=False, verbose=0, return_argmin=True,
         max_queue_len=1):
    """Minimise ``fn`` over ``space`` with ``algo`` in ``max_evals`` trials
    (hyperopt/fmin.py:203-321); returns ``trials.argmin``.

    ``rstate`` defaults to RandomState($HYPEROPT_FMIN_SEED) when that is set.
    ``max_queue_len`` > 1 asks the algorithm for that many suggestions per
    call (batched TPE suggestions on the GPU)."""
    if rstate is None:
        env = os.environ.get('HYPEROPT_FMIN_SEED', '')
        rstate = np.random.RandomState(int(env)) if env else np.random.RandomState()
    if allow_trials_fmin and hasattr(trials, 'fmin'):
        return trials.fmin(fn, space, algo=algo, max_evals=max_evals, rstate=rstate,
                           pass_expr_memo_ctrl=pass_expr_memo_ctrl, verbose=verbose,
                           catch_eval_exceptions=catch_eval_exceptions,
                           return_argmin=return_argmin, max_queue_len=max_queue_len)
    trials = base.Trials() if trials is None else trials
    domain = base.Domain(fn, space, pass_expr_memo_ctrl=pass_expr_memo_ctrl)
    it = FMinIter(algo, domain, trials, rstate=rstate, max_evals=max_evals, verbose=verbose,
                  max_queue_len=max_queue_len)
    it.catch_eval_exceptions = catch_eval_exceptions
    it.exhaust()
    return trials.argmin if return_argmin else None


def space_eval(space, hp_assignment):
    """The point of ``space`` an assignment {label: value} selects
    (fmin.py:324-342)."""
    return _expr.evaluate(space, hp_assignment)
