"""fmin driver (hyperopt/fmin.py) -- same signature and seeding semantics.

Each call of ``algo(new_ids, domain, trials, seed)`` gets
``rstate.randint(2 ** 31 - 1)`` exactly as the reference does
(hyperopt/fmin.py:155-156), so a reference user's seeds reproduce.
"""
from __future__ import annotations

import functools
import logging
import os
import sys

import numpy as np

from . import base
from . import expr as _expr

logger = logging.getLogger(__name__)


def fmin_pass_expr_memo_ctrl(f):
    f.fmin_pass_expr_memo_ctrl = True
    return f


def partial(fn, **kwargs):
    rval = functools.partial(fn, **kwargs)
    if hasattr(fn, 'fmin_pass_expr_memo_ctrl'):
        rval.fmin_pass_expr_memo_ctrl = fn.fmin_pass_expr_memo_ctrl
    return rval


class FMinIter(object):
    """hyperopt/fmin.py:46-200 (serial evaluation; async trials poll)."""
    catch_eval_exceptions = False

    def __init__(self, algo, domain, trials, rstate, async_=None, max_queue_len=1,
                 poll_interval_secs=1.0, max_evals=sys.maxsize, verbose=0):
        self.algo = algo
        self.domain = domain
        self.trials = trials
        self.async_ = trials.async_ if async_ is None else async_
        self.poll_interval_secs = poll_interval_secs
        self.max_queue_len = max_queue_len
        self.max_evals = max_evals
        self.rstate = rstate

    def serial_evaluate(self, N=-1):
        for trial in self.trials._dynamic_trials:
            if trial['state'] == base.JOB_STATE_NEW:
                now = base.coarse_utcnow()
                trial['book_time'] = now
                trial['refresh_time'] = now
                spec = base.spec_from_misc(trial['misc'])
                ctrl = base.Ctrl(self.trials, current_trial=trial)
                try:
                    result = self.domain.evaluate(spec, ctrl)
                except Exception as e:
                    logger.info('job exception: %s' % str(e))
                    trial['state'] = base.JOB_STATE_ERROR
                    trial['misc']['error'] = (str(type(e)), str(e))
                    trial['refresh_time'] = base.coarse_utcnow()
                    if not self.catch_eval_exceptions:
                        self.trials.refresh()
                        raise
                else:
                    trial['state'] = base.JOB_STATE_DONE
                    trial['result'] = result
                    trial['refresh_time'] = base.coarse_utcnow()
                N -= 1
                if N == 0:
                    break
        self.trials.refresh()

    def block_until_done(self):
        if self.async_:
            import time
            unfinished = [base.JOB_STATE_NEW, base.JOB_STATE_RUNNING]
            while self.trials.count_by_state_unsynced(unfinished) > 0:
                time.sleep(self.poll_interval_secs)
            self.trials.refresh()
        else:
            self.serial_evaluate()

    def run(self, N, block_until_done=True):
        trials = self.trials
        n_queued = 0

        def get_queue_len():
            return self.trials.count_by_state_unsynced(base.JOB_STATE_NEW)

        stopped = False
        while n_queued < N:
            qlen = get_queue_len()
            while qlen < self.max_queue_len and n_queued < N:
                n_to_enqueue = min(self.max_queue_len - qlen, N - n_queued)
                new_ids = trials.new_trial_ids(n_to_enqueue)
                self.trials.refresh()
                new_trials = self.algo(new_ids, self.domain, trials,
                                       self.rstate.randint(2 ** 31 - 1))
                assert len(new_ids) >= len(new_trials)
                if len(new_trials):
                    self.trials.insert_trial_docs(new_trials)
                    self.trials.refresh()
                    n_queued += len(new_trials)
                    qlen = get_queue_len()
                else:
                    stopped = True
                    break
            if self.async_:
                import time
                time.sleep(self.poll_interval_secs)
            else:
                self.serial_evaluate()
            if stopped:
                break
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

    def exhaust(self):
        n_done = len(self.trials)
        self.run(self.max_evals - n_done, block_until_done=self.async_)
        self.trials.refresh()
        return self


def fmin(fn, space, algo, max_evals, trials=None, rstate=None, allow_trials_fmin=True,
         pass_expr_memo_ctrl=None, catch_eval_exceptions=False, verbose=0, return_argmin=True):
    """Minimize ``fn`` over ``space`` (hyperopt/fmin.py:203-321)."""
    if rstate is None:
        env_rseed = os.environ.get('HYPEROPT_FMIN_SEED', '')
        rstate = np.random.RandomState(int(env_rseed)) if env_rseed else np.random.RandomState()
    if allow_trials_fmin and hasattr(trials, 'fmin'):
        return trials.fmin(fn, space, algo=algo, max_evals=max_evals, rstate=rstate,
                           pass_expr_memo_ctrl=pass_expr_memo_ctrl, verbose=verbose,
                           catch_eval_exceptions=catch_eval_exceptions,
                           return_argmin=return_argmin)
    if trials is None:
        trials = base.Trials()
    domain = base.Domain(fn, space, pass_expr_memo_ctrl=pass_expr_memo_ctrl)
    rval = FMinIter(algo, domain, trials, max_evals=max_evals, rstate=rstate, verbose=verbose)
    rval.catch_eval_exceptions = catch_eval_exceptions
    rval.exhaust()
    if return_argmin:
        return trials.argmin


def space_eval(space, hp_assignment):
    """Point of ``space`` for an assignment {label: value} (fmin.py:324-342)."""
    return _expr.evaluate(space, hp_assignment)
