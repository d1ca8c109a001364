"""Domain (objective + compiled search space) and Ctrl (the handle an
objective gets on its trial) -- hyperopt/base.py:653-906 interface.

The space is compiled once into per-hyperparameter descriptors
(``space.compile_space``) instead of a vectorised pyll graph; a trial's
configuration is evaluated through ``expr.evaluate``.
"""
from __future__ import annotations

import logging

import numpy as np

from . import expr as _expr
from . import status as S
from .space import compile_space

logger = logging.getLogger(__name__)


class InvalidResultStatus(ValueError):
    """The objective returned a status outside STATUS_STRINGS."""


class InvalidLoss(ValueError):
    """A STATUS_OK result without a float-convertible loss."""


def _as_result(rval):
    """The objective's return value as a result document (base.py:845-858):
    a bare number is an OK loss; a dict must carry a known status and, when
    OK, a float loss."""
    if isinstance(rval, (float, int, np.number)):
        return {'loss': float(rval), 'status': S.STATUS_OK}
    res = dict(rval)
    if res['status'] not in S.STATUS_STRINGS:
        raise InvalidResultStatus(res)
    if res['status'] == S.STATUS_OK:
        try:
            res['loss'] = float(res['loss'])
        except (TypeError, KeyError):
            raise InvalidLoss(res)
    return res


class Domain(object):
    """An objective ``fn`` over the search space ``expr``."""

    def __init__(self, fn, expr, workdir=None, pass_expr_memo_ctrl=None, name=None,
                 loss_target=None):
        self.fn = fn
        self.expr = expr
        self.workdir = workdir
        self.name = name
        self.loss_target = loss_target
        self.pass_expr_memo_ctrl = (getattr(fn, 'fmin_pass_expr_memo_ctrl', False)
                                    if pass_expr_memo_ctrl is None else pass_expr_memo_ctrl)
        self.space = compile_space(expr)
        self.params = {h.label: h.node for h in self.space.hps}
        self.cmd = ('domain_attachment', 'FMinIter_Domain')

    def __getstate__(self):
        # the per-domain engine state (device plan, history mirrors, a lock)
        # stays with the process; a pickled Domain starts without it
        d = dict(self.__dict__)
        d.pop('_tpe_state', None)
        return d

    def memo_from_config(self, config):
        return dict(config)

    def evaluate(self, config, ctrl, attach_attachments=True):
        """Run the objective on one configuration {label: value}."""
        if self.pass_expr_memo_ctrl:
            out = self.fn(expr=self.expr, memo=self.memo_from_config(config), ctrl=ctrl)
        else:
            out = self.fn(_expr.evaluate(self.expr, config))
        res = _as_result(out)
        if attach_attachments:
            for k, v in res.pop('attachments', {}).items():
                ctrl.attachments[k] = v
        return res

    def short_str(self):
        return 'Domain{%s}' % str(self.fn)

    # -- result accessors (base.py:874-906) --------------------------------
    def loss(self, result, config=None):
        return result.get('loss', None)

    def loss_variance(self, result, config=None):
        return result.get('loss_variance', 0.0)

    def true_loss(self, result, config=None):
        return result['true_loss'] if 'true_loss' in result else self.loss(result, config=config)

    def true_loss_variance(self, config=None):
        raise NotImplementedError()

    def status(self, result, config=None):
        return result['status']

    def new_result(self):
        return {'status': S.STATUS_NEW}


class Ctrl(object):
    """What an objective sees of its running trial (base.py:653-708)."""
    info = logger.info
    warn = logger.warning
    error = logger.error
    debug = logger.debug

    def __init__(self, trials, current_trial=None):
        if trials is None:
            from .trials import Trials
            trials = Trials()
        self.trials = trials
        self.current_trial = current_trial

    def checkpoint(self, r=None):
        """Publish a partial result of the current trial."""
        if not any(d is self.current_trial for d in self.trials.trials):
            raise AssertionError('current trial is not a visible trial')
        if r is not None:
            self.current_trial['result'] = r

    @property
    def attachments(self):
        return self.trials.trial_attachments(trial=self.current_trial)

    def inject_results(self, specs, results, miscs, new_tids=None):
        """Insert finished trials derived from the current one (their misc
        gets from_tid = the current tid, so TPE merges them into it)."""
        src = self.current_trial
        if src is None:
            raise AssertionError('no current trial')
        if not len(specs) == len(results) == len(miscs):
            raise AssertionError('specs / results / miscs differ in length')
        tids = self.trials.new_trial_ids(len(specs)) if new_tids is None else new_tids
        docs = self.trials.source_trial_docs(tids=tids, specs=specs, results=results,
                                             miscs=miscs, sources=[src])
        for d in docs:
            d['state'] = S.JOB_STATE_DONE
        return self.trials.insert_trial_docs(docs)
