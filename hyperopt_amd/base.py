"""Trials / Domain / Ctrl -- host bookkeeping with the reference's interface.

Mirrors hyperopt/base.py (Trials :217-638, Ctrl :641-708, Domain :711-906,
miscs helpers :156-214) so code written against the reference's trial
documents keeps working.  The search space is compiled once per Domain
(space.compile_space) instead of being vectorized as a pyll graph.
"""
from __future__ import annotations

import datetime
import logging

import numpy as np

from . import expr as _expr
from .space import compile_space, DuplicateLabel  # noqa: F401  (re-export)

logger = logging.getLogger(__name__)

STATUS_NEW = 'new'
STATUS_RUNNING = 'running'
STATUS_SUSPENDED = 'suspended'
STATUS_OK = 'ok'
STATUS_FAIL = 'fail'
STATUS_STRINGS = ('new', 'running', 'suspended', 'ok', 'fail')

JOB_STATE_NEW = 0
JOB_STATE_RUNNING = 1
JOB_STATE_DONE = 2
JOB_STATE_ERROR = 3
JOB_STATES = [JOB_STATE_NEW, JOB_STATE_RUNNING, JOB_STATE_DONE, JOB_STATE_ERROR]

TRIAL_KEYS = ['tid', 'spec', 'result', 'misc', 'state', 'owner', 'book_time',
              'refresh_time', 'exp_key']
TRIAL_MISC_KEYS = ['tid', 'cmd', 'idxs', 'vals']


class InvalidTrial(ValueError):
    pass


class InvalidResultStatus(ValueError):
    pass


class InvalidLoss(ValueError):
    pass


def coarse_utcnow():
    now = datetime.datetime.utcnow()
    return now.replace(microsecond=(now.microsecond // 1000) * 1000)


def SONify(arg, memo=None):
    """numpy scalars/arrays -> plain Python (hyperopt/base.py:108-150)."""
    if isinstance(arg, np.floating):
        return float(arg)
    if isinstance(arg, np.integer):
        return int(arg)
    if isinstance(arg, np.bool_):
        return bool(arg)
    if isinstance(arg, np.ndarray):
        return SONify(arg.item()) if arg.ndim == 0 else [SONify(a) for a in arg]
    if isinstance(arg, (list, tuple)):
        return type(arg)(SONify(a) for a in arg)
    if isinstance(arg, dict):
        return {SONify(k): SONify(v) for k, v in arg.items()}
    return arg


def miscs_update_idxs_vals(miscs, idxs, vals, assert_all_vals_used=True, idxs_map=None):
    """hyperopt/base.py:156-184."""
    if idxs_map is None:
        idxs_map = {}
    assert set(idxs.keys()) == set(vals.keys())
    misc_by_id = {m['tid']: m for m in miscs}
    for m in miscs:
        m['idxs'] = {key: [] for key in idxs}
        m['vals'] = {key: [] for key in idxs}
    for key in idxs:
        assert len(idxs[key]) == len(vals[key])
        for tid, val in zip(idxs[key], vals[key]):
            tid = idxs_map.get(tid, tid)
            if assert_all_vals_used or tid in misc_by_id:
                misc_by_id[tid]['idxs'][key] = [tid]
                misc_by_id[tid]['vals'][key] = [val]
    return miscs


def miscs_to_idxs_vals(miscs, keys=None):
    """hyperopt/base.py:187-202."""
    if keys is None:
        if len(miscs) == 0:
            raise ValueError('cannot infer keys from empty miscs')
        keys = miscs[0]['idxs'].keys()
    idxs = {k: [] for k in keys}
    vals = {k: [] for k in keys}
    for misc in miscs:
        for node_id in idxs:
            t_idxs = misc['idxs'][node_id]
            t_vals = misc['vals'][node_id]
            assert len(t_idxs) == len(t_vals)
            assert t_idxs == [] or t_idxs == [misc['tid']]
            idxs[node_id].extend(t_idxs)
            vals[node_id].extend(t_vals)
    return idxs, vals


def spec_from_misc(misc):
    spec = {}
    for k, v in misc['vals'].items():
        if len(v) == 0:
            pass
        elif len(v) == 1:
            spec[k] = v[0]
        else:
            raise NotImplementedError('multiple values', (k, v))
    return spec


class Trials(object):
    """In-memory trial document store (hyperopt/base.py:217-638)."""

    async_ = False

    def __init__(self, exp_key=None, refresh=True):
        self._ids = set()
        self._dynamic_trials = []
        self._exp_key = exp_key
        self.attachments = {}
        if refresh:
            self.refresh()

    def view(self, exp_key=None, refresh=True):
        rval = object.__new__(self.__class__)
        rval._exp_key = exp_key
        rval._ids = self._ids
        rval._dynamic_trials = self._dynamic_trials
        rval.attachments = self.attachments
        if refresh:
            rval.refresh()
        return rval

    def aname(self, trial, name):
        return 'ATTACH::%s::%s' % (trial['tid'], name)

    def trial_attachments(self, trial):
        outer = self

        class Attachments(object):
            def __contains__(self, name):
                return outer.aname(trial, name) in outer.attachments

            def __getitem__(self, name):
                return outer.attachments[outer.aname(trial, name)]

            def __setitem__(self, name, value):
                outer.attachments[outer.aname(trial, name)] = value

            def __delitem__(self, name):
                del outer.attachments[outer.aname(trial, name)]

        return Attachments()

    def __iter__(self):
        return iter(self._trials)

    def __len__(self):
        return len(self._trials)

    def __getitem__(self, item):
        raise NotImplementedError('')

    def refresh(self):
        if self._exp_key is None:
            self._trials = [tt for tt in self._dynamic_trials if tt['state'] != JOB_STATE_ERROR]
        else:
            self._trials = [tt for tt in self._dynamic_trials
                            if tt['state'] != JOB_STATE_ERROR and tt['exp_key'] == self._exp_key]
        self._ids.update([tt['tid'] for tt in self._trials])

    @property
    def trials(self):
        return self._trials

    @property
    def tids(self):
        return [tt['tid'] for tt in self._trials]

    @property
    def specs(self):
        return [tt['spec'] for tt in self._trials]

    @property
    def results(self):
        return [tt['result'] for tt in self._trials]

    @property
    def miscs(self):
        return [tt['misc'] for tt in self._trials]

    @property
    def idxs_vals(self):
        return miscs_to_idxs_vals(self.miscs)

    @property
    def idxs(self):
        return self.idxs_vals[0]

    @property
    def vals(self):
        return self.idxs_vals[1]

    def assert_valid_trial(self, trial):
        if not (hasattr(trial, 'keys') and hasattr(trial, 'values')):
            raise InvalidTrial('trial should be dict-like', trial)
        for key in TRIAL_KEYS:
            if key not in trial:
                raise InvalidTrial('trial missing key %s', key)
        for key in TRIAL_MISC_KEYS:
            if key not in trial['misc']:
                raise InvalidTrial('trial["misc"] missing key', key)
        if trial['tid'] != trial['misc']['tid']:
            raise InvalidTrial('tid mismatch between root and misc', trial)
        if trial['exp_key'] != self._exp_key:
            raise InvalidTrial('wrong exp_key', (trial['exp_key'], self._exp_key))
        return trial

    def _insert_trial_docs(self, docs):
        rval = [doc['tid'] for doc in docs]
        self._dynamic_trials.extend(docs)
        return rval

    def insert_trial_doc(self, doc):
        doc = self.assert_valid_trial(SONify(doc))
        return self._insert_trial_docs([doc])[0]

    def insert_trial_docs(self, docs):
        docs = [self.assert_valid_trial(SONify(doc)) for doc in docs]
        return self._insert_trial_docs(docs)

    def new_trial_ids(self, N):
        aa = len(self._ids)
        rval = list(range(aa, aa + N))
        self._ids.update(rval)
        return rval

    def new_trial_docs(self, tids, specs, results, miscs):
        assert len(tids) == len(specs) == len(results) == len(miscs)
        rval = []
        for tid, spec, result, misc in zip(tids, specs, results, miscs):
            doc = dict(state=JOB_STATE_NEW, tid=tid, spec=spec, result=result, misc=misc)
            doc['exp_key'] = self._exp_key
            doc['owner'] = None
            doc['version'] = 0
            doc['book_time'] = None
            doc['refresh_time'] = None
            rval.append(doc)
        return rval

    def source_trial_docs(self, tids, specs, results, miscs, sources):
        assert len(set(map(len, [tids, specs, results, miscs, sources]))) == 1
        rval = []
        for tid, spec, result, misc, source in zip(tids, specs, results, miscs, sources):
            doc = dict(version=0, tid=tid, spec=spec, result=result, misc=misc,
                       state=source['state'], exp_key=source['exp_key'], owner=source['owner'],
                       book_time=source['book_time'], refresh_time=source['refresh_time'])
            for k, v in (('tid', tid), ('cmd', None), ('from_tid', source['tid'])):
                assert doc['misc'].setdefault(k, v) == v
            rval.append(doc)
        return rval

    def delete_all(self):
        self._dynamic_trials = []
        self.attachments = {}
        self.refresh()

    def count_by_state_synced(self, arg, trials=None):
        if trials is None:
            trials = self._trials
        if arg in JOB_STATES:
            queue = [doc for doc in trials if doc['state'] == arg]
        elif hasattr(arg, '__iter__'):
            states = set(arg)
            assert all(x in JOB_STATES for x in states)
            queue = [doc for doc in trials if doc['state'] in states]
        else:
            raise TypeError(arg)
        return len(queue)

    def count_by_state_unsynced(self, arg):
        if self._exp_key is not None:
            exp_trials = [tt for tt in self._dynamic_trials if tt['exp_key'] == self._exp_key]
        else:
            exp_trials = self._dynamic_trials
        return self.count_by_state_synced(arg, trials=exp_trials)

    def losses(self, bandit=None):
        if bandit is None:
            return [r.get('loss') for r in self.results]
        return list(map(bandit.loss, self.results, self.specs))

    def statuses(self, bandit=None):
        if bandit is None:
            return [r.get('status') for r in self.results]
        return list(map(bandit.status, self.results, self.specs))

    def average_best_error(self, bandit=None):
        """hyperopt/base.py:536-586 (zero-variance branch and the pmin form)."""
        results = self.results
        if bandit is None:
            ok = [r for r in results if r['status'] == STATUS_OK]
            loss = [r['loss'] for r in ok]
            loss_v = [r.get('loss_variance', 0) for r in ok]
            true_loss = [r.get('true_loss', r['loss']) for r in ok]
        else:
            ok = [(r, s) for r, s in zip(results, self.specs) if bandit.status(r) == STATUS_OK]
            loss = [bandit.loss(r, s) for r, s in ok]
            loss_v = [bandit.loss_variance(r, s) for r, s in ok]
            true_loss = [bandit.true_loss(r, s) for r, s in ok]
        loss3 = sorted(zip(loss, loss_v, true_loss))
        if not loss3:
            raise ValueError('Empty loss vector')
        loss3 = np.asarray(loss3, dtype=float)
        if np.all(loss3[:, 1] == 0):
            return loss3[np.argmin(loss3[:, 0]), 2]
        cutoff = 0
        sigma = np.sqrt(loss3[0][1])
        while cutoff < len(loss3) and loss3[cutoff][0] < loss3[0][0] + 3 * sigma:
            cutoff += 1
        pmin = _pmin_sampled(loss3[:cutoff, 0], loss3[:cutoff, 1])
        return (pmin * loss3[:cutoff, 2]).sum()

    @property
    def best_trial(self):
        candidates = [t for t in self.trials if t['result']['status'] == STATUS_OK]
        losses = [float(t['result']['loss']) for t in candidates]
        assert not np.any(np.isnan(losses))
        if losses:
            return candidates[int(np.argmin(losses))]
        return None

    @property
    def argmin(self):
        best_trial = self.best_trial
        vals = best_trial['misc']['vals'] if best_trial is not None else {}
        return {k: v[0] for k, v in vals.items() if v}

    def fmin(self, fn, space, algo, max_evals, rstate=None, verbose=0,
             pass_expr_memo_ctrl=None, catch_eval_exceptions=False, return_argmin=True):
        from .fmin import fmin
        return fmin(fn, space, algo, max_evals, trials=self, rstate=rstate, verbose=verbose,
                    allow_trials_fmin=False, pass_expr_memo_ctrl=pass_expr_memo_ctrl,
                    catch_eval_exceptions=catch_eval_exceptions, return_argmin=return_argmin)


def _pmin_sampled(mean, var, n_samples=1000, rng=None):
    """hyperopt/utils.py:pmin_sampled -- probability each entry is the min."""
    if rng is None:
        rng = np.random.RandomState(232342)
    samples = rng.randn(n_samples, len(mean)) * np.sqrt(var) + mean
    winners = (samples.T == samples.min(axis=1)).T
    wincounts = winners.sum(axis=0)
    assert wincounts.shape == mean.shape
    return wincounts.astype('float64') / wincounts.sum()


def trials_from_docs(docs, validate=True, **kwargs):
    rval = Trials(**kwargs)
    if validate:
        rval.insert_trial_docs(docs)
    else:
        rval._insert_trial_docs(docs)
    rval.refresh()
    return rval


class Ctrl(object):
    """hyperopt/base.py:641-708."""
    info = logger.info
    warn = logger.warning
    error = logger.error
    debug = logger.debug

    def __init__(self, trials, current_trial=None):
        self.trials = Trials() if trials is None else trials
        self.current_trial = current_trial

    def checkpoint(self, r=None):
        assert self.current_trial in self.trials._trials
        if r is not None:
            self.current_trial['result'] = r

    @property
    def attachments(self):
        return self.trials.trial_attachments(trial=self.current_trial)

    def inject_results(self, specs, results, miscs, new_tids=None):
        trial = self.current_trial
        assert trial is not None
        num_news = len(specs)
        assert len(specs) == len(results) == len(miscs)
        if new_tids is None:
            new_tids = self.trials.new_trial_ids(num_news)
        new_trials = self.trials.source_trial_docs(tids=new_tids, specs=specs, results=results,
                                                   miscs=miscs, sources=[trial])
        for t in new_trials:
            t['state'] = JOB_STATE_DONE
        return self.trials.insert_trial_docs(new_trials)


class Domain(object):
    """Search space + objective (hyperopt/base.py:711-906)."""

    def __init__(self, fn, expr, workdir=None, pass_expr_memo_ctrl=None, name=None,
                 loss_target=None):
        self.fn = fn
        if pass_expr_memo_ctrl is None:
            self.pass_expr_memo_ctrl = getattr(fn, 'fmin_pass_expr_memo_ctrl', False)
        else:
            self.pass_expr_memo_ctrl = pass_expr_memo_ctrl
        self.expr = expr
        self.space = compile_space(expr)
        self.params = {h.label: h.node for h in self.space.hps}
        self.loss_target = loss_target
        self.name = name
        self.workdir = workdir
        self.cmd = ('domain_attachment', 'FMinIter_Domain')

    def memo_from_config(self, config):
        return dict(config)

    def evaluate(self, config, ctrl, attach_attachments=True):
        if self.pass_expr_memo_ctrl:
            rval = self.fn(expr=self.expr, memo=self.memo_from_config(config), ctrl=ctrl)
        else:
            rval = self.fn(_expr.evaluate(self.expr, config))
        if isinstance(rval, (float, int, np.number)):
            dict_rval = {'loss': float(rval), 'status': STATUS_OK}
        else:
            dict_rval = dict(rval)
            status = dict_rval['status']
            if status not in STATUS_STRINGS:
                raise InvalidResultStatus(dict_rval)
            if status == STATUS_OK:
                try:
                    dict_rval['loss'] = float(dict_rval['loss'])
                except (TypeError, KeyError):
                    raise InvalidLoss(dict_rval)
        if attach_attachments:
            attachments = dict_rval.pop('attachments', {})
            for key, val in attachments.items():
                ctrl.attachments[key] = val
        return dict_rval

    def short_str(self):
        return 'Domain{%s}' % str(self.fn)

    def loss(self, result, config=None):
        return result.get('loss', None)

    def loss_variance(self, result, config=None):
        return result.get('loss_variance', 0.0)

    def true_loss(self, result, config=None):
        try:
            return result['true_loss']
        except KeyError:
            return self.loss(result, config=config)

    def true_loss_variance(self, config=None):
        raise NotImplementedError()

    def status(self, result, config=None):
        return result['status']

    def new_result(self):
        return {'status': STATUS_NEW}
