"""An fmin ``algo`` that runs the CPU oracle (test infrastructure only):
host history assembly from hyperopt_amd, numerics from oracle/tpe_oracle.py.
``kind=None`` ties like the reference (numpy default argsort), ``'stable'``
like the GPU engine."""
import numpy as np

from hyperopt_amd import rand
from hyperopt_amd.base import miscs_update_idxs_vals
from hyperopt_amd.tpe import build_history
from oracle import tpe_oracle as O


def oracle_hps(cs):
    return {h.label: dict(dist=h.dist, args=h.args, paths=[tuple(p) for p in h.paths])
            for h in cs.hps}


def oracle_suggest(new_ids, domain, trials, seed, prior_weight=1.0, n_startup_jobs=20,
                   n_EI_candidates=24, gamma=0.25, linear_forgetting=25, kind=None):
    new_id, = new_ids
    cs = domain.space
    tids, losses, vals, active = build_history(domain, trials, cs.labels)
    if len(tids) < n_startup_jobs:
        return rand.suggest(new_ids, domain, trials, seed)
    tids = np.asarray(tids)
    obs = {lab: (tids[active[i] == 1], vals[i][active[i] == 1])
           for i, lab in enumerate(cs.labels)}
    with np.errstate(all='ignore'):
        chosen, _ = O.suggest_reference_stream(oracle_hps(cs), tids, losses, obs, seed,
                                               n_ei=n_EI_candidates, prior_weight=prior_weight,
                                               gamma=gamma, kind=kind)
    out = {}
    for lab, v in chosen.items():
        out[lab] = int(v) if cs.by_label[lab].is_categorical else float(v)
    idxs = {lab: ([new_id] if lab in out else []) for lab in cs.labels}
    vls = {lab: ([out[lab]] if lab in out else []) for lab in cs.labels}
    misc = dict(tid=new_id, cmd=domain.cmd, workdir=domain.workdir)
    miscs_update_idxs_vals([misc], idxs, vls)
    return trials.new_trial_docs([new_id], [None], [domain.new_result()], [misc])


def trajectory(trials):
    return [{k: (v[0] if v else None) for k, v in tr['misc']['vals'].items()}
            for tr in trials.trials]
