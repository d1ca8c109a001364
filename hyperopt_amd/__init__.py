"""hyperopt_amd -- MI355X-native TPE suggestion engine behind hyperopt's API.

    from hyperopt_amd import fmin, hp, tpe, Trials
    best = fmin(fn, hp.uniform('x', -5, 5), algo=tpe.suggest, max_evals=100)

The numeric hot path of ``tpe.suggest`` (good/bad split, Parzen fits,
candidate draws, GMM/LGMM/categorical lpdf, EI argmax) runs as hand-written
gfx950 HIP kernels in ``libtpe_engine.so`` (C ABI: include/tpe_engine.h).
"""
from .base import (STATUS_STRINGS, STATUS_NEW, STATUS_RUNNING, STATUS_SUSPENDED,  # noqa: F401
                   STATUS_OK, STATUS_FAIL, JOB_STATES, JOB_STATE_NEW, JOB_STATE_RUNNING,
                   JOB_STATE_DONE, JOB_STATE_ERROR, Ctrl, Trials, trials_from_docs, Domain)
from .fmin import fmin, fmin_pass_expr_memo_ctrl, FMinIter, partial, space_eval  # noqa: F401
from .workers import ThreadTrials  # noqa: F401
from .expr import scope  # noqa: F401
from . import hp, rand, tpe  # noqa: F401

__version__ = '0.1.0'
