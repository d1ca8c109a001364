import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'tests')):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP engine calls)')
    config.addinivalue_line('markers', 'slow: long-running CPU test')


import pytest  # noqa: E402


@pytest.fixture(scope='session')
def cfg4_plan():
    """Config 4 at BASELINE size (100 x uniform(-5, 5), N = 1e4, K_a ~ 9976),
    fitted on the device once per session (GPU tests only)."""
    import big_configs
    from hyperopt_amd import hp, _engine as E
    from hyperopt_amd.base import Domain
    dom, L, vals, act = big_configs.cfg4_domain_history(hp, Domain)
    hps, conds, pprior = dom.space.engine_tables()
    plan = E.Plan(E.default_engine(), hps, conds, pprior, max_trials=L.size)
    plan.set_history(L, vals, act)
    plan.fit()
    return dom, plan
