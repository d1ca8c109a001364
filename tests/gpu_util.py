"""Helpers for GPU parity tests."""
import numpy as np

# lpdf tolerance (north star): 1e-6 relative to float64 numpy; values near 0
# are compared absolutely at the same scale.
RTOL = 1e-6


def close(a, b, rtol=RTOL):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    same_nan = np.isnan(a) & np.isnan(b)
    same_inf = np.isinf(a) & np.isinf(b) & (np.sign(a) == np.sign(b))
    fin = np.isfinite(a) & np.isfinite(b)
    ok = same_nan | same_inf
    ok[fin] = np.abs(a[fin] - b[fin]) <= rtol * np.maximum(1.0, np.abs(b[fin]))
    return ok


def assert_close(a, b, rtol=RTOL, msg=''):
    ok = close(a, b, rtol)
    if not ok.all():
        i = np.where(~ok)[0][:5]
        raise AssertionError('%s: %d/%d mismatches, e.g. idx %s got %s want %s' % (
            msg, (~ok).sum(), ok.size, i, np.asarray(a)[i], np.asarray(b)[i]))


def argmax_equiv(score_ref, idx_got, rtol=RTOL):
    """idx_got is acceptable if it is the reference argmax or its score ties
    the reference maximum within tolerance (north star tie rule)."""
    score_ref = np.asarray(score_ref)
    ref = int(np.argmax(score_ref))
    if idx_got == ref:
        return True
    a, b = score_ref[idx_got], score_ref[ref]
    if np.isnan(b):
        return False
    return np.isfinite(a) and abs(a - b) <= rtol * max(1.0, abs(b))


def assert_winners_match(got, want, rtol=RTOL, msg=''):
    """Two runs' per-hp winners (RESULT_DTYPE rows) agree under the north
    star tie rule: same index and value, or -- where the runs' scoring
    rounded differently (other tiling, one exponent per wave) -- different
    winners whose scores tie within tolerance (each run's winner scores at
    least the other's, so |delta| <= the scoring error bound)."""
    got, want = np.asarray(got).reshape(-1), np.asarray(want).reshape(-1)
    np.testing.assert_array_equal(got['active'], want['active'], err_msg=msg)
    same = got['index'] == want['index']
    np.testing.assert_array_equal(got['value'][same], want['value'][same], err_msg=msg)
    assert_close(got['score'], want['score'], rtol, msg=msg)
    return int((~same).sum())
