"""ctypes binding of libtpe_engine.so (include/tpe_engine.h).

This is the only place the Python host touches the HIP engine.  There is no
CPU fallback: if the library or a gfx950 device is missing, ``Engine()``
raises ``EngineUnavailable`` and the TPE suggest path fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('TPE_ENGINE_LIB', os.path.join(_HERE, 'libtpe_engine.so'))

# ---- constants mirrored from include/tpe_engine.h -----------------------
TPE_OK = 0
TPE_E_INVALID = -1
TPE_E_BOUNDS = -2
TPE_E_NEGATIVE = -3
TPE_E_NOMEM = -4
TPE_E_HIP = -5
TPE_E_NODEVICE = -6
TPE_E_INDEX = -7

GMM, LGMM, CAT = 0, 1, 2
HAS_LOW, HAS_HIGH, HAS_Q, PCHOICE = 1, 2, 4, 8
OBS_IDENT, OBS_LOG, OBS_LOG_CLIP_EXPLOW, OBS_LOG_CLIP_EPS = 0, 1, 2, 3
KIND_NAMES = ('lse_gmm', 'lse_lgmm', 'erf_gmm', 'erf_lgmm', 'categorical')

# every symbol include/tpe_engine.h declares (checked by tests)
EXPORTS = (
    'tpe_version', 'tpe_device_count', 'tpe_create', 'tpe_destroy', 'tpe_last_error',
    'tpe_synchronize', 'tpe_split', 'tpe_parzen_fit', 'tpe_categorical_posterior',
    'tpe_lpdf', 'tpe_score', 'tpe_sample', 'tpe_plan_create', 'tpe_plan_destroy',
    'tpe_plan_num_levels', 'tpe_plan_set_history', 'tpe_plan_fit', 'tpe_plan_get_mixture',
    'tpe_plan_get_table',
    'tpe_plan_suggest', 'tpe_plan_suggest_shard', 'tpe_plan_merge', 'tpe_plan_score_candidates', 'tpe_plan_last_stats',
    'tpe_plan_profile', 'tpe_plan_profile_read', 'tpe_microbench', 'tpe_plan_get_results',
    'tpe_plan_results_device', 'tpe_plan_census', 'tpe_plan_fit_suggest',
    'tpe_plan_set_lattice', 'tpe_plan_update_history', 'tpe_plan_set_prune',
    'tpe_plan_sample_prior', 'tpe_plan_score_candidates_sorted', 'tpe_plan_census_n',
)

# include/tpe_engine.h TPE_SHARD_ALIGN: candidate splits at multiples of this
# give byte-identical suggests (the large-draw value-bucketing block)
SHARD_ALIGN = 8192


class EngineUnavailable(RuntimeError):
    """The HIP engine library or an MI355X (gfx950) device is not available."""


class EngineError(RuntimeError):
    pass


class TpeHp(C.Structure):
    _fields_ = [('family', C.c_int32), ('flags', C.c_uint32), ('obs_transform', C.c_int32),
                ('upper', C.c_int32), ('prior_mu', C.c_double), ('prior_sigma', C.c_double),
                ('low', C.c_double), ('high', C.c_double), ('q', C.c_double),
                ('cond_begin', C.c_int32), ('cond_count', C.c_int32),
                ('pprior_begin', C.c_int64)]


class TpeSpace(C.Structure):
    _fields_ = [('n_hp', C.c_int32), ('hp', C.POINTER(TpeHp)), ('n_cond', C.c_int32),
                ('cond_parent', C.POINTER(C.c_int32)), ('cond_branch', C.POINTER(C.c_int32)),
                ('n_pprior', C.c_int64), ('pprior', C.POINTER(C.c_double))]


RESULT_DTYPE = np.dtype([('score', '<f8'), ('value', '<f8'), ('index', '<i8'),
                         ('active', '<i4'), ('pad', '<i4')])

_D = C.POINTER(C.c_double)
_lib = None
_lib_lock = threading.Lock()


def _share_hip_runtime():
    """Make the engine and PyTorch use ONE HIP runtime.

    libtpe_engine.so needs ``libamdhip64.so.7``; PyTorch-ROCm ships its own
    copy (same soname) and loads it by file name.  Whichever loads second
    would bring a second runtime into the process, and the second one sees no
    GPU.  Pre-loading torch's copy (without importing torch) makes the engine
    bind to it, so torch tensors and engine launches share one runtime.
    TPE_ENGINE_HIP_RUNTIME=system keeps /opt/rocm's runtime instead."""
    if os.environ.get('TPE_ENGINE_HIP_RUNTIME', '') == 'system':
        return
    import importlib.util
    try:
        spec = importlib.util.find_spec('torch')
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.origin:
        return
    hip = os.path.join(os.path.dirname(spec.origin), 'lib', 'libamdhip64.so')
    if os.path.exists(hip):
        C.CDLL(hip, mode=C.RTLD_GLOBAL)


def load_library(path: str = LIB_PATH):
    """Load libtpe_engine.so and declare its signatures (no device needed)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise EngineUnavailable(
                'libtpe_engine.so not found at %s: build it with `make -C '
                'hyperopt_amd/csrc` or __graft_entry__.build()' % path)
        _share_hip_runtime()
        lib = C.CDLL(path)
        vp, i32, i64, u32, u64, dbl = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64, C.c_double
        sig = {
            'tpe_version': (C.c_char_p, []),
            'tpe_device_count': (C.c_int, [C.POINTER(i32)]),
            'tpe_create': (C.c_int, [i32, C.POINTER(vp)]),
            'tpe_destroy': (C.c_int, [vp]),
            'tpe_last_error': (C.c_char_p, [vp]),
            'tpe_synchronize': (C.c_int, [vp]),
            'tpe_split': (C.c_int, [vp, _D, i64, dbl, i32, C.POINTER(C.c_uint8)]),
            'tpe_parzen_fit': (C.c_int, [vp, _D, i64, dbl, dbl, dbl, i32, _D, _D, _D]),
            'tpe_categorical_posterior': (C.c_int, [vp, C.POINTER(i64), i64, i32, dbl, _D, i32, _D]),
            'tpe_lpdf': (C.c_int, [vp, i32, _D, i64, _D, _D, _D, i64, dbl, dbl, dbl, u32, _D]),
            'tpe_score': (C.c_int, [vp, i32, _D, i64, _D, _D, _D, i64, _D, _D, _D, i64,
                                    dbl, dbl, dbl, u32, _D, _D, C.POINTER(i64), _D]),
            'tpe_sample': (C.c_int, [vp, i32, _D, _D, _D, i64, dbl, dbl, dbl, u32, u64, u64,
                                     i64, i64, _D]),
            'tpe_plan_create': (C.c_int, [vp, C.POINTER(TpeSpace), i64, C.POINTER(vp)]),
            'tpe_plan_destroy': (C.c_int, [vp]),
            'tpe_plan_num_levels': (C.c_int, [vp, C.POINTER(i32)]),
            'tpe_plan_set_history': (C.c_int, [vp, vp, vp, vp, i64, i32, vp]),
            'tpe_plan_update_history': (C.c_int, [vp, i64, i64, i64, vp, vp, i64, i64, vp, i32,
                                                  vp]),
            'tpe_plan_fit': (C.c_int, [vp, dbl, i32, dbl, i32, vp]),
            'tpe_plan_get_mixture': (C.c_int, [vp, i32, i32, _D, _D, _D, i64, C.POINTER(i64)]),
            'tpe_plan_get_table': (C.c_int, [vp, i32, i32, i32, vp, i64, C.POINTER(i64)]),
            'tpe_plan_suggest': (C.c_int, [vp, C.POINTER(u64), i64, i64, i64, i32, vp, i32, vp]),
            'tpe_plan_suggest_shard': (C.c_int, [vp, C.POINTER(u64), i64, i64, i64, i64, i32, vp,
                                                 i32, vp]),
            'tpe_plan_fit_suggest': (C.c_int, [vp, dbl, i32, dbl, i32, C.POINTER(u64), i64, i64,
                                               vp, i32, vp]),
            'tpe_plan_merge': (C.c_int, [vp, vp, i32, i32, vp, i32, vp]),
            'tpe_plan_score_candidates': (C.c_int, [vp, i32, _D, i64, _D, _D, C.POINTER(i64), _D]),
            'tpe_plan_score_candidates_sorted': (C.c_int, [vp, i32, i32, _D, i64, _D, _D,
                                                           C.POINTER(i64), _D]),
            'tpe_plan_last_stats': (C.c_int, [vp, _D, _D]),
            'tpe_plan_profile': (C.c_int, [vp, i32]),
            'tpe_plan_profile_read': (C.c_int, [vp, i32, _D, C.POINTER(i64), _D]),
            'tpe_microbench': (C.c_int, [vp, i32, _D]),
            'tpe_plan_get_results': (C.c_int, [vp, vp, i32, vp]),
            'tpe_plan_results_device': (vp, [vp]),
            'tpe_plan_census': (C.c_int, [vp, i32, C.POINTER(i64)]),
            'tpe_plan_census_n': (C.c_int, [vp, i32, C.POINTER(i64), i32]),
            'tpe_plan_set_lattice': (C.c_int, [vp, i32]),
            'tpe_plan_set_prune': (C.c_int, [vp, i32]),
            'tpe_plan_sample_prior': (C.c_int, [vp, C.POINTER(u64), i64, vp, i32, vp]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def _seeds(seeds):
    """uint64 seed array (exact: a mixed list of Python ints would round
    through float64 in np.asarray)."""
    seeds = [int(x) & (2 ** 64 - 1) for x in np.atleast_1d(np.asarray(seeds, dtype=object))]
    return np.fromiter(seeds, dtype=np.uint64, count=len(seeds))


def _dp(a):
    return None if a is None else a.ctypes.data_as(_D)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


class Engine(object):
    """One HIP device bound to the TPE engine (tpe_create)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        n = C.c_int32(0)
        self.lib.tpe_device_count(C.byref(n))
        if n.value <= 0:
            raise EngineUnavailable('no HIP device visible (TPE engine needs an MI355X)')
        h = C.c_void_p()
        rc = self.lib.tpe_create(int(device), C.byref(h))
        if rc != TPE_OK:
            raise EngineUnavailable('tpe_create(%d) failed (%d): not a gfx950 device?' % (device, rc))
        self.h = h
        self.device = device
        self.lock = threading.RLock()

    def close(self):
        if getattr(self, 'h', None):
            self.lib.tpe_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- error mapping onto the reference's exceptions ---------------------
    def check(self, rc):
        if rc == TPE_OK:
            return
        msg = (self.lib.tpe_last_error(self.h) or b'').decode()
        if rc == TPE_E_BOUNDS:
            raise ValueError('low >= high', msg)                 # tpe.py:80-81
        if rc == TPE_E_NEGATIVE:
            raise ValueError('negative arg to lognormal_cdf', msg)  # tpe.py:181-182
        if rc == TPE_E_INDEX:
            raise IndexError(msg)
        if rc == TPE_E_INVALID:
            raise ValueError(msg)
        raise EngineError('TPE engine error %d: %s' % (rc, msg))

    def synchronize(self):
        """Wait for all of this engine's device work (tpe_synchronize)."""
        with self.lock:
            self.check(self.lib.tpe_synchronize(self.h))

    def microbench(self, which):
        r = C.c_double(0)
        with self.lock:
            self.check(self.lib.tpe_microbench(self.h, int(which), C.byref(r)))
        return r.value

    # -- operator level ----------------------------------------------------
    def split(self, losses, gamma, gamma_cap=25):
        losses = _f64(losses)
        out = np.zeros(losses.size, dtype=np.uint8)
        with self.lock:
            self.check(self.lib.tpe_split(self.h, _dp(losses), losses.size, float(gamma),
                                          int(gamma_cap), out.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out.astype(bool)

    def parzen_fit(self, obs, prior_weight, prior_mu, prior_sigma, lf=25):
        obs = _f64(obs).ravel()
        k = obs.size + 1
        w, mu, sg = np.empty(k), np.empty(k), np.empty(k)
        with self.lock:
            self.check(self.lib.tpe_parzen_fit(self.h, _dp(obs), obs.size, float(prior_weight),
                                               float(prior_mu), float(prior_sigma), int(lf),
                                               _dp(w), _dp(mu), _dp(sg)))
        return w, mu, sg

    def categorical_posterior(self, obs, upper, prior_weight, p_prior=None, lf=25):
        obs = np.ascontiguousarray(obs, dtype=np.int64).ravel()
        p = np.empty(int(upper))
        pp = None if p_prior is None else _f64(p_prior)
        with self.lock:
            self.check(self.lib.tpe_categorical_posterior(
                self.h, obs.ctypes.data_as(C.POINTER(C.c_int64)), obs.size, int(upper),
                float(prior_weight), _dp(pp), int(lf), _dp(p)))
        return p

    @staticmethod
    def _flags(low, high, q):
        f = 0
        if low is not None:
            f |= HAS_LOW
        if high is not None:
            f |= HAS_HIGH
        if q is not None:
            f |= HAS_Q
        return f

    def score(self, family, x, below, above, low=None, high=None, q=None, want_llik=True):
        """Fused lpdf(below), lpdf(above), argmax(below - above)."""
        x = _f64(x).ravel()
        if family == CAT:
            wb, mb, sb = _f64(below), None, None
            wa, ma, sa = _f64(above), None, None
        else:
            wb, mb, sb = (_f64(a) for a in below)
            wa, ma, sa = (_f64(a) for a in above)
        lb = np.empty(x.size) if want_llik else None
        la = np.empty(x.size) if want_llik else None
        bi, bs = C.c_int64(-1), C.c_double(np.nan)
        with self.lock:
            self.check(self.lib.tpe_score(
                self.h, family, _dp(x), x.size, _dp(wb), _dp(mb), _dp(sb), wb.size,
                _dp(wa), _dp(ma), _dp(sa), wa.size,
                float(low) if low is not None else 0.0, float(high) if high is not None else 0.0,
                float(q) if q is not None else 0.0, self._flags(low, high, q),
                _dp(lb), _dp(la), C.byref(bi), C.byref(bs)))
        return lb, la, bi.value, bs.value

    def lpdf(self, family, x, w, mu=None, sigma=None, low=None, high=None, q=None):
        xa = _f64(x)
        xs = xa.ravel()
        w = _f64(w)
        mu = None if mu is None else _f64(mu)
        sigma = None if sigma is None else _f64(sigma)
        out = np.empty(xs.size)
        with self.lock:
            self.check(self.lib.tpe_lpdf(
                self.h, family, _dp(xs), xs.size, _dp(w), _dp(mu), _dp(sigma), w.size,
                float(low) if low is not None else 0.0, float(high) if high is not None else 0.0,
                float(q) if q is not None else 0.0, self._flags(low, high, q), _dp(out)))
        return out.reshape(xa.shape)

    def sample(self, family, w, mu=None, sigma=None, low=None, high=None, q=None, seed=0,
               stream=0, offset=0, n=1):
        w = _f64(w)
        mu = None if mu is None else _f64(mu)
        sigma = None if sigma is None else _f64(sigma)
        out = np.empty(int(n))
        with self.lock:
            self.check(self.lib.tpe_sample(
                self.h, family, _dp(w), _dp(mu), _dp(sigma), w.size,
                float(low) if low is not None else 0.0, float(high) if high is not None else 0.0,
                float(q) if q is not None else 0.0, self._flags(low, high, q),
                int(seed) & (2 ** 64 - 1), int(stream), int(offset), int(n), _dp(out)))
        return out


class Plan(object):
    """A compiled search space with a device-resident history (tpe_plan_*)."""

    def __init__(self, engine: Engine, hps, conds, pprior, max_trials):
        self.engine = engine
        lib = engine.lib
        self.n_hp = len(hps)
        arr = (TpeHp * self.n_hp)(*hps)
        cp = np.ascontiguousarray([c[0] for c in conds], dtype=np.int32)
        cb = np.ascontiguousarray([c[1] for c in conds], dtype=np.int32)
        pp = _f64(pprior if len(pprior) else np.zeros(0))
        sp = TpeSpace(self.n_hp, arr, len(conds), cp.ctypes.data_as(C.POINTER(C.c_int32)),
                      cb.ctypes.data_as(C.POINTER(C.c_int32)), pp.size, _dp(pp))
        self._keep = (arr, cp, cb, pp)
        p = C.c_void_p()
        with engine.lock:
            engine.check(lib.tpe_plan_create(engine.h, C.byref(sp), int(max_trials), C.byref(p)))
        self.p = p
        self.max_trials = int(max_trials)
        nl = C.c_int32(0)
        lib.tpe_plan_num_levels(p, C.byref(nl))
        self.n_levels = nl.value

    def close(self):
        if getattr(self, 'p', None):
            self.engine.lib.tpe_plan_destroy(self.p)
            self.p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_history(self, losses, vals, active, stream=None):
        """Whole history from host arrays: losses[n], vals[n_hp, n] float64,
        active[n_hp, n] uint8."""
        losses = _f64(losses)
        vals = _f64(vals)
        active = np.ascontiguousarray(active, dtype=np.uint8)
        n = losses.size
        assert vals.shape == (self.n_hp, n) and active.shape == (self.n_hp, n)
        self.update_history(n, 0, vals, active, n, 0, losses, stream=stream)

    def update_history(self, n, row0, vals, active, ld, loss0, losses, stream=None):
        """Incremental history (tpe_plan_update_history): rows [row0, n) of
        the host columns vals[n_hp, ld] / active[n_hp, ld] (C-contiguous) and
        losses[loss0:n]; rows below row0 stay as the device has them."""
        e = self.engine
        if n > self.max_trials:
            raise ValueError('history of %d trials exceeds the plan capacity %d'
                             % (n, self.max_trials))
        if vals.dtype != np.float64 or active.dtype != np.uint8 or \
                not vals.flags.c_contiguous or not active.flags.c_contiguous or \
                vals.shape != (self.n_hp, ld) or active.shape != (self.n_hp, ld):
            raise ValueError('history columns must be C-contiguous [n_hp, ld] f64 / u8')
        losses = np.asarray(losses)
        if losses.dtype != np.float64 or not losses.flags.c_contiguous:
            raise ValueError('losses must be C-contiguous float64')
        nr = n - row0
        vp = vals.ctypes.data + 8 * row0 if nr > 0 else None
        ap = active.ctypes.data + row0 if nr > 0 else None
        lp = losses.ctypes.data + 8 * loss0 if loss0 < n else None
        self._hist = (vals, active, losses)   # keep the host memory alive
        with e.lock:
            e.check(e.lib.tpe_plan_update_history(self.p, int(n), int(row0), int(nr), vp, ap,
                                                  int(ld), int(loss0), lp, 0, stream))
        self.n = int(n)

    def set_history_device(self, losses_ptr, vals_ptr, active_ptr, n, stream=None):
        e = self.engine
        with e.lock:
            e.check(e.lib.tpe_plan_set_history(self.p, losses_ptr, vals_ptr, active_ptr, int(n),
                                               1, stream))
        self.n = int(n)

    def fit(self, gamma=0.25, prior_weight=1.0, lf=25, gamma_cap=25, stream=None):
        e = self.engine
        with e.lock:
            e.check(e.lib.tpe_plan_fit(self.p, float(gamma), int(gamma_cap), float(prior_weight),
                                       int(lf), stream))

    def mixture(self, hp, side=0):
        e = self.engine
        cap = max(self.max_trials + 1, 1)
        # categorical hps may have more categories than trials
        cap = max(cap, 1 << 16)
        w, mu, sg = np.empty(cap), np.empty(cap), np.empty(cap)
        k = C.c_int64(0)
        with e.lock:
            e.check(e.lib.tpe_plan_get_mixture(self.p, int(hp), int(side), _dp(w), _dp(mu),
                                               _dp(sg), cap, C.byref(k)))
        k = k.value
        return w[:k].copy(), mu[:k].copy(), sg[:k].copy()

    def table(self, hp, side=0, which=2):
        """Raw scoring table of slot (hp, side) as bytes (tpe_plan_get_table:
        0 coefficients, 1 block-local fp32, 2 moment chunks, 3 8-wide moment
        blocks, 4 degree-15 moment chunks; diagnostics)."""
        e = self.engine
        n = C.c_int64(0)
        with e.lock:
            e.check(e.lib.tpe_plan_get_table(self.p, int(hp), int(side), int(which), None, 0,
                                             C.byref(n)))
            buf = np.empty(n.value, dtype=np.uint8)
            e.check(e.lib.tpe_plan_get_table(self.p, int(hp), int(side), int(which),
                                             buf.ctypes.data, buf.size, C.byref(n)))
        return buf

    def suggest(self, seeds, n_cand, cand_begin=0, level=-1, out=None, stream=None, fetch=True,
                n_total=None):
        """Returns a structured array [n_suggest, n_hp] of RESULT_DTYPE (host)
        unless ``out`` is a device pointer (int) or ``fetch`` is False (the
        results stay in the plan: ``results_device_ptr()`` / ``results()``).
        ``n_total``: the candidate count of the whole suggestion when this
        call is a shard [cand_begin, cand_begin + n_cand) of it
        (tpe_plan_suggest_shard; default cand_begin + n_cand)."""
        e = self.engine
        seeds = _seeds(seeds)
        host = out is None and fetch
        res = np.empty((seeds.size, self.n_hp), dtype=RESULT_DTYPE) if host else None
        optr = res.ctypes.data if host else out
        total = int(cand_begin) + int(n_cand) if n_total is None else int(n_total)
        with e.lock:
            e.check(e.lib.tpe_plan_suggest_shard(
                self.p, seeds.ctypes.data_as(C.POINTER(C.c_uint64)), seeds.size, total,
                int(cand_begin), int(n_cand), int(level), optr, 0 if host else 1, stream))
        self._last_nsug = seeds.size
        self._last_ncand = int(n_cand)
        return res

    def fit_suggest(self, seeds, n_cand, gamma=0.25, prior_weight=1.0, lf=25, gamma_cap=25,
                    out=None, stream=None, fetch=True):
        """fit() + suggest() over all levels in one engine call; repeated calls
        of one shape replay a captured hipGraph of the step (tpe_engine.h)."""
        e = self.engine
        seeds = _seeds(seeds)
        host = out is None and fetch
        res = np.empty((seeds.size, self.n_hp), dtype=RESULT_DTYPE) if host else None
        optr = res.ctypes.data if host else out
        with e.lock:
            e.check(e.lib.tpe_plan_fit_suggest(
                self.p, float(gamma), int(gamma_cap), float(prior_weight), int(lf),
                seeds.ctypes.data_as(C.POINTER(C.c_uint64)), seeds.size, int(n_cand),
                optr, 0 if host else 1, stream))
        self._last_nsug = seeds.size
        self._last_ncand = int(n_cand)
        return res

    def sample_prior(self, seeds, stream=None):
        """Prior draws of len(seeds) whole suggestions (rand.suggest on the
        device): [S, n_hp] RESULT_DTYPE, value/active per hp."""
        e = self.engine
        seeds = _seeds(seeds)
        res = np.empty((seeds.size, self.n_hp), dtype=RESULT_DTYPE)
        with e.lock:
            e.check(e.lib.tpe_plan_sample_prior(self.p, seeds.ctypes.data_as(C.POINTER(C.c_uint64)),
                                                seeds.size, res.ctypes.data, 0, stream))
        self._last_nsug = seeds.size
        return res

    def results(self):
        e = self.engine
        res = np.empty((getattr(self, '_last_nsug', 1), self.n_hp), dtype=RESULT_DTYPE)
        with e.lock:
            e.check(e.lib.tpe_plan_get_results(self.p, res.ctypes.data, 0, None))
        return res

    def get_results(self, out, stream=None):
        """Copy the last suggest's records to the device pointer ``out``
        (tpe_plan_get_results, stream-ordered)."""
        e = self.engine
        with e.lock:
            e.check(e.lib.tpe_plan_get_results(self.p, out, 1, stream))

    def results_device_ptr(self):
        return self.engine.lib.tpe_plan_results_device(self.p)

    def merge(self, gathered_ptr, world, level, out=None, stream=None, n_suggest=1,
              in_place=False):
        """tpe_plan_merge; in_place: ``out`` (device) already holds the
        level's suggest records (suggest(..., out=out)), only the merged
        slots are stored into it (out_on_device 2, no copy launch)."""
        e = self.engine
        host = out is None
        res = np.empty((n_suggest, self.n_hp), dtype=RESULT_DTYPE) if host else None
        optr = res.ctypes.data if host else out
        mode = 0 if host else (2 if in_place else 1)
        with e.lock:
            e.check(e.lib.tpe_plan_merge(self.p, gathered_ptr, int(world), int(level), optr,
                                         mode, stream))
        return res

    def score_candidates(self, hp, x, sorted_mode=None, want_llik=True):
        """Below / above lpdf and argmax of given candidates of one hp with
        the fitted mixtures.  sorted_mode None: each candidate scored on its
        own (exact sums); 0 / 1 / 2 / 3: the large-draw production form
        (tpe_plan_score_candidates_sorted: value-bucketed blocks, log-sum-exp
        prune mode 0 / 1 / 2 / 3).  want_llik False: no lpdf outputs -- the
        scorer then takes the suggest's EI-only finalize (one log2 of the
        ratio of the two sums) and (None, None, index, score) is returned."""
        e = self.engine
        x = _f64(x).ravel()
        lb, la = (np.empty(x.size), np.empty(x.size)) if want_llik else (None, None)
        bi, bs = C.c_int64(-1), C.c_double(np.nan)
        mode = -1 if sorted_mode is None else int(sorted_mode)
        with e.lock:
            e.check(e.lib.tpe_plan_score_candidates_sorted(
                self.p, int(hp), mode, _dp(x), x.size, _dp(lb) if want_llik else None,
                _dp(la) if want_llik else None, C.byref(bi), C.byref(bs)))
        return lb, la, bi.value, bs.value

    def profile(self, capacity):
        e = self.engine
        with e.lock:
            e.check(e.lib.tpe_plan_profile(self.p, int(capacity)))

    def profile_read(self, kind):
        """(avg_ms, launches, pairs_per_launch) of one scoring kind."""
        e = self.engine
        ms, n, pairs = C.c_double(0), C.c_int64(0), C.c_double(0)
        with e.lock:
            e.check(e.lib.tpe_plan_profile_read(self.p, int(kind), C.byref(ms), C.byref(n),
                                                C.byref(pairs)))
        return ms.value, n.value, pairs.value

    def set_lattice(self, enable):
        """Score bounded quantized hps on their value lattice (default) or
        every candidate on its own (tpe_plan_set_lattice)."""
        e = self.engine
        with e.lock:
            e.check(e.lib.tpe_plan_set_lattice(self.p, int(bool(enable))))

    def set_prune(self, mode):
        """Log-sum-exp on bucketed large draws (tpe_plan_set_prune): 0 / False
        every pair, 1 skip negligible component blocks, 2 skip + one exponent
        per wave, 3 / True (default) the same with block-local fp32 pairs."""
        mode = 3 if mode is True else int(mode)
        e = self.engine
        with e.lock:
            e.check(e.lib.tpe_plan_set_prune(self.p, mode))

    def census(self, enable, n=7):
        """Pair census since the last call: (quantized total, live, evaluated,
        log-sum-exp total, log-sum-exp evaluated in the one-exponent form,
        log-sum-exp evaluated, of those in the fp32 per-group-lift form[,
        one-exponent pairs re-evaluated by a wave's second attempt,
        one-exponent pairs of wide blocks (mode 3's fp64 loop), one-exponent
        pairs evaluated in the moment form of their chunk, of those the
        8-wide form, of those the 16-wide degree-15 form]) -- the first
        ``n`` (7 .. 12); enable it for the following suggests."""
        if not 0 <= n <= 12:
            raise ValueError('the census has 12 counters')
        e = self.engine
        out = (C.c_int64 * 12)()
        with e.lock:
            e.check(e.lib.tpe_plan_census_n(self.p, int(bool(enable)), out, int(n)))
        return tuple(int(v) for v in out[:n])

    def last_stats(self):
        e = self.engine
        ms, pairs = C.c_double(0), C.c_double(0)
        with e.lock:
            e.check(e.lib.tpe_plan_last_stats(self.p, C.byref(ms), C.byref(pairs)))
        return ms.value, pairs.value


_default = {}
_default_lock = threading.Lock()


def default_engine(device: int | None = None) -> Engine:
    """Process-wide engine for ``device`` (default: LOCAL_RANK or 0)."""
    if device is None:
        device = int(os.environ.get('LOCAL_RANK', '0'))
    with _default_lock:
        eng = _default.get(device)
        if eng is None:
            eng = Engine(device)
            _default[device] = eng
        return eng
