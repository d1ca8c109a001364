#!/usr/bin/env python3
"""Numerics study (CPU, numpy emulation): the moment form of a log-sum-exp
block against the float64 oracle.

A coefficient block of 8 consecutive (mu-sorted) components that share one
sigma -- every component whose adaptive-Parzen sigma sits at the
prior_sigma / min(100, 1 + N) floor, the common case of long histories
(reference tpe.py:440-456) -- has, at a candidate y' = centre + v,

  sum_k 2^(t_k) = 2^(T* - a^2 v^2) * sum_k rho_k exp(q_k v)
  T_k = t_k(centre), T* = max_k T_k, rho_k = 2^(T_k - T*), q_k = 2 a^2 ln2 d_k,
  d_k = mu'_k - centre,

and exp(q_k v) = sum_j (q_k v)^j / j! truncated at degree P: the block's 8
exponentials become one exp2 and a degree-P polynomial in v whose
coefficients m_j = sum_k rho_k q_k^j / j! are fixed per block (written once by
the fit).  Truncation: relative error per term <= x^(P+1) / (P+1)! e^x,
x = |v| max_k |q_k|, so a block is taken in this form by a wave only while
x <= X_LIM over the wave's candidate range.

This script emulates the fp32 kernel arithmetic (v = fp32(y' - centre), arg
= fma32(-a^2, v*v, fp32(T* - A) + (A - M)), exp2, Horner in fp32, e * P,
two blocks' sums added in fp32, fp64 accumulation) for waves of 128
value-sorted candidates, and prints the max relative lpdf error against the
oracle next to the current pair form, with the fraction of blocks the moment
form takes.
usage: moment_error.py [cfg4|cfg5|cfg3] [n_cand] [hp index]
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from oracle import tpe_oracle as O  # noqa: E402
import big_configs  # noqa: E402

LOG2E = 1.4426950408889634
LN2 = math.log(2.0)
P = int(os.environ.get('MOM_P', '9'))  # degree, tpe_internal.hpp kMomDeg
X_LIM = float(os.environ.get('MOM_XLIM', '0.65'))  # x^(P+1)/(P+1)! e^x <= 7.1e-9, kMomXLim
X_CAP = float(os.environ.get('MOM_XCAP', '2.5'))  # kMomXCap
CH = int(os.environ.get('MOM_CH', '16'))  # components per chunk, kMomChunk


def f32(x):
    return np.asarray(x, dtype=np.float64).astype(np.float32)


def fma32(a, b, c):
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) +
            np.asarray(c, np.float64)).astype(np.float32)


def mixture(cfg, hp_i):
    """(w, mu, sigma, low, high, prior_mu, prior_sigma) of the above-side fit."""
    if cfg == 'cfg4':
        U, L = big_configs.cfg4_columns()
        x = U[:, hp_i]
        lo, hi = -5.0, 5.0
    else:
        n = int(os.environ.get('MOM_N', 1000 if cfg == 'cfg5' else 1400))
        rs = np.random.RandomState(hp_i + 3)
        x = rs.uniform(-5, 5, n)
        L = np.random.RandomState(2).rand(n)
        lo, hi = -5.0, 5.0
    tids = np.arange(L.size)
    b, a = O.split_observations(tids, x, tids, L, 0.25, kind='stable')
    pm, ps = 0.5 * (lo + hi), hi - lo
    w, mu, sg = O.parzen_fit(a, 1.0, pm, ps, kind='stable')
    return w, mu, sg, lo, hi, pm


def tables(w, mu, sg, lo, hi, pm):
    sgc = np.maximum(sg, 1e-12)
    pacc = np.sum(w * (O.normal_cdf(hi, mu, sgc) - O.normal_cdf(lo, mu, sgc)))
    c = LOG2E * np.log(w / np.sqrt(2 * np.pi * sgc ** 2) / pacc)
    a2 = LOG2E / (2 * sgc ** 2)
    m = mu - pm
    K = w.size
    pad = (-K) % CH
    cP = np.concatenate([c, np.full(pad, -np.inf)])
    a2P = np.concatenate([a2, np.full(pad, a2[-1])])
    mP = np.concatenate([m, np.full(pad, m[-1])])
    valid = np.concatenate([np.ones(K, bool), np.zeros(pad, bool)])
    nb = cP.size // CH
    B = dict(c=cP.reshape(nb, CH), a2=a2P.reshape(nb, CH), m=mP.reshape(nb, CH),
             valid=valid.reshape(nb, CH), sg=np.concatenate([sgc, np.full(pad, sgc[-1])]).reshape(nb, CH))
    cen = 0.5 * (np.where(B['valid'], B['m'], np.inf).min(1) + np.where(B['valid'], B['m'], -np.inf).max(1))
    d = B['m'] - cen[:, None]
    T = np.where(B['valid'], B['c'] - B['a2'] * d * d, -np.inf)
    Ts = T.max(1)
    base = np.floor(Ts)
    eq = np.array([np.all(B['sg'][i][B['valid'][i]] == B['sg'][i][B['valid'][i]][0]) for i in range(nb)])
    rho = np.where(B['valid'], np.exp2(T - Ts[:, None]), 0.0)
    q = 2.0 * B['a2'] * LN2 * d
    mom = np.stack([(rho * q ** j).sum(1) / math.factorial(j) for j in range(P + 1)], 1)
    h = np.where(B['valid'], np.abs(d), 0).max(1)
    xh = np.where(eq, h * 2.0 * B['a2'][:, 0] * LN2, np.inf)
    B.update(cen=cen, base=base, cm=f32(Ts - base), gam=f32(-B['a2'][:, 0]), mom=f32(mom), xh=xh,
             lo=np.where(B['valid'], B['m'], np.inf).min(1), hi=np.where(B['valid'], B['m'], -np.inf).max(1))
    # block-local pair form (Coef32)
    al = T
    B['pa'] = f32(np.where(B['valid'], al - base[:, None], -np.inf))
    B['pb'] = f32(2 * B['a2'] * d)
    B['pc'] = f32(-B['a2'])
    return B


def score(B, y):
    """lpdf (log2 sums, kernel emulation) of 128 sorted candidates y' and the
    number of blocks taken in the moment form."""
    nb = B['cen'].size
    t = B['c'].reshape(-1)[None, :] - B['a2'].reshape(-1)[None, :] * (y[:, None] - B['m'].reshape(-1)[None, :]) ** 2
    M = np.ceil(np.max(t)) + 1.0
    lo, hi = y.min(), y.max()
    x = np.maximum(np.abs(lo - B['cen']), np.abs(hi - B['cen'])) * B['xh']
    # weighted criterion (tpe_score.hip): tau(x) 2^(bound - L) <= 2^-dead,
    # bound = the chunk's largest term over the window, L = the smallest lane
    # maximum (the kernel uses envelope bounds and the tightened threshold)
    tt = t.reshape(y.size, nb, CH)
    bound = tt.max(axis=(0, 2))
    L = t.max(axis=1).min()
    dead = 26 + math.ceil(math.log2(max(t.shape[1] - 1, 1)))
    with np.errstate(divide='ignore'):
        l2tau = (P + 1) * np.log2(x) + x * math.log2(math.e) - math.log2(math.factorial(P + 1))
    use = (x <= X_LIM) | ((x <= X_CAP) & (l2tau + bound <= L - dead))
    live = bound >= L - dead - 1
    score.live = getattr(score, 'live', 0) + int(live.sum())
    score.live_mom = getattr(score, 'live_mom', 0) + int((live & use).sum())
    bs = np.empty((y.size, nb), np.float32)
    # moment blocks
    v = f32(y[:, None] - B['cen'][None, :])                       # (n, nb)
    off = (B['cm'] + f32(B['base'] - M)).astype(np.float32)
    arg = fma32(B['gam'][None, :], (v * v).astype(np.float32), off[None, :])
    e = np.exp2(arg.astype(np.float64)).astype(np.float32)
    mom = B['mom']
    acc = fma32(mom[None, :, P], v, mom[None, :, P - 1])
    for j in range(P - 2, -1, -1):
        acc = fma32(acc, v, mom[None, :, j])
    bm = (e * acc).astype(np.float32)
    # pair form
    u = f32(y[:, None] - B['cen'][None, :])
    am = (B['pa'] + f32(B['base'] - M)[:, None]).astype(np.float32)     # (nb, CH)
    uu = (u * u).astype(np.float32)
    z = fma32(B['pc'][None], uu[:, :, None], fma32(B['pb'][None], u[:, :, None], am[None]))
    ep = np.exp2(z.astype(np.float64)).astype(np.float32)
    bp = ep.sum(axis=2, dtype=np.float32)
    bs = np.where(use[None, :], bm, bp)
    if nb % 2:
        bs = np.concatenate([bs, np.zeros((bs.shape[0], 1), np.float32)], axis=1)
    s = (bs[:, 0::2] + bs[:, 1::2]).astype(np.float64).sum(axis=1)
    s_pair = np.concatenate([bp, np.zeros((bp.shape[0], nb % 2), np.float32)], axis=1)
    s_pair = (s_pair[:, 0::2] + s_pair[:, 1::2]).astype(np.float64).sum(axis=1)
    return (M + np.log2(s)) / LOG2E, (M + np.log2(s_pair)) / LOG2E, int(use.sum())


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else 'cfg4'
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    hp_i = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    w, mu, sg, lo, hi, pm = mixture(cfg, hp_i)
    B = tables(w, mu, sg, lo, hi, pm)
    rs = np.random.RandomState(5)
    xc = np.concatenate([rs.uniform(lo, hi, n // 2),
                         O.gmm_sample(rs, w, mu, sg, lo, hi, None, n=n - n // 2)])
    ref = O.gmm_lpdf(xc, w, mu, sg, lo, hi, None)
    order = np.argsort(xc, kind='stable')
    got_m, got_p = np.empty(xc.size), np.empty(xc.size)
    used = 0
    for w0 in range(0, xc.size, 128):
        idx = order[w0:w0 + 128]
        a, b, u = score(B, xc[idx] - pm)
        # (the lpdf of GMM is the log2 sum in nats; pacc is in c)
        got_m[idx], got_p[idx] = a, b
        used += u
    nw = -(-xc.size // 128)
    for name, g in (('moment', got_m), ('pair', got_p)):
        err = np.abs(g - ref) / np.maximum(1.0, np.abs(ref))
        print('%-6s %s K=%d n=%d max rel %.3g  p99.9 %.3g  mean %.3g' % (
            name, cfg, w.size, xc.size, err.max(), np.quantile(err, 0.999), err.mean()))
    print('live (wave, chunk) pairs %d, of them in the moment form %.3f' % (
        score.live, score.live_mom / max(score.live, 1)))
    print('moment-form blocks: %.3f of the (wave, block) pairs; equal-sigma blocks %.3f; '
          'xh median %.3g' % (used / (nw * B['cen'].size), np.isfinite(B['xh']).mean(),
                              np.median(B['xh'][np.isfinite(B['xh'])]) if np.isfinite(B['xh']).any() else np.nan))


if __name__ == '__main__':
    main()
