#!/usr/bin/env python3
"""Numerics study (CPU, numpy emulation): log-sum-exp pair arithmetic of
k_score's one-exponent form against the float64 oracle at config 4.

  current : t = alpha + y'(beta + gamma y') in fp64, z = fp32(t - M), v_exp_f32
  blockf32: block-local fp32 quadratic, u = fp32(y - m_b) per (candidate,
            block of 8 components), alpha'_k stored fp32 relative to an
            integer block offset A_b, z = fma32(fma32(gamma', u, beta'_k), u,
            fp32(A_b - M) + alpha'_k)

Both sum 2^z in fp32 per group of 8 and in fp64 across groups, with one
exponent M per wave of 128 value-sorted candidates (the bucketed tiles).
Prints max |lpdf - oracle| / max(1, |oracle|) for each scheme.
usage: fp32_pair_error.py [n_cand] [hp index]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from oracle import tpe_oracle as O  # noqa: E402
import big_configs  # noqa: E402

LOG2E = 1.4426950408889634


def f32(x):
    return np.asarray(x, dtype=np.float64).astype(np.float32)


def fma32(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)


def mixture(hp_i):
    U, L = big_configs.cfg4_columns()
    x = U[:, hp_i]
    tids = np.arange(L.size)
    b, a = O.split_observations(tids, x, tids, L, 0.25, kind='stable')
    w, mu, sg = O.parzen_fit(a, 1.0, 0.0, 10.0, kind='stable')
    return w, mu, sg


def schemes(xc, w, mu, sg, low=-5.0, high=5.0):
    sgc = np.maximum(sg, 1e-12)
    pacc = np.sum(w * (O.normal_cdf(high, mu, sgc) - O.normal_cdf(low, mu, sgc)))
    c = LOG2E * np.log(w / np.sqrt(2 * np.pi * sgc ** 2) / pacc)
    a2 = LOG2E / (2 * sgc ** 2)
    K = w.size
    pad = (-K) % 8
    cP = np.concatenate([c, np.full(pad, -np.inf)])
    a2P = np.concatenate([a2, np.ones(pad)])
    muP = np.concatenate([mu, np.full(pad, mu[-1])])
    nb = cP.size // 8
    cB, a2B, muB = cP.reshape(nb, 8), a2P.reshape(nb, 8), muP.reshape(nb, 8)
    # block-local fp32 table
    m_b = muB.mean(axis=1)
    d = muB - m_b[:, None]
    alpha_full = cB - a2B * d * d
    A_b = np.floor(np.max(np.where(np.isfinite(alpha_full), alpha_full, -1e300), axis=1))
    al32 = f32(alpha_full - A_b[:, None])
    be32 = f32(2 * a2B * d)
    ga32 = f32(-a2B)
    order = np.argsort(xc, kind='stable')
    out = {k: np.empty(xc.size) for k in ('current', 'blockf32', 'blockf32_uu', 'blockf32_uu_pair')}
    for w0 in range(0, xc.size, 128):
        idx = order[w0:w0 + 128]
        y = xc[idx]
        t = cP[None, :] - a2P[None, :] * (y[:, None] - muP[None, :]) ** 2  # (n, K') fp64
        M = np.ceil(np.max(t)) + 1.0
        # current: fp32(t - M)
        z = f32(t - M)
        e = np.exp2(z.astype(np.float64)).astype(np.float32).reshape(y.size, nb, 8)
        s = e.sum(axis=2, dtype=np.float32).astype(np.float64).sum(axis=1)
        out['current'][idx] = (M + np.log2(s)) / LOG2E
        # block-local fp32
        u = f32(y[:, None] - m_b[None, :])                                 # (n, nb)
        am = (f32(A_b - M)[None, :, None] + al32[None, :, :]).astype(np.float32)  # (1, nb, 8)
        am = np.broadcast_to(am, (y.size, nb, 8))
        uu = np.broadcast_to(u[:, :, None], (y.size, nb, 8))
        zb = fma32(fma32(np.broadcast_to(ga32, uu.shape), uu, np.broadcast_to(be32, uu.shape)), uu, am)
        e = np.exp2(zb.astype(np.float64)).astype(np.float32)
        s = e.sum(axis=2, dtype=np.float32).astype(np.float64).sum(axis=1)
        out['blockf32'][idx] = (M + np.log2(s)) / LOG2E
        # round 4: gamma u^2 + (beta u + alpha'), u^2 rounded to fp32 once
        u2 = np.broadcast_to(f32(u.astype(np.float64) ** 2)[:, :, None], uu.shape)
        zc = fma32(np.broadcast_to(ga32, uu.shape), u2,
                   fma32(np.broadcast_to(be32, uu.shape), uu, am))
        e = np.exp2(zc.astype(np.float64)).astype(np.float32)
        s = e.sum(axis=2, dtype=np.float32).astype(np.float64).sum(axis=1)
        out['blockf32_uu'][idx] = (M + np.log2(s)) / LOG2E
        # the same with two blocks' fp32 sums added in fp32 before the fp64 sum
        bs = e.sum(axis=2, dtype=np.float32)                       # (n, nb) fp32
        if nb % 2:
            bs = np.concatenate([bs, np.zeros((bs.shape[0], 1), np.float32)], axis=1)
        s2 = (bs[:, 0::2] + bs[:, 1::2]).astype(np.float64).sum(axis=1)
        out['blockf32_uu_pair'][idx] = (M + np.log2(s2)) / LOG2E
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    hp_i = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    w, mu, sg = mixture(hp_i)
    rs = np.random.RandomState(5)
    xc = np.concatenate([rs.uniform(-5, 5, n // 2),
                         O.gmm_sample(rs, w, mu, sg, -5.0, 5.0, None, n=n - n // 2)])
    ref = O.gmm_lpdf(xc, w, mu, sg, -5.0, 5.0, None)
    got = schemes(xc, w, mu, sg)
    for k, v in got.items():
        err = np.abs(v - ref) / np.maximum(1.0, np.abs(ref))
        print('%-9s K=%d n=%d max rel %.3g  p99.9 %.3g  mean %.3g' % (
            k, w.size, xc.size, err.max(), np.quantile(err, 0.999), err.mean()))


if __name__ == '__main__':
    main()
