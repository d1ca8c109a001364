#!/usr/bin/env python3
"""Fold rocprofv3 SQ / GRBM --pmc passes (rocpd SQLite, one row per counter
instance) into per-dispatch figures for profiles/.

Per dispatch, every counter is summed over its instances (SQ: one per shader
engine, GRBM: one per XCD), then averaged over the dispatches of a kernel.
Derived ratios (MI355X_MICROARCH.md: SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* /
SQ_WAIT_* count quad-cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs):
  clock_ghz            = GRBM_GUI_ACTIVE / 8 / kernel duration (trace db)
  valu_busy            = 4 * SQ_ACTIVE_INST_VALU / (SIMDs * GRBM_GUI_ACTIVE / 8)
                         (fraction of SIMD cycles with a VALU instruction in flight)
  valu_issue_per_cycle = SQ_INSTS_VALU / (SIMDs * GRBM_GUI_ACTIVE / 8)
                         (wave64 VALU instructions per SIMD cycle; one per 4
                         cycles is the wave64 issue rate of a full-rate op)
  waves_per_simd       = 4 * SQ_WAVE_CYCLES / (SIMDs * GRBM_GUI_ACTIVE / 8)
  wait_inst_frac       = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  wait_any_frac        = SQ_WAIT_ANY / SQ_WAVE_CYCLES (pass B, its own waves)
A label that names a bench config (cfg2 ... cfg5) also writes
traffic.json[<label>]['valu_insts_per_launch']: the dispatch-weighted mean
SQ_INSTS_VALU of its scoring launches (k_score, k_score_wave,
k_score_wave1; census builds excluded), which bench.py turns into
roofline.valu_per_evaluated_pair (x 64 lanes / evaluated pairs).
usage: sq_summary.py <out.json> <label>=<dir> [<label>=<dir> ...]
"""
import collections
import json
import os
import re
import sqlite3
import sys

SIMDS = 256 * 4


def short(name):
    m = re.search(r'(k_[a-z_0-9]+?)(?:I(L[ib]\d+E)+E|$|[^a-z_0-9])', name)
    if not m:
        return None
    base = m.group(1)
    if base == 'k_score' and ('ILb0ELb1E' in name or 'ILb1ELb1E' in name):
        return base + '_census'
    if base.startswith('k_score_wave') and 'ILb1E' in name:   # k_score_wave<true>: census build
        return base + '_census'
    return base


def load(d):
    c = sqlite3.connect(d + '/run_results.db')
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names, durs = {}, {}
    q = ('select d.event_id, k.kernel_name, i.name, p.value, d.start, d."end" from rocpd_pmc_event p '
         'join rocpd_info_pmc i on p.pmc_id = i.id '
         'join rocpd_kernel_dispatch d on p.event_id = d.event_id '
         'join rocpd_info_kernel_symbol k on d.kernel_id = k.id')
    for ev, kn, cn, v, s, e in c.execute(q):
        per[ev][cn] += float(v)
        names[ev] = kn
        durs[ev] = float(e) - float(s)
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for ev, cs in per.items():
        k = short(names[ev])
        if k is None:
            continue
        for cn, v in cs.items():
            out[k][cn].append(v)
        out[k]['_dur_ns'].append(durs[ev])
    return {k: {cn: sum(v) / len(v) for cn, v in cs.items()} | {'_dispatches': len(cs['_dur_ns'])}
            for k, cs in out.items()}


def main(argv):
    dst, specs = argv[0], argv[1:]
    res = {}
    for spec in specs:
        label, d = spec.split('=', 1)
        for k, cs in load(d).items():
            e = res.setdefault(label, {}).setdefault(k, {})
            pas = d.rstrip('/').split('/')[-1]
            e.setdefault('_passes', []).append(pas)
            for cn, v in cs.items():
                if cn in ('_dur_ns', '_dispatches'):
                    e.setdefault(cn + '_' + pas, v)
                else:
                    e[cn] = v
    for label, ks in res.items():
        for k, e in ks.items():
            durs = [v for n, v in e.items() if n.startswith('_dur_ns')]
            g = e.get('GRBM_GUI_ACTIVE')
            if g:
                cyc = g / 8.0
                dur = [v for n, v in e.items() if n.startswith('_dur_ns') and 'sqa' in n]
                if dur:
                    e['clock_ghz'] = cyc / dur[0]
                simd_cyc = SIMDS * cyc
                if 'SQ_ACTIVE_INST_VALU' in e:
                    e['valu_busy'] = 4 * e['SQ_ACTIVE_INST_VALU'] / simd_cyc
                if 'SQ_INSTS_VALU' in e:
                    e['valu_issue_per_cycle'] = e['SQ_INSTS_VALU'] / simd_cyc
                if 'SQ_WAVE_CYCLES' in e:
                    e['waves_per_simd'] = 4 * e['SQ_WAVE_CYCLES'] / simd_cyc
            if e.get('SQ_WAVE_CYCLES') and 'SQ_WAIT_INST_ANY' in e:
                e['wait_inst_frac'] = e['SQ_WAIT_INST_ANY'] / e['SQ_WAVE_CYCLES']
            if e.get('SQ_WAVE_CYCLES') and 'SQ_WAIT_ANY' in e:
                e['wait_any_frac'] = e['SQ_WAIT_ANY'] / e['SQ_WAVE_CYCLES']
            del durs
    res['_note'] = __doc__.split('usage:')[0].strip()
    with open(dst, 'w') as f:
        json.dump(res, f, indent=1, sort_keys=True)
    tpath = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'traffic.json')
    traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
    for label, ks in res.items():
        if not re.fullmatch(r'cfg\d', label):
            continue
        parts = []
        for k in ('k_score', 'k_score_wave', 'k_score_wave1'):
            e = ks.get(k, {})
            nd = [v for n, v in e.items() if n.startswith('_dispatches')]
            if 'SQ_INSTS_VALU' in e and nd:
                parts.append((nd[0], e['SQ_INSTS_VALU']))
        if parts:
            t = traffic.setdefault(label, {})
            t['valu_insts_per_launch'] = sum(n * v for n, v in parts) / sum(n for n, _ in parts)
            t['_sq_source'] = '%s (SQ_INSTS_VALU, wave64 instructions per score launch)' % (
                os.path.basename(dst))
    with open(tpath, 'w') as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    for label, ks in res.items():
        if label.startswith('_'):
            continue
        for k, e in sorted(ks.items()):
            print(label, k, {n: round(e[n], 3) for n in ('clock_ghz', 'valu_busy', 'valu_issue_per_cycle',
                                                        'waves_per_simd', 'wait_inst_frac',
                                                        'wait_any_frac') if n in e})


if __name__ == '__main__':
    main(sys.argv[1:])
