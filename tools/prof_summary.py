#!/usr/bin/env python3
"""Fold rocprofv3 outputs (kernel-trace stats + separate --pmc passes) into
profiles/: a per-kernel stats CSV copy, per-kernel PMC averages and
profiles/traffic.json, which bench.py reads for roofline.traffic.

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md (HBM):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads half the
bytes of a wide streaming read, so traffic = 2*FETCH_SIZE*1024 +
WRITE_SIZE*1024 (raw values kept beside it).

A launch of "score" in bench.py's roofline is one level's score launch,
k_score or k_score_wave: traffic.json's figure is the call-weighted mean
over both (census variants excluded).

usage: tools/prof_summary.py <rocprof out dir> <round tag> <config>
       tools/prof_summary.py --dirs <round tag> <config> <trace dir> <pmc dir>...
"""
import collections
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KIND = {0: 'lse_gmm', 1: 'lse_lgmm', 2: 'erf_gmm', 3: 'erf_lgmm', 4: 'categorical'}


def short(name):
    if 'k_score' in name:   # k_score<erf, census>: the census variants run in
        if ', true>' in name or 'k_score_wave<true' in name or 'k_score_wave1<true' in name:
            return 'k_score_census'  # (the census pass)
        if 'k_score_wave' in name:
            return 'k_score_wave'
        return 'k_score_erf' if 'k_score<true, false>' in name else 'k_score'
    m = re.search(r'(k_\w+(?:<\d>)?)', name)
    return m.group(1) if m else name.split('(')[0]


def pmc(path):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[(short(r['Kernel_Name']), r['Counter_Name'])].append(float(r['Counter_Value']))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(src, tag, config, trace=None, pmc_dirs=None):
    out = os.path.join(ROOT, 'profiles')
    os.makedirs(out, exist_ok=True)
    if trace is None:
        trace = os.path.join(src, 'trace')
        pmc_dirs = [os.path.join(src, sub) for sub in sorted(os.listdir(src))]
    stats = os.path.join(trace, 'run_kernel_stats.csv')
    shutil.copy(stats, os.path.join(out, '%s_%s_kernel_stats.csv' % (tag, config)))
    counters = {}
    for d in pmc_dirs:
        p = os.path.join(d, 'run_counter_collection.csv')
        if os.path.exists(p):
            for (k, c), v in pmc(p).items():
                counters.setdefault(k, {})[c] = v
    durations = {}
    for r in csv.DictReader(open(stats)):
        durations[short(r['Name'])] = dict(calls=int(r['Calls']), avg_ns=float(r['AverageNs']))
    summary = {}
    for k in sorted(set(counters) | set(durations)):
        e = dict(durations.get(k, {}))
        e.update(counters.get(k, {}))
        if 'FETCH_SIZE' in e and 'WRITE_SIZE' in e:
            e['hbm_bytes'] = 2 * e['FETCH_SIZE'] * 1024 + e['WRITE_SIZE'] * 1024
        summary[k] = e
    with open(os.path.join(out, '%s_%s_pmc.json' % (tag, config)), 'w') as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    tpath = os.path.join(ROOT, 'traffic.json')
    traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
    parts = [(v['calls'], v['hbm_bytes']) for k, v in summary.items()
             if k in ('k_score', 'k_score_wave') and 'hbm_bytes' in v and 'calls' in v]
    traffic[config] = {}
    if parts:
        traffic[config]['score'] = sum(c * b for c, b in parts) / sum(c for c, _ in parts)
    traffic[config]['_source'] = '%s_%s_pmc.json (2*FETCH_SIZE+WRITE_SIZE KiB per launch)' % (
        tag, config)
    with open(tpath, 'w') as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    for k, v in summary.items():
        print(k, {a: round(b, 1) for a, b in v.items()})


if __name__ == '__main__':
    if sys.argv[1] == '--dirs':
        main(None, sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5:])
    else:
        main(*sys.argv[1:4])
