#!/usr/bin/env python3
"""Fold rocprofv3 outputs (kernel-trace stats + separate --pmc passes) into
profiles/: a per-kernel stats CSV copy, per-kernel PMC averages and
profiles/traffic.json, which bench.py reads for roofline.traffic.

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md (HBM):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads half the
bytes of a wide streaming read, so traffic = 2*FETCH_SIZE*1024 +
WRITE_SIZE*1024 (raw values kept beside it).

usage: tools/prof_summary.py <rocprof out dir> <round tag> <config>
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
        if ', true>' in name:                  # the bench's separate census pass
            return 'k_score_census'
        return 'k_score_erf' if 'k_score<true, false>' in name else 'k_score'
    m = re.search(r'(k_\w+(?:<\d>)?)', name)
    return m.group(1) if m else name.split('(')[0]


def pmc(path):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[(short(r['Kernel_Name']), r['Counter_Name'])].append(float(r['Counter_Value']))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(src, tag, config):
    out = os.path.join(ROOT, 'profiles')
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(src, 'trace', 'run_kernel_stats.csv')
    shutil.copy(stats, os.path.join(out, '%s_%s_kernel_stats.csv' % (tag, config)))
    counters = {}
    for sub in sorted(os.listdir(src)):
        p = os.path.join(src, sub, 'run_counter_collection.csv')
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
    traffic[config] = {'score': v['hbm_bytes'] for k, v in summary.items()
                       if k == 'k_score' and 'hbm_bytes' in v}
    traffic[config]['_source'] = '%s_%s_pmc.json (2*FETCH_SIZE+WRITE_SIZE KiB per launch)' % (
        tag, config)
    with open(tpath, 'w') as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    for k, v in summary.items():
        print(k, {a: round(b, 1) for a, b in v.items()})


if __name__ == '__main__':
    main(*sys.argv[1:4])
