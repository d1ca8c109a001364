#!/usr/bin/env python3
"""Median kernel timeline of one suggest step from a rocprofv3 --kernel-trace
--output-format csv run (<dir>/run_kernel_trace.csv): the steps are split at
each k_fit, the most common kernel sequence is kept, and each kernel's start
and end (us from its step's k_fit start) are the medians over those steps.
Diagnostic only.  usage: step_timeline.py <dir>"""
import collections
import csv
import sys

import numpy as np


def main(d):
    ker = list(csv.DictReader(open(d + '/run_kernel_trace.csv')))
    ks = sorted((int(k['Start_Timestamp']), int(k['End_Timestamp']),
                 k['Kernel_Name'].split('(')[0].replace('void ', ''), k.get('Stream_Id', ''))
                for k in ker)
    calls, cur = [], None
    for k in ks:
        if 'k_fit' in k[2]:
            if cur:
                calls.append(cur)
            cur = [k]
        elif cur is not None and 'micro' not in k[2]:
            cur.append(k)
    if cur:
        calls.append(cur)
    sig = collections.Counter(tuple(x[2] for x in c) for c in calls)
    top, cnt = sig.most_common(1)[0]
    print('%d steps, %d with the typical sequence' % (len(calls), cnt))
    rows = collections.defaultdict(list)
    ends = []
    for c in calls:
        if tuple(x[2] for x in c) != top:
            continue
        t0 = c[0][0]
        for i, (s, e, n, st) in enumerate(c):
            rows[(i, n, st)].append(((s - t0) / 1e3, (e - t0) / 1e3))
        ends.append((max(x[1] for x in c) - t0) / 1e3)
    for (i, n, st), v in rows.items():
        a = np.median(np.array(v), axis=0)
        print('  %2d %-55s stream %-3s start %7.1f end %7.1f' % (i, n[:55], st, a[0], a[1]))
    print('  step end (last kernel end, median): %.1f us' % float(np.median(ends)))


if __name__ == '__main__':
    main(sys.argv[1])
