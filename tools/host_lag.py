#!/usr/bin/env python3
"""Host issue against device start for one suggest step, from a rocprofv3
--kernel-trace --hip-runtime-trace --output-format csv run: for each kernel of
the typical step (split at k_fit), the median time (us from the step's k_fit
start) at which its launch API call began and ended on the host, and at which
the kernel started and ended on the device.  A kernel that starts right
after its launch call ended, with the device idle before, waited on the
host.  Diagnostic only.  usage: host_lag.py <dir>"""
import collections
import csv
import sys

import numpy as np


def main(d):
    api = {}
    for a in csv.DictReader(open(d + '/run_hip_api_trace.csv')):
        if 'Launch' in a['Function']:
            api[a['Correlation_Id']] = (int(a['Start_Timestamp']), int(a['End_Timestamp']))
    ks = []
    for k in csv.DictReader(open(d + '/run_kernel_trace.csv')):
        ks.append((int(k['Start_Timestamp']), int(k['End_Timestamp']),
                   k['Kernel_Name'].split('(')[0].replace('void ', ''), api.get(k['Correlation_Id'])))
    ks.sort()
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
    print('%d steps, %d typical' % (len(calls), cnt))
    rows = collections.defaultdict(list)
    for c in calls:
        if tuple(x[2] for x in c) != top or any(x[3] is None for x in c):
            continue
        t0 = c[0][0]
        for i, (s, e, n, a) in enumerate(c):
            rows[(i, n)].append(((a[0] - t0) / 1e3, (a[1] - t0) / 1e3, (s - t0) / 1e3, (e - t0) / 1e3))
    for (i, n), v in rows.items():
        m = np.median(np.array(v), axis=0)
        print('  %2d %-50s launch call %7.1f .. %7.1f   kernel %7.1f .. %7.1f' % (i, n[:50], *m))


if __name__ == '__main__':
    main(sys.argv[1])
