"""Per-call device chain of a short tpe.suggest loop from a rocprofv3
--kernel-trace --hip-runtime-trace CSV pair: medians of the first launch's
API time, launch-to-first-kernel-start, each kernel's duration, and the span
from the first launch call to the last kernel's end.  Diagnostic only.
usage: call_chain.py <prefix of *_hip_api_trace.csv / *_kernel_trace.csv>"""
import csv
import sys

import numpy as np


def main(prefix):
    api = list(csv.DictReader(open(prefix + '_hip_api_trace.csv')))
    ker = list(csv.DictReader(open(prefix + '_kernel_trace.csv')))
    api_by = {a['Correlation_Id']: (int(a['Start_Timestamp']), int(a['End_Timestamp'])) for a in api}
    ks = sorted((int(k['Start_Timestamp']), int(k['End_Timestamp']), k['Kernel_Name'].split('(')[0],
                 api_by.get(k['Correlation_Id'])) for k in ker)
    # a call = the kernels from one k_fit up to the next (k_publish, when
    # launched, is its last)
    calls, cur = [], None
    for k in ks:
        if 'k_fit' in k[2]:
            if cur:
                calls.append(cur)
            cur = [k]
        elif cur is not None:
            cur.append(k)
    if cur:
        calls.append(cur)
    rows = {}
    for c in calls[10:]:
        first = c[0][3]  # the k_fit launch call (correlation id)
        if first is None:
            continue
        rows.setdefault('k_fit launch API', []).append((first[1] - first[0]) / 1e3)
        rows.setdefault('k_fit launch call -> k_fit start', []).append((c[0][0] - first[0]) / 1e3)
        prev = None
        for s, e, n, a in c:
            nm = n.replace('void ', '')
            if prev is not None:
                rows.setdefault('gap before ' + nm, []).append((s - prev) / 1e3)
            rows.setdefault(nm, []).append((e - s) / 1e3)
            prev = e
        rows.setdefault('k_fit launch call -> last kernel end', []).append((c[-1][1] - first[0]) / 1e3)
    print('%d calls (first 10 skipped); medians in us' % max(len(calls) - 10, 0))
    for k, v in rows.items():
        print('  %-40s %7.1f' % (k[:40], float(np.median(v))))


if __name__ == '__main__':
    main(sys.argv[1])
