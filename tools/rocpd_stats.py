#!/usr/bin/env python3
"""Read rocprofv3's default rocpd SQLite output (<dir>/run_results.db) and
write the CSVs tools/prof_summary.py folds into profiles/:
  kernel trace  -> <dir>/run_kernel_stats.csv (Name, Calls, TotalDurationNs, AverageNs, ...)
  --pmc pass    -> <dir>/run_counter_collection.csv (Kernel_Name, Counter_Name, Counter_Value)
usage: rocpd_stats.py [--schema] <dir> [<dir> ...]      (reporting only)"""
import csv
import os
import sqlite3
import statistics
import sys


def tables(c):
    return [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]


def cols(c, t):
    return [r[1] for r in c.execute('pragma table_info("%s")' % t)]


def kernel_stats(c, out):
    durs = {}
    for n, s, e in c.execute('select coalesce(nullif(k.display_name, ""), k.kernel_name), d.start, d."end" from rocpd_kernel_dispatch d '
                             'join rocpd_info_kernel_symbol k on d.kernel_id = k.id'):
        durs.setdefault(n, []).append(float(e) - float(s))
    if not durs:
        return False
    tot_all = sum(sum(v) for v in durs.values())
    with open(out, 'w', newline='') as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage', 'MinNs',
                    'MaxNs', 'StdDev'])
        for n, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([n, len(v), int(sum(v)), sum(v) / len(v), 100.0 * sum(v) / tot_all,
                        int(min(v)), int(max(v)), statistics.pstdev(v)])
    return True


def counters(c, out):
    rows = list(c.execute('select coalesce(nullif(k.display_name, ""), k.kernel_name), i.name, p.value from rocpd_pmc_event p '
                          'join rocpd_info_pmc i on p.pmc_id = i.id '
                          'join rocpd_kernel_dispatch d on p.event_id = d.event_id '
                          'join rocpd_info_kernel_symbol k on d.kernel_id = k.id'))
    if not rows:
        return False
    with open(out, 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['Kernel_Name', 'Counter_Name', 'Counter_Value'])
        w.writerows(rows)
    return True


def main(argv):
    schema = argv[:1] == ['--schema']
    for d in argv[1:] if schema else argv:
        c = sqlite3.connect(os.path.join(d, 'run_results.db'))
        if schema:
            for t in tables(c):
                print(d, t, cols(c, t))
            continue
        for fn, name in ((kernel_stats, 'run_kernel_stats.csv'),
                         (counters, 'run_counter_collection.csv')):
            try:
                if fn(c, os.path.join(d, name)):
                    print(d, 'wrote', name)
            except sqlite3.Error as e:
                print(d, name, 'skipped:', e)


if __name__ == '__main__':
    main(sys.argv[1:])
