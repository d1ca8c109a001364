#!/usr/bin/env python3
"""Average PMC counters per kernel from rocprofv3 --pmc passes under <dir>/*/.
usage: pmc_print.py <dir> <kernel substring>"""
import collections
import csv
import glob
import sys

d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + '/*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if sys.argv[2] in r['Kernel_Name']:
            d[(r['Kernel_Name'][:40], r['Counter_Name'])].append(float(r['Counter_Value']))
for (k, c), v in sorted(d.items()):
    print('%-40s %-28s %14.0f  (n=%d)' % (k, c, sum(v) / len(v), len(v)))
