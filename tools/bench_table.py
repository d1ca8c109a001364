#!/usr/bin/env python3
"""One line per bench.py JSON file of a gpurun output directory: ms per step,
scoring launch time, roofline fraction, v_exp_f32 issue fraction and the
moment-form pair counts.  usage: bench_table.py <dir> [name ...]"""
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    names = sys.argv[2:] or sorted(os.path.basename(f)[:-5] for f in glob.glob(os.path.join(d, '*.json')))
    for f in names:
        try:
            b = json.load(open(os.path.join(d, f + '.json')))
        except Exception as e:  # noqa: BLE001
            print('%-16s %s' % (f, e))
            continue
        r = b['roofline']
        print('%-16s ms/step %10.4f  launch %9.4f ms  frac %.3f  exp %.3f  mom %.3g mom8 %.3g '
              'eval %.3g' % (f, b['ms_per_step'], r['avg_launch_ms'], r['frac'] or 0,
                             r.get('exp_issue_frac') or 0,
                             r.get('lse_evaluated_moment_pairs_per_launch', 0),
                             r.get('lse_evaluated_moment8_pairs_per_launch', 0),
                             r['lse_evaluated_pairs_per_launch']))


if __name__ == '__main__':
    main()
