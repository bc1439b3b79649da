"""Summarise rocprofv3 --pmc counter CSVs: per (kernel, counter) the mean over dispatches.

    python tools/pmc_summary.py DIR [DIR ...] [--kernel SUBSTR]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d, kfilter=None):
    out = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get('Kernel_Name', '')
                if kfilter and kfilter not in k:
                    continue
                key = (row.get('Dispatch_Id'), k)
                out[k][row['Counter_Name']].append((key, float(row['Counter_Value'])))
    res = {}
    for k, cs in out.items():
        res[k] = {}
        for c, vals in cs.items():
            per = defaultdict(float)  # sum over dimension instances (XCDs / SEs) per dispatch
            for key, v in vals:
                per[key] += v
            res[k][c] = sum(per.values()) / max(1, len(per))
    return res


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    kf = None
    if '--kernel' in sys.argv:
        kf = sys.argv[sys.argv.index('--kernel') + 1]
        args = [a for a in args if a != kf]
    for d in args:
        for k, cs in load(d, kf).items():
            print('## %s :: %s' % (os.path.basename(d.rstrip('/')), k[:90]))
            for c in sorted(cs):
                print('   %-40s %16.1f' % (c, cs[c]))
            if 'SQ_WAVE_CYCLES' in cs and cs['SQ_WAVE_CYCLES']:
                w = cs['SQ_WAVE_CYCLES']
                print('   -> wait_any %.1f%%  wait_inst %.1f%%' % (100 * cs.get('SQ_WAIT_ANY', 0) / w,
                                                                 100 * cs.get('SQ_WAIT_INST_ANY', 0) / w))
            if 'TCC_HIT_sum' in cs:
                h, m = cs['TCC_HIT_sum'], cs.get('TCC_MISS_sum', 0)
                print('   -> L2 hit %.1f%%' % (100 * h / max(1, h + m)))


if __name__ == '__main__':
    main()
