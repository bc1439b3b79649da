"""Group a rocprofv3 kernel_trace.csv by (kernel, grid, workgroup) over the last N steps.

    python tools/trace_groups.py gpurun_out/prof/run_kernel_trace.csv [--marker nms_reduce_mc] [--steps 10] [--top 60]

A "step" boundary is an occurrence of the marker kernel (one per training step).  Prints, per
launch shape: ms/step, launches/step, mean us, VGPRs, LDS bytes -- enough to map the dispatches of
one kernel template back to the layers that issue them.
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    n = re.sub(r'\(.*', '', name)
    n = n.replace('void ', '').replace('mxr::', '')
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--marker', default='nms_reduce_mc')
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--top', type=int, default=60)
    ap.add_argument('--filter', default='')
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    marks = [i for i, r in enumerate(rows) if args.marker in r['Kernel_Name']]
    steps = min(args.steps, len(marks) - 1) if len(marks) > 1 else 1
    start = marks[-steps - 1] + 1 if len(marks) > steps else 0
    end = marks[-1] + 1 if marks else len(rows)
    sel = rows[start:end]
    g = defaultdict(lambda: [0, 0.0, None])
    total = 0.0
    for r in sel:
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        total += d
        key = (short(r['Kernel_Name']), r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'], r['Workgroup_Size_X'])
        e = g[key]
        e[0] += 1
        e[1] += d
        e[2] = (r['VGPR_Count'], r['Accum_VGPR_Count'], r['LDS_Block_Size'])
    wall = (int(sel[-1]['End_Timestamp']) - int(sel[0]['Start_Timestamp'])) / 1e3 if sel else 0
    print('steps=%d  kernel time %.3f ms/step  wall(first start->last end) %.3f ms/step  launches/step %.0f'
          % (steps, total / steps / 1e3, wall / steps / 1e3, len(sel) / steps))
    items = sorted(g.items(), key=lambda kv: -kv[1][1])
    print('%9s %6s %9s  %-70s %s' % ('ms/step', 'n/step', 'us/call', 'kernel', 'grid x,y,z / wg  (vgpr,agpr,lds)'))
    for (k, gx, gy, gz, wg), (n, t, meta) in items[:args.top]:
        if args.filter and args.filter not in k:
            continue
        print('%9.3f %6.1f %9.1f  %-70s %s,%s,%s / %s %s' % (t / steps / 1e3, n / steps, t / n, k, gx, gy, gz, wg, meta))


if __name__ == '__main__':
    main()
