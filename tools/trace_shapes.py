"""Per-launch-shape breakdown of a rocprofv3 kernel trace over the last N steps.

    python tools/trace_shapes.py gpurun_out/prof/run_kernel_trace.csv 10 nms_reduce [name_filter]
"""
import csv
import sys


def main(path, steps, marker, filt=''):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    idx = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    rows = rows[idx[-steps]:] if len(idx) >= steps else rows
    span = (int(rows[-1]['End_Timestamp']) - int(rows[0]['Start_Timestamp'])) / 1e6
    busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in rows) / 1e6
    print('last %d steps: wall %.3f ms/step, kernel-busy %.3f ms/step, %d launches/step' % (
        steps, span / steps, busy / steps, len(rows) // steps))
    agg = {}
    for r in rows:
        n = r['Kernel_Name']
        if filt and filt not in n:
            continue
        key = (n[:70], int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X'])), r['Grid_Size_Y'])
        a = agg.setdefault(key, [0, 0.0])
        a[0] += 1
        a[1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    tot = sum(v[1] for v in agg.values())
    print('%d shapes, %.3f ms/step in filter' % (len(agg), tot / 1e3 / steps))
    for (n, gx, gy), (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:60]:
        print('%8.1f us/step %4d/step avg %6.2f us  wg %6d x %s  %s' % (us / steps, c // steps, us / c, gx, gy, n))


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else '')
