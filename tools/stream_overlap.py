"""Per-queue busy time, chip-level idle time and the critical-path picture of graph-replayed
training steps from a rocprofv3 kernel trace.

    python tools/stream_overlap.py gpurun_out/prof/run_kernel_trace.csv [--marker nms_reduce_mc] [--steps 5]

Steps are delimited by a once-per-step marker kernel; the last --steps complete steps are used.
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--marker', default='nms_reduce_mc')
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--gaps', type=int, default=15, help='largest idle gaps to list')
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    mk = [i for i, r in enumerate(rows) if a.marker in r['Kernel_Name']]
    s0, s1 = mk[-a.steps - 1], mk[-1]
    seg = rows[s0:s1]
    t0, t1 = int(seg[0]['Start_Timestamp']), int(rows[s1]['Start_Timestamp'])
    n = a.steps
    print('wall per step %.3f ms (marker %s)' % ((t1 - t0) / n / 1e6, a.marker))
    byq = collections.defaultdict(list)
    for r in seg:
        byq[r['Queue_Id']].append(r)
    for q, rs in sorted(byq.items()):
        busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in rs)
        top = collections.Counter()
        for r in rs:
            top[r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0][:48]] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        print('queue %s: %.1f launches/step, busy %.3f ms/step; top: %s' % (
            q, len(rs) / n, busy / n / 1e6, ', '.join('%s %.2f' % (k, v / n / 1e6) for k, v in top.most_common(4))))
    iv = sorted((int(r['Start_Timestamp']), min(int(r['End_Timestamp']), t1), r['Kernel_Name']) for r in seg)
    union, gaps = 0, []
    cs, ce, cn = iv[0]
    for s, e, nm in iv[1:]:
        if s > ce:
            union += ce - cs
            gaps.append((s - ce, cn, nm))
            cs, ce, cn = s, e, nm
        else:
            if e > ce:
                ce, cn = e, nm
    union += ce - cs
    print('chip busy (any kernel) %.3f ms/step, fully idle %.3f ms/step in %d gaps/step' % (
        union / n / 1e6, (t1 - t0 - union) / n / 1e6, len(gaps) / n))
    agg = collections.Counter()
    for g, before, after in gaps:
        agg[(before.replace('(anonymous namespace)::', '').split('(')[0][:48], after.replace('(anonymous namespace)::', '').split('(')[0][:48])] += g
    print('largest idle transitions (us/step):')
    for (b, f), g in agg.most_common(a.gaps):
        print('  %7.1f  %s -> %s' % (g / n / 1e3, b, f))


if __name__ == '__main__':
    main()
