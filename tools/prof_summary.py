"""Summarise a rocprofv3 --stats kernel_stats.csv: top kernels, per-step ms, grouped families."""
import csv
import re
import sys


def family(name):
    n = name
    if n.startswith('mxr::') or 'mxr::' in n[:40]:
        return 'HIP(ours) ' + re.sub(r'[<(].*', '', n.split('mxr::')[1])
    if n.startswith('igemm_') or 'gtcx' in n:
        return 'MIOpen conv ' + n.split('_')[1]
    if n.startswith('Cijk'):
        return 'hipBLASLt GEMM'
    if 'rocprim' in n:
        return 'rocPRIM sort'
    if 'batch_norm' in n:
        return 'torch batch_norm'
    if 'elementwise' in n or 'reduce_kernel' in n or 'copyBuffer' in n or 'SubTensor' in n:
        return 'elementwise/copy/reduce'
    return 'other'


def rows_from_db(path, last_n_marker=None):
    """rocprofv3 SQLite (rocpd) output -> kernel_stats-like rows.  With ``last_n_marker`` =
    (kernel-name substring, n), only dispatches after the n-th-from-last occurrence of that
    kernel are kept (steady-state steps, e.g. ('nms_reduce', 10))."""
    import sqlite3
    c = sqlite3.connect(path)
    q = ('select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d '
         'join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start')
    disp = list(c.execute(q))
    if last_n_marker:
        sub, n = last_n_marker
        idx = [i for i, (name, _, _) in enumerate(disp) if sub in name]
        if len(idx) >= n:
            disp = disp[idx[-n]:]
    agg = {}
    for name, s0, e0 in disp:
        a = agg.setdefault(name, [0, 0.0])
        a[0] += 1
        a[1] += e0 - s0
    return [{'Name': k, 'Calls': str(v[0]), 'TotalDurationNs': str(v[1])} for k, v in agg.items()], disp


def main(path, steps, marker=None):
    if path.endswith('.db'):
        rows, disp = rows_from_db(path, (marker, steps) if marker else None)
        if disp:
            span = (disp[-1][2] - disp[0][1]) / 1e6
            print('wall span of the kept dispatches: %.3f ms = %.3f ms/step' % (span, span / steps))
    else:
        rows = list(csv.DictReader(open(path)))
    tot = sum(float(r['TotalDurationNs']) for r in rows)
    print('total GPU kernel time %.3f ms over %d steps = %.3f ms/step' % (tot / 1e6, steps, tot / 1e6 / steps))
    fam = {}
    for r in rows:
        f = family(r['Name'])
        fam[f] = fam.get(f, 0.0) + float(r['TotalDurationNs'])
    print('\n-- by family (ms/step) --')
    for f, v in sorted(fam.items(), key=lambda x: -x[1]):
        print('%9.3f  %5.1f%%  %s' % (v / 1e6 / steps, v / tot * 100, f))
    print('\n-- top kernels --')
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:30]:
        print('%9.3f ms/step %6s calls %5.1f%%  %s' % (float(r['TotalDurationNs']) / 1e6 / steps, r['Calls'],
                                                     float(r['TotalDurationNs']) / tot * 100, r['Name'][:100]))


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1, sys.argv[3] if len(sys.argv) > 3 else None)
