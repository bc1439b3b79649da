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


def main(path, steps):
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
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
