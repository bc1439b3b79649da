"""Per-kernel PMC summary of a rocprofv3 --pmc run (counter_collection.csv): mean counter value per
dispatch for the kernels whose name matches a filter, plus derived ratios.

    python tools/pmc_summary.py DIR [--match conv_igemm_buf_kernel,conv_x2w_kernel] [--label NAME]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--match', default='conv_igemm_buf_kernel,conv_x2w_kernel,conv_dgrad_wgrad_kernel,conv_igemm_kg_kernel,conv_wgrad_buf_kernel')
    ap.add_argument('--label', default='')
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, '**', '*counter_collection.csv'), recursive=True)
    if not files:
        raise SystemExit('no counter_collection.csv under %s' % a.dir)
    pats = [p for p in a.match.split(',') if p]
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get('Kernel_Name', '')
                pat = next((p for p in pats if p in name), None)
                if pat is None:
                    continue
                key = '%s grid=%s' % (pat, row.get('Grid_Size', row.get('Grid_Size_X', '?')))
                acc[key][row['Counter_Name']] += float(row['Counter_Value'])
                disp[key].add(row.get('Dispatch_Id', row.get('Correlation_Id', '')))
    for key in sorted(acc):
        n = max(1, len(disp[key]))
        c = {k: v / n for k, v in acc[key].items()}
        out = {'label': a.label, 'kernel': key, 'dispatches': n}
        out.update({k: round(v, 1) for k, v in sorted(c.items())})
        hit, miss = c.get('TCC_HIT_sum'), c.get('TCC_MISS_sum')
        if hit is not None and miss is not None and hit + miss > 0:
            out['l2_hit_rate'] = round(hit / (hit + miss), 4)
        if c.get('SQ_WAVE_CYCLES'):
            out['wait_frac'] = round(c.get('SQ_WAIT_ANY', 0.0) / c['SQ_WAVE_CYCLES'], 4)
        if c.get('SQ_VALU_MFMA_BUSY_CYCLES') is not None and c.get('GRBM_GUI_ACTIVE'):
            # MFMA-pipe busy cycles summed over the 1024 SIMDs, against the kernel's active cycles
            # (GRBM_GUI_ACTIVE is summed over the 8 XCDs): the fraction of the matrix-core peak in use
            out['mfma_util'] = round(c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['GRBM_GUI_ACTIVE'] / 8.0 * 1024), 4)
        print(json.dumps(out))


if __name__ == '__main__':
    main()
