"""Windowed loss curve from a Speedometer log (core/callback.py, reference `rcnn/callback.py`).

The Speedometer prints each metric's running average since the start of the epoch every
``frequent`` batches; consecutive lines of an epoch give the average over the window between
them: (n2 * avg2 - n1 * avg1) / (n2 - n1).  Prints one JSON line per window (global step, the
four losses and their sum) and a summary of how the summed loss moves window to window.

    python tools/speedometer_windows.py LOG [--every 1000]
"""
import argparse
import json
import re

LINE = re.compile(r'Epoch\[(\d+)\] Batch \[(\d+)\]\s+Speed: ([\d.]+) samples/sec\s+(.*)')
LOSSES = ('RPN-LogLoss', 'RPN-SmoothL1Loss', 'LogLoss', 'SmoothL1Loss')


def windows(path):
    prev = {}
    out = []
    step0 = {}  # global step at the start of each epoch
    last_epoch, last_batch, base = None, 0, 0
    with open(path) as f:
        for line in f:
            m = LINE.search(line)
            if not m:
                continue
            ep, nb, speed = int(m.group(1)), int(m.group(2)), float(m.group(3))
            vals = dict(kv.split('=') for kv in m.group(4).split() if kv.startswith('Train-'))
            vals = {k[len('Train-'):]: float(v) for k, v in vals.items()}
            if ep != last_epoch:
                if last_epoch is not None:
                    base += last_batch
                step0[ep] = base
                prev = {}
                last_epoch = ep
            n1 = prev.get('_n', 0)
            rec = {'epoch': ep, 'step': base + nb, 'speed': speed}
            for k in LOSSES:
                if k in vals:
                    a1 = prev.get(k, 0.0)
                    rec[k] = round((nb * vals[k] - n1 * a1) / max(nb - n1, 1), 5)
            rec['loss_sum'] = round(sum(rec.get(k, 0.0) for k in LOSSES), 5)
            out.append(rec)
            prev = dict(vals)
            prev['_n'] = nb
            last_batch = nb
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('log')
    ap.add_argument('--every', type=int, default=0, help='merge windows to about this many steps')
    a = ap.parse_args()
    ws = windows(a.log)
    if a.every:
        merged, acc, n0 = [], None, 0
        for w in ws:
            if acc is None:
                acc, n0 = dict(w), 1
            else:
                for k in LOSSES + ('loss_sum',):
                    acc[k] = acc.get(k, 0.0) + w.get(k, 0.0)
                n0 += 1
                acc['step'] = w['step']
            if acc['step'] // a.every != (acc['step'] - 1) // a.every or w is ws[-1]:
                for k in LOSSES + ('loss_sum',):
                    acc[k] = round(acc[k] / n0 if n0 > 1 else acc[k], 5)
                merged.append(acc)
                acc = None
        ws = merged
    for w in ws:
        print(json.dumps(w))
    s = [w['loss_sum'] for w in ws]
    falls = sum(1 for x, y in zip(s, s[1:]) if y < x)
    print(json.dumps({'windows': len(s), 'first': s[0] if s else None, 'last': s[-1] if s else None,
                      'falling_transitions': falls, 'transitions': max(len(s) - 1, 0)}))


if __name__ == '__main__':
    main()
