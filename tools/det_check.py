"""Run tools/dp_step_check.py twice per precision (no process group, fixed conv plan) and list every
state array that differs between the two runs -- a run-to-run determinism probe."""
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(out, precision, extra, val=None):
    if val is not None:  # --dirty-val differs between the two runs: a read of unwritten memory shows
        extra = extra + ['--dirty-val', str(val)]
    env = dict(os.environ, MXR_CONV_TUNE='0')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'dp_step_check.py'), out, '--precision', precision,
                        '--steps', '1'] + extra, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=300)
    if r.returncode != 0:
        print(r.stdout[-3000:])
        sys.exit(1)
    return torch.load(out, weights_only=True)


def main():
    tmp = os.environ.get('TMPDIR', '/tmp')
    extra = sys.argv[2:]
    for p in sys.argv[1].split(','):
        vary = '--dirty-gb' in extra
        a = run(os.path.join(tmp, 'det_a.pt'), p, extra, 1000.0 if vary else None)
        b = run(os.path.join(tmp, 'det_b.pt'), p, extra, -7.0 if vary else None)
        keys = [k for k in a if not k.startswith('_')]
        bad = [(k, float((a[k].float() - b[k].float()).abs().max())) for k in keys if not torch.equal(a[k], b[k])]
        print('%s: %d of %d arrays differ' % (p, len(bad), len(keys)), flush=True)
        for k, d in bad:
            print('   %-40s %.3g' % (k, d))


if __name__ == '__main__':
    main()
