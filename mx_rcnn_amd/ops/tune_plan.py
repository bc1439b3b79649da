"""Persistent, shareable conv autotune plans (csrc/bindings.cpp ``conv_tune_*``).

The implicit-GEMM conv times its candidate tiles / K splits on the first eager call of a shape
and caches the fastest (MIOpen-find style).  Split-K and K-group candidates sum K in a different
order, so WHICH candidate wins changes the low bits of the result: a timing-based choice would
make reruns -- and, in principle, ranks -- differ.  This module makes the plan an explicit,
reproducible artefact:

* a plan SHIPPED with the package (``mx_rcnn_amd/tune/gfx950.json``, measured on MI355X for the
  benchmark configurations) and, when ``MXR_TUNE_FILE`` names one, a user plan file are loaded
  before the first conv; a shape in the plan is never re-timed, so two runs of the same
  configuration take the same kernels and produce bitwise-equal weights;
* shapes tuned in this process are merged into that user file (:func:`save`) -- the next run
  reuses them.  Without ``MXR_TUNE_FILE`` nothing is read or written outside the package: no
  hidden per-machine state decides which kernels a run takes;
* under data parallelism rank 0's plan is broadcast before the step is captured
  (:func:`sync_from_rank0`), and :func:`plan_hash` goes into the capture-agreement check and
  the benchmark record.

The reference has no autotuner (MXNet's cuDNN algorithm choice is its analogue,
`train_end2end.py:98-105` leaves it at the default); this is part of the MI355X runtime.
"""
import json
import logging
import os
import zlib

ARCH = 'gfx950'
VERSION = 1  # bump when tile codes change meaning: older plan files are then ignored
SHIPPED = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tune', ARCH + '.json')
_STATE = {'loaded': False}


def user_file():
    """The opt-in user plan file (``MXR_TUNE_FILE``), or None."""
    return os.environ.get('MXR_TUNE_FILE') or None


def read_plan(path):
    """-> [(key, tile, splits)] from a plan file ([] when absent or unreadable)."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return []
    if d.get('arch') != ARCH or d.get('version') != VERSION:
        return []
    return [(str(k), int(v[0]), int(v[1])) for k, v in sorted(d.get('plan', {}).items())]


def write_plan(path, entries):
    os.makedirs(os.path.dirname(path) or '.', exist_ok=True)
    tmp = '%s.%d.tmp' % (path, os.getpid())
    with open(tmp, 'w') as f:
        json.dump({'arch': ARCH, 'version': VERSION, 'plan': {k: [t, s] for k, t, s in sorted(entries)}}, f, indent=0, sort_keys=True)
    os.replace(tmp, path)


def ensure_loaded(ext=None):
    """Load the shipped and user plans into the extension once per process (MXR_TUNE_PLAN=0: skip,
    time every shape afresh)."""
    if _STATE['loaded']:
        return
    _STATE['loaded'] = True
    if os.environ.get('MXR_TUNE_PLAN', '1') == '0':
        return
    if ext is None:
        from ._ext import need_ext
        ext = need_ext()
    uf = user_file()
    entries = read_plan(SHIPPED) + (read_plan(uf) if uf else [])  # user entries override shipped ones
    if entries:
        n = ext.conv_tune_set(entries, False)
        logging.debug('conv plan: %d entries loaded (%d in the table)', len(entries), n)


def table(ext=None):
    if ext is None:
        from ._ext import need_ext
        ext = need_ext()
    return sorted((str(k), int(t), int(s)) for k, t, s in ext.conv_tune_table())


def plan_hash(entries=None):
    """CRC32 of the plan (hex): equal on every rank that will run the same kernels."""
    entries = table() if entries is None else sorted(entries)
    blob = '\n'.join('%s=%d,%d' % e for e in entries).encode()
    return '%08x' % (zlib.crc32(blob) & 0xffffffff)


def save(path=None):
    """Merge this process's plan into the user plan file (rank 0 only under DP; a no-op unless a
    path is given or ``MXR_TUNE_FILE`` is set)."""
    if os.environ.get('MXR_TUNE_PLAN', '1') == '0':
        return None
    path = path or user_file()
    if not path:
        return None
    cur = {k: (t, s) for k, t, s in read_plan(path)}
    shipped = {k: (t, s) for k, t, s in read_plan(SHIPPED)}
    new = {k: (t, s) for k, t, s in table() if shipped.get(k) != (t, s)}
    if not new or all(cur.get(k) == v for k, v in new.items()):
        return path
    cur.update(new)
    try:
        write_plan(path, [(k, t, s) for k, (t, s) in cur.items()])
    except OSError as e:  # read-only home: the plan stays per process
        logging.warning('conv plan not saved to %s: %s', path, e)
        return None
    return path


def sync_from_rank0(device=None):
    """Data parallelism: make every rank's plan rank 0's (call after the eager warm-up that tunes,
    before capture).  Returns the plan hash every rank now holds."""
    import torch.distributed as dist
    from ._ext import need_ext
    ext = need_ext()
    mine = table(ext)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return plan_hash(mine)
    box = [mine if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(box, src=0, device=device)
    ext.conv_tune_set(box[0], True)
    return plan_hash(box[0])
