"""Single-command multi-GPU launch: one fresh child process per GPU.

The reference takes ``--gpus 0,1,2,3`` and builds one MXNet context per device inside a single
process (`train_end2end.py:168`, `run.sh:7-8`).  On MI355X the engine is one process per GPU
over RCCL, so the entry points that accept ``--gpus`` re-launch themselves: the parent starts
N children with ``RANK`` / ``LOCAL_RANK`` / ``WORLD_SIZE`` / ``MASTER_ADDR`` / ``MASTER_PORT``
set (the torchrun contract), waits for them, and exits with the first failure's code.

The parent NEVER initialises the GPU: call :func:`maybe_spawn` before anything touches HIP
(importing torch is fine; ``torch.cuda.is_available()`` is not).  Children are started with
``subprocess`` (no fork of a HIP-initialised process, no exec of the parent).  If one child
fails, the others are terminated by PID (they would otherwise block in a collective forever).

This module imports nothing heavy so entry scripts can call it before ``import torch``.
"""
import os
import signal
import socket
import subprocess
import sys
import time

_RANK_VARS = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE', 'GROUP_RANK', 'MASTER_ADDR', 'MASTER_PORT')


def free_port(host='127.0.0.1'):
    s = socket.socket()
    s.bind((host, 0))
    port = s.getsockname()[1]
    s.close()
    return port


def parse_gpus(spec):
    """Number of ranks for ``--gpus``: the length of the reference's device list (``'0,1,2'`` -> 3,
    ``'3'`` -> 1: device 3), or an int count (bench.py)."""
    return len(device_ids(spec))


def device_ids(spec):
    """The reference's ``--gpus`` device list (`train_end2end.py:168`): ``'0,1,2'`` -> [0, 1, 2],
    ``'3'`` -> [3] (one device, the one named), ``''`` -> [0].  An int (bench.py's ``--gpus N``)
    is a count: [0 .. N-1]."""
    if isinstance(spec, int):
        return list(range(max(1, spec)))
    spec = str(spec).strip()
    ids = [int(t) for t in spec.split(',') if t.strip() != '']
    return ids or [0]


def visible_mask(with_source=False):
    """The device list a scheduler already restricted this job to (``HIP_VISIBLE_DEVICES``, else
    ``CUDA_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES``), or None when every device is visible.
    ``with_source``: -> (list, variable name) / (None, None)."""
    for var in ('HIP_VISIBLE_DEVICES', 'CUDA_VISIBLE_DEVICES', 'ROCR_VISIBLE_DEVICES'):
        v = os.environ.get(var)
        if v is not None and v.strip() != '':
            ids = [t.strip() for t in v.split(',') if t.strip() != '']
            return (ids, var) if with_source else ids
    return (None, None) if with_source else None


def map_devices(ids, mask=None, source='HIP_VISIBLE_DEVICES'):
    """``--gpus`` ids index the devices this job can see, like the reference's ``mx.gpu(i)`` ->
    the ``HIP_VISIBLE_DEVICES`` entries that select them.

    HIP applies ``HIP_VISIBLE_DEVICES`` (or, when unset, ``CUDA_VISIBLE_DEVICES``) ON TOP of the
    devices ROCr exposes.  So with a HIP / CUDA mask (e.g. HIP_VISIBLE_DEVICES=4,5,6,7 from a
    scheduler) id i is the mask's i-th entry -- ``--gpus 2,3`` runs on devices 6 and 7 -- and the
    new HIP mask replaces the old one.  A ``ROCR_VISIBLE_DEVICES`` mask has already renumbered the
    devices 0..k-1 below HIP, so the HIP mask must hold the indices themselves.  An id outside the
    mask is an error."""
    if mask is None:
        mask, source = visible_mask(with_source=True)
    if mask is None:
        return [str(i) for i in ids]
    bad = [i for i in ids if i < 0 or i >= len(mask)]
    if bad:
        raise SystemExit('--gpus %s: device(s) %s outside the %d visible device(s) %s' % (
            ','.join(str(i) for i in ids), bad, len(mask), ','.join(mask)))
    if source == 'ROCR_VISIBLE_DEVICES':
        return [str(i) for i in ids]
    return [mask[i] for i in ids]


def select_devices(spec):
    """Make this job run on the devices ``spec`` names (indices into the visible devices, see
    :func:`map_devices`).  More than one: returns the ``HIP_VISIBLE_DEVICES`` list for the rank
    children (rank r uses visible device r).  One: restricts THIS process to it (before anything
    touches the GPU) and returns None."""
    ids = device_ids(spec)
    if launched_rank():
        return None  # the launcher placed this rank already
    mask, source = visible_mask(with_source=True)
    vis = ','.join(map_devices(ids, mask, source))
    if len(ids) > 1:
        return vis
    if ids != [0] or source in ('HIP_VISIBLE_DEVICES', 'CUDA_VISIBLE_DEVICES'):
        os.environ['HIP_VISIBLE_DEVICES'] = vis
    return None


def launched_rank():
    """True when this process already is one rank of a launched job (torchrun or ours)."""
    return 'WORLD_SIZE' in os.environ and 'RANK' in os.environ


def spawn_local(nprocs, argv, master_addr='127.0.0.1', master_port=None, extra_env=None, poll_s=0.2):
    """Run ``python argv...`` as ``nprocs`` ranks on this node; returns the job's exit code
    (0 when every rank exited 0, else the first non-zero code observed)."""
    port = master_port or free_port(master_addr)
    procs = []
    for r in range(nprocs):
        env = {k: v for k, v in os.environ.items() if k not in _RANK_VARS}
        env.update(extra_env or {})
        env.update({'RANK': str(r), 'LOCAL_RANK': str(r), 'WORLD_SIZE': str(nprocs),
                    'LOCAL_WORLD_SIZE': str(nprocs), 'GROUP_RANK': '0', 'MASTER_ADDR': master_addr,
                    'MASTER_PORT': str(port)})
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=env))
    rc = 0

    def _terminate(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except ProcessLookupError:
                    pass

    prev = {}
    for s in (signal.SIGINT, signal.SIGTERM):
        try:
            prev[s] = signal.signal(s, lambda signum, _f: _terminate(signum))
        except ValueError:  # not the main thread
            pass
    try:
        alive = set(range(nprocs))
        while alive:
            for r in sorted(alive):
                code = procs[r].poll()
                if code is None:
                    continue
                alive.discard(r)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code  # -SIG -> 128+SIG like a shell
                    sys.stderr.write('[spawn] rank %d exited with %d; stopping the other ranks\n' % (r, code))
                    _terminate()
            if alive:
                time.sleep(poll_s)
    finally:
        deadline = time.time() + 30
        for p in procs:
            if p.poll() is None:
                try:
                    p.wait(timeout=max(0.1, deadline - time.time()))
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
        for s, h in prev.items():
            signal.signal(s, h)
    return rc


def maybe_spawn(n_gpus, script, argv, visible=None):
    """Entry-script helper.  ``n_gpus`` > 1 and not already a launched rank -> run the job
    (``script argv``) as ``n_gpus`` children and ``sys.exit`` with its code.  ``visible``: the
    ``HIP_VISIBLE_DEVICES`` list the children get (the user's ``--gpus`` device ids), so rank r
    runs on the r-th named device.  Inside a launched job, check that the launcher's world size
    agrees with ``--gpus``."""
    if launched_rank():
        world = int(os.environ['WORLD_SIZE'])
        if n_gpus > 1 and world != n_gpus:
            raise SystemExit('--gpus %d but the launcher started WORLD_SIZE=%d ranks' % (n_gpus, world))
        return
    if n_gpus > 1:
        extra = {'HIP_VISIBLE_DEVICES': visible} if visible else None
        sys.exit(spawn_local(n_gpus, [script] + list(argv), extra_env=extra))
