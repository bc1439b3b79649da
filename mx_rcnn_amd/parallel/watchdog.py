"""Step heartbeat and stall watchdog (SURVEY §5.3 failure detection).

The reference has no failure detection beyond the proposal NaN guard
(rcnn/rpn/proposal.py NaN check): a hung rank simply blocks the kvstore reduce
forever.  Here every rank runs a daemon thread that

* watches its own training loop: if ``beat()`` has not been called for ``stall_s`` seconds
  (a hung collective, a wedged data loader, a kernel that never returns) it reports a
  ``local`` stall once per stalled step -- by default an ERROR log line plus a dump of every
  Python thread's stack -- and, with ``abort=True``, ends the process with exit code 124 so
  that torchrun tears the job down instead of waiting on a dead ring;
* publishes ``(step, wall time of its last beat)`` under ``mxr_hb/<rank>`` in the process
  group's key-value store (the same TCPStore the RCCL rendezvous uses; no extra sockets), and
  on rank 0 reads every peer's entry and reports a ``peer`` stall for a rank whose last beat
  is older than ``stall_s`` -- naming the rank and the step it stopped at.

The beat is a host-side integer store (no device sync), so it is free inside the hipGraph
step loop.  Enabled in ``Module.fit`` by ``MXR_WATCHDOG=<stall seconds>``
(``MXR_WATCHDOG_ABORT=1`` to abort on a local stall).
"""
import faulthandler
import logging
import os
import sys
import threading
import time

import torch.distributed as dist

KEY = 'mxr_hb/%d'


def default_store():
    """The default process group's store, or None (single process / not initialised)."""
    if not (dist.is_available() and dist.is_initialized()):
        return None
    try:
        return dist.distributed_c10d._get_default_store()
    except Exception:  # private accessor: degrade to local-only watching
        return None


class Heartbeat:
    def __init__(self, stall_s=600.0, period_s=None, rank=None, world=None, store='default', on_stall=None,
                 abort=False):
        self.stall_s = float(stall_s)
        self.period_s = float(period_s) if period_s is not None else max(0.05, min(10.0, self.stall_s / 4))
        self.rank = dist.get_rank() if rank is None and dist.is_initialized() else (rank or 0)
        self.world = dist.get_world_size() if world is None and dist.is_initialized() else (world or 1)
        self.store = default_store() if store == 'default' else store
        self.on_stall = on_stall or self._report
        self.abort = abort
        self._step = -1
        self._last = time.monotonic()
        self._last_wall = time.time()
        self._reported_local = None
        self._reported_peer = {}
        self._paused = 0
        self._stop = threading.Event()
        self._thread = None
        self.stalls = []  # (kind, rank, step, age_s) -- kept for tests and post-mortems

    # ------------------------------------------------------------------ API
    def beat(self, step):
        self._step = int(step)
        self._last = time.monotonic()
        self._last_wall = time.time()

    def pause(self):
        """Enter a known long host phase (graph capture, checkpoint write, epoch-end gather):
        no local stall is reported and peers see this rank as alive until :meth:`resume`."""
        self._paused += 1

    def resume(self, step=None):
        self._paused = max(0, self._paused - 1)
        self.beat(self._step if step is None else step)

    def paused(self):
        """``with hb.paused(): ...`` -- pause/resume around a block."""
        import contextlib

        @contextlib.contextmanager
        def _cm():
            self.pause()
            try:
                yield self
            finally:
                self.resume()
        return _cm()

    def start(self):
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name='mxr-heartbeat', daemon=True)
            self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5 * self.period_s + 1)
            self._thread = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    # ------------------------------------------------------------------ thread
    def _run(self):
        while not self._stop.wait(self.period_s):
            try:
                self._tick()
            except Exception as e:  # a store that went away (peer shutdown) must not kill training
                logging.debug('heartbeat tick failed: %s', e)

    def _tick(self):
        if self._paused:
            self._last, self._last_wall = time.monotonic(), time.time()
        step, age = self._step, time.monotonic() - self._last
        if self.store is not None:
            # the time of the last beat, not of this publish: a rank whose loop is stuck but
            # whose heartbeat thread still runs must look stale to rank 0
            self.store.set(KEY % self.rank, '%d %.3f' % (step, self._last_wall))
        if age > self.stall_s and self._reported_local != step:
            self._reported_local = step
            self._fire('local', self.rank, step, age)
        if self.store is not None and self.rank == 0:
            now = time.time()
            for r in range(1, self.world):
                k = KEY % r
                if not self.store.check([k]):
                    continue
                s, t = self.store.get(k).decode().split()
                s, page = int(s), now - float(t)
                if page > self.stall_s and self._reported_peer.get(r) != s:
                    self._reported_peer[r] = s
                    self._fire('peer', r, s, page)

    def _fire(self, kind, rank, step, age):
        self.stalls.append((kind, rank, step, age))
        self.on_stall(kind, rank, step, age)
        if kind == 'local' and self.abort:
            logging.error('watchdog: aborting rank %d', self.rank)
            sys.stderr.flush()
            os._exit(124)

    def _report(self, kind, rank, step, age):
        if kind == 'local':
            logging.error('watchdog: rank %d made no progress for %.0f s after step %d; thread stacks follow',
                          rank, age, step)
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        else:
            logging.error('watchdog: peer rank %d made no progress for %.0f s (last step %d)',
                          rank, age, step)


def from_env():
    """``MXR_WATCHDOG=<stall seconds>`` -> a started Heartbeat, else None."""
    v = os.environ.get('MXR_WATCHDOG')
    if not v:
        return None
    return Heartbeat(float(v), abort=os.environ.get('MXR_WATCHDOG_ABORT', '0') == '1').start()
