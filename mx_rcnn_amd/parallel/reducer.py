"""Bucketed gradient all-reduce overlapped with backward.

Gradients live in flat per-group buffers (core/params.py) ordered by gradient readiness.
Each buffer is cut into buckets of ~``bucket_mb``; a post-accumulate-grad hook counts the
parameters of each bucket and, when the last one lands, issues an async ``all_reduce(SUM)``
on that slice.  RCCL runs it on its own stream (ordered after the compute stream's prior
work), so the reduction of the head / stage-4 / fc6 gradients overlaps the rest of the
backward pass.  ``finish()`` makes the compute stream wait on every outstanding bucket
before the optimizer touches the buffers -- no host blocking.

Semantics: SUM across ranks (MXNet kvstore 'device', rescale_grad=1: `train_end2end.py:104`);
``average=True`` switches to mean.  Bucket sizing: xGMI is point-to-point, a ring uses one
link per hop, so messages must stay large enough to run at link bandwidth (a 25 MB ring
all-reduce over 8 GPUs is bandwidth-, not latency-bound), but small enough that the first
buckets are reduced while most of the backward is still running: the default 25 MB cuts
ResNet-101's ~90 MB of bf16 gradients into 4 buckets, the last of which is the only exposed one;
VGG16's fc6 (205 MB bf16) still gets a bucket of its own.
"""
import os

import torch
import torch.distributed as dist

from ..ops import grad_sink
from .dist import get_world_size, is_distributed


class _Bucket:
    __slots__ = ('buf', 'start', 'end', 'names', 'pending', 'work')

    def __init__(self, buf, start, end):
        self.buf, self.start, self.end = buf, start, end
        self.names = []
        self.pending = 0
        self.work = None


class BucketReducer:
    def __init__(self, store, bucket_mb=25, average=False, overlap=True):
        self.store = store
        self.world = get_world_size()
        self.average = average
        self.overlap = overlap and is_distributed()
        self.buckets = []
        self._param_bucket = {}
        self._hooks = []
        if not is_distributed() or (self.world == 1 and os.environ.get('MXR_FORCE_DIST', '0') != '1'):
            return
        for g in store.groups:
            esize = g.grad.element_size()
            cap = max(1, int(bucket_mb * (1 << 20) // esize))
            cur = None
            for (n, _, _, numel, _, _), off in zip(g.entries, g.offsets):
                if cur is None or (off + numel - cur.start > cap and cur.end > cur.start):
                    cur = _Bucket(g.grad, off, off)
                    self.buckets.append(cur)
                cur.end = off + numel
                cur.names.append(n)
                self._param_bucket[n] = cur
        if self.overlap:
            for n, p in store.params.items():
                if n in self._param_bucket:
                    grad_sink.add_hook(p, self._make_hook(n))

    def _make_hook(self, name):
        def hook(_p):
            b = self._param_bucket[name]
            b.pending -= 1
            if b.pending == 0:
                self._launch(b)
        return hook

    def _launch(self, b):
        t = b.buf[b.start:b.end]
        if self.average:
            t.div_(self.world)
        b.work = dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)

    def prepare(self):
        """Call before backward: reset per-bucket pending counters."""
        for b in self.buckets:
            b.pending = len(b.names)
            b.work = None

    def finish(self):
        """After backward: launch buckets whose params got no gradient, then stream-wait all."""
        for b in self.buckets:
            if b.work is None:
                self._launch(b)
        for b in self.buckets:
            b.work.wait()
            b.work = None

    def bucket_sizes(self):
        return [(b.end - b.start) * b.buf.element_size() for b in self.buckets]
