"""Bucketed gradient all-reduce overlapped with backward.

Gradients live in flat per-group buffers (core/params.py) ordered by gradient readiness.
Each buffer is cut into buckets of ~``bucket_mb``; a post-accumulate-grad hook counts the
parameters of each bucket and, when the last one lands, issues an async ``all_reduce(SUM)``
on that slice.  RCCL runs it on its own stream (ordered after the compute stream's prior
work), so the reduction of the head / stage-4 / fc6 gradients overlaps the rest of the
backward pass.  ``finish()`` makes the compute stream wait on every outstanding bucket
before the optimizer touches the buffers -- no host blocking.

Semantics: SUM across ranks (MXNet kvstore 'device', rescale_grad=1: `train_end2end.py:104`);
``average=True`` switches to mean.

Precision: the kvstore sums fp32 gradients.  With bf16 compute the per-rank flat gradient
buffers are bf16 (the MFMA wgrad kernels round once when they store), so by default
(``comm_dtype=float32``) each ready bucket is widened into an fp32 communication buffer (one
cast kernel on the compute stream), the ring sums fp32, and the optimizer reads the fp32 sum
(:meth:`BucketReducer.grad_for`) -- no per-hop bf16 rounding, at twice the bytes on the wire.
``comm_dtype=bfloat16`` keeps the half-size wire format (opt-in, measured by bench.py).

Bucket sizing: xGMI is point-to-point, a ring uses one link per hop, so messages must stay
large enough to run at link bandwidth (a 25 MB ring all-reduce over 8 GPUs is bandwidth-, not
latency-bound), but small enough that the first buckets are reduced while most of the backward
is still running.  Sizes are in bytes of the WIRE dtype: 25 MB cuts ResNet-101's ~180 MB of
fp32 gradient traffic into 8 buckets, the last (capped at ``tail_mb``) is the only exposed one.
"""
import os

import torch
import torch.distributed as dist

from ..ops import grad_sink
from .dist import get_world_size, is_distributed


class _nullctx(object):
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class _Bucket:
    __slots__ = ('group', 'buf', 'comm', 'start', 'end', 'names', 'pending', 'work', 'updated', 'early')

    def __init__(self, group, start, end, comm=None):
        self.group, self.buf, self.start, self.end = group, group.grad, start, end
        self.comm = comm  # fp32 flat buffer of the group (wire format), or None (reduce in place)
        self.names = []
        self.pending = 0
        self.work = None
        self.updated = False
        self.early = False  # gets its SGD right after its all-reduce (BucketReducer sgd_names)


class BucketReducer:
    """Gradient buckets with readiness hooks.  Two jobs, either or both:

    * data parallel: all-reduce each bucket as soon as its last gradient lands;
    * overlapped optimizer (``prepare(sgd=...)``, GPU): run the fused SGD of each bucket on an
      optimizer stream as soon as the bucket is final (after its all-reduce under DP), so the
      update of the head / stage-4 / RPN weights runs under the rest of the backward pass instead
      of after it.  SGD is elementwise per parameter (MXNet clips each element, no global norm),
      and a parameter's value is not read again once its gradient is final (each weight belongs
      to one layer; its dgrad and wgrad are both done when the readiness hook fires), so
      updating it early is exact.  Single-GPU buckets are ``sgd_bucket_mb`` (smaller: only the
      last one is exposed after the backward);
    * under data parallelism, ``sgd_names``: only the buckets holding those parameters take their
      update on the optimizer stream right after their all-reduce (VGG16's fc6 / fc7: 120 M of its
      137 M weights, whose HBM-bound update would otherwise be the end-of-step tail -- the
      single-process step fuses it into the weight gradient instead, which DP cannot: the gradient
      must be summed first); the end-of-step SGD covers the rest (``store.mark_updated``).
    """

    def __init__(self, store, bucket_mb=25, average=False, overlap=True, sgd_bucket_mb=8, tail_mb=4,
                 comm_dtype=None, sgd_names=None):
        self.store = store
        self.world = get_world_size()
        self.average = average
        self.dp = is_distributed() and (self.world > 1 or os.environ.get('MXR_FORCE_DIST', '0') == '1')
        if comm_dtype is None:
            comm_dtype = {'bf16': torch.bfloat16, 'fp32': torch.float32}[os.environ.get('MXR_GRAD_COMM', 'fp32')]
        self.comm_dtype = comm_dtype
        self._comm = {}  # id(group) -> fp32 wire buffer (DP with low-precision gradient buffers)
        self.overlap = overlap and self.dp
        # off by default: measured 2-3 % slower on 1-GPU ResNet-101 (scripts/gpu_sgd.sh A/B, 125-126
        # vs 128-129 img/s): the HBM-bound update steals bandwidth from the concurrent backward
        # convs for less than it hides (the whole update is ~0.16 ms)
        # (multi-plane stores: a bucket's planes are slices one group plane apart -- plane_stride)
        self.sgd_capable = store.device.type == 'cuda' and os.environ.get('MXR_OVERLAP_SGD', '0') == '1'
        self.buckets = []
        self._param_bucket = {}
        self._sgd = None
        self._clear = False
        self._widen_stream = None
        self._opt_stream = None
        self._early_sgd = None
        self.sgd_applied = False
        self.early_names = []
        if not (self.dp or self.sgd_capable):
            return
        mb = bucket_mb if self.dp else sgd_bucket_mb
        tail = min(tail_mb, mb) if tail_mb else mb
        for g in store.groups:
            comm = None
            if self.dp and g.grad.dtype != torch.float32 and self.comm_dtype == torch.float32:
                comm = torch.zeros(g.numel, dtype=torch.float32, device=g.grad.device)
                self._comm[id(g)] = comm
            esize = comm.element_size() if comm is not None else g.grad.element_size()
            cap = max(1, int(mb * (1 << 20) // esize))
            tail_cap = max(1, int(tail * (1 << 20) // esize))
            # cut from the LAST-ready end: the bucket that completes when the backward pass ends
            # is the only one whose collective is fully exposed, so it is capped at ``tail_mb``;
            # the rest get ``bucket_mb`` (entries are in readiness order)
            rev = []  # [start, end, names] from the last-ready end
            for (n, _, _, numel, _, _), off in reversed(list(zip(g.entries, g.offsets))):
                cur = rev[-1] if rev else None
                limit = tail_cap if len(rev) == 1 else cap
                if cur is None or (cur[1] - off > limit and cur[1] > cur[0]):
                    cur = [off, off + numel, []]
                    rev.append(cur)
                cur[0] = off
                cur[2].append(n)
            for start, end, names in reversed(rev):
                bkt = _Bucket(g, start, start, comm)
                bkt.end = end
                bkt.names = list(reversed(names))
                self.buckets.append(bkt)
                for n in names:
                    self._param_bucket[n] = bkt
        if self.dp and sgd_names and not self.sgd_capable:
            for b in self.buckets:
                b.early = any(n in sgd_names for n in b.names)
        self.early_names = sorted(n for b in self.buckets if b.early for n in b.names)
        if self.overlap or self.sgd_capable:
            grad_sink.clear_hooks(store.params.values())  # an earlier reducer on these parameters
            for n, p in store.params.items():
                if n in self._param_bucket:
                    grad_sink.add_hook(p, self._make_hook(n))

    def _make_hook(self, name):
        def hook(_p):
            b = self._param_bucket[name]
            b.pending -= 1
            if b.pending == 0:
                if self.overlap:
                    self._launch(b)
                if self._sgd is not None or (b.early and self._early_sgd is not None):
                    self._update(b)
        return hook

    def grad_for(self, group):
        """The buffer holding ``group``'s reduced gradient after :meth:`finish` (the fp32 wire
        buffer under DP with fp32 communication, else the group's own gradient buffer)."""
        return self._comm.get(id(group), group.grad)

    def _launch(self, b):
        t = b.buf[b.start:b.end]
        if b.comm is not None and t.is_cuda and os.environ.get('MXR_WIDEN_SIDE', '1') != '0':
            # widen on a side stream (ordered after the producers of t, which the compute stream has
            # issued), and issue the collective from it: RCCL's stream waits for the widening, the
            # compute stream goes on with the backward instead of running ~50 us of casts per step
            cur = torch.cuda.current_stream(t.device)
            if self._widen_stream is None:
                self._widen_stream = torch.cuda.Stream(device=t.device)
            ws = self._widen_stream
            ws.wait_stream(cur)
            with torch.cuda.stream(ws):
                w = b.comm[b.start:b.end]
                w.copy_(t)
                if self.average:
                    w.div_(self.world)
                b.work = dist.all_reduce(w, op=dist.ReduceOp.SUM, async_op=True)
            return
        if b.comm is not None:
            w = b.comm[b.start:b.end]
            w.copy_(t)  # widen on the compute stream, ordered after the producers of t
            t = w
        if self.average:
            t.div_(self.world)
        b.work = dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)

    def _update(self, b):
        """SGD of one final bucket on the optimizer stream (after its all-reduce under DP; the CPU
        runs it in order)."""
        from ..ops.sgd import sgd_momentum_
        cuda = b.buf.is_cuda
        if cuda and self._opt_stream is None:
            self._opt_stream = torch.cuda.Stream(device=b.buf.device)
        os_ = self._opt_stream
        if cuda:
            os_.wait_stream(torch.cuda.current_stream(b.buf.device))
        g, s, e = b.group, b.start, b.end
        lr, mu, wd, rescale, clip = self._sgd if self._sgd is not None else self._early_sgd
        with (torch.cuda.stream(os_) if cuda else _nullctx()):
            if b.work is not None:
                b.work.wait()  # the optimizer stream waits for this bucket's collective
            if g.shadow is not None and g.x2:  # planes g.plane apart: the view from s reaches all of them
                sh, planes, stride = g.shadow[s:], g.x2, g.plane
            else:
                sh, planes, stride = (None if g.shadow is None else g.shadow[s:e]), 1, 0
            sgd_momentum_(g.master[s:e], g.mom[s:e], self.grad_for(g)[s:e], lr, mu, wd if g.decay else 0.0, rescale,
                          clip, sh, planes=planes, zero=g.grad[s:e] if self._clear else None, plane_stride=stride)
        b.updated = True
        if self._sgd is None:  # early (sgd_names) bucket: the end-of-step SGD skips it
            self.store.mark_updated(g, s, e)

    def prepare(self, sgd=None, clear=False):
        """Call before backward: reset per-bucket counters.  ``sgd=(lr_tensor, momentum, wd,
        rescale, clip)`` enables the overlapped optimizer for this step (GPU only); ``clear``: its
        update kernels zero the gradient buffers they consumed."""
        self._sgd = sgd if (sgd is not None and self.sgd_capable and self.buckets) else None
        self._early_sgd = sgd if (sgd is not None and self._sgd is None and self.early_names) else None
        self.store._early = {}  # ranges a step that raised mid-backward marked are void
        self._clear = bool(clear)
        self.sgd_applied = False
        for b in self.buckets:
            b.pending = len(b.names)
            b.work = None
            b.updated = False

    def finish(self):
        """After backward: launch / update buckets whose params got no gradient, then make the
        compute stream wait for every collective and the optimizer stream.  ``sgd_applied`` tells
        the caller whether the update already happened."""
        if self.dp:
            for b in self.buckets:
                if b.work is None:
                    self._launch(b)
        if self._sgd is not None:
            for b in self.buckets:
                if not b.updated:
                    self._update(b)
            self.sgd_applied = True
        elif self._early_sgd is not None:
            for b in self.buckets:
                if b.early and not b.updated:
                    self._update(b)
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                b.work = None
        if self._opt_stream is not None and (self._sgd is not None or self._early_sgd is not None):
            torch.cuda.current_stream(self._opt_stream.device).wait_stream(self._opt_stream)
        self._sgd = None
        self._early_sgd = None

    def bucket_sizes(self):
        """Bytes each bucket puts on the wire."""
        return [(b.end - b.start) * (b.comm if b.comm is not None else b.buf).element_size() for b in self.buckets]

    def measure_collectives(self, iters=10, warmup=2):
        """Time every bucket's all-reduce in isolation (same buffers, dtype and order as the
        step, outside any graph): -> {'bucket_bytes': [...], 'bucket_ms': [...], 'total_ms',
        'busbw_GBps'}.  ``total_ms`` is the per-step collective time if nothing overlapped;
        bus bandwidth uses the ring formula 2(n-1)/n * bytes / time.  Collective call; every
        rank must call it.  Clobbers the gradient / wire buffers (call between steps)."""
        if not self.dp or not self.buckets:
            return None
        import time
        cuda = self.store.device.type == 'cuda'
        tensors = [(b.comm if b.comm is not None else b.buf)[b.start:b.end] for b in self.buckets]
        out_ms = []
        for t in tensors:
            for _ in range(warmup):
                dist.all_reduce(t)
            if cuda:
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                ev0.record()
                for _ in range(iters):
                    dist.all_reduce(t)
                ev1.record()
                ev1.synchronize()
                ms = ev0.elapsed_time(ev1) / iters
            else:
                t0 = time.perf_counter()
                for _ in range(iters):
                    dist.all_reduce(t)
                ms = (time.perf_counter() - t0) * 1e3 / iters
            out_ms.append(ms)
        # the slowest rank defines the collective time
        agg = torch.tensor(out_ms, dtype=torch.float64, device=self.store.device)
        dist.all_reduce(agg, op=dist.ReduceOp.MAX)
        out_ms = [float(v) for v in agg.tolist()]
        nbytes = self.bucket_sizes()
        total = sum(out_ms)
        n = self.world
        busbw = (2.0 * (n - 1) / n * sum(nbytes) / (total * 1e-3) / 1e9) if total > 0 and n > 1 else 0.0
        return {'bucket_bytes': nbytes, 'bucket_ms': [round(v, 4) for v in out_ms], 'total_ms': round(total, 4),
                'busbw_GBps': round(busbw, 2), 'wire_dtype': str((tensors[0].dtype)).replace('torch.', '')}
