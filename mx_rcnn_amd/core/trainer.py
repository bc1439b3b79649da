"""Training step engine.

One step = forward (mode-specific model entry) -> backward -> bucketed all-reduce (overlapped)
-> fused SGD on flat buffers -> device-side metric accumulation.  No host synchronisation,
so ``GraphedStep`` can capture the entire step into one hipGraph and replay it (static
shapes: the detection ops are designed for it).
"""
import os

import torch

from ..ops import grad_sink
from ..parallel.reducer import BucketReducer
from ..utils import profiler as prof
from .params import FlatParamStore


class Trainer:
    def __init__(self, model, mode='e2e', fixed_param_prefix=None, lr=0.001, momentum=0.9, wd=0.0005,
                 clip_gradient=1.0, rescale_grad=1.0, lr_scheduler=None, compute_dtype=None, device=None,
                 bucket_mb=25, average_grads=False, channels_last=None, grad_comm_dtype=None, precision=None):
        """precision (ops/precision.py):
        'fp32'   -- the reference's precision on the GPU: every MFMA operand and every tensor stored
                    between kernels is an EXACT (mid, hi, lo) bf16 triple of the fp32 value, products
                    as six bf16 MFMAs (hh + hm + mh + hl + lh + mm) with fp32 accumulation, fp32
                    gradients, BN statistics, SGD state and masters;
        'bf16x3' -- hi / lo pairs (16 significant bits), three products: faster, below fp32;
        'bf16'   -- bf16 operands, fp32 accumulation / masters;
        'torch'  -- plain fp32 PyTorch / vendor ops on the GPU (a reference arm for precision probes).
        Default: bf16 on the GPU unless compute_dtype says fp32 (then 'fp32'); the CPU path is plain
        fp32 whatever the name."""
        dev = torch.device(device) if device is not None else next(model.parameters()).device
        if precision is None:
            precision = 'fp32' if (compute_dtype == torch.float32 and dev.type == 'cuda') else 'bf16'
        if precision not in ('fp32', 'bf16x3', 'bf16', 'torch'):
            raise ValueError('precision must be fp32, bf16x3, bf16 or torch, not %r' % (precision,))
        # plane count of the multi-plane mode (0: off)
        self.x2 = {'fp32': 3, 'bf16x3': 2}.get(precision, 0) if dev.type == 'cuda' else 0
        if self.x2 or precision == 'torch':
            compute_dtype = torch.float32
        if compute_dtype is None:
            compute_dtype = torch.bfloat16 if dev.type == 'cuda' else torch.float32
        if channels_last is None:
            channels_last = dev.type == 'cuda'
        self.device, self.compute_dtype, self.channels_last = dev, compute_dtype, channels_last
        if self.x2:
            self.precision = precision
        else:
            self.precision = 'fp32' if compute_dtype == torch.float32 else 'bf16'
        self.model = model.to(dev)
        self.mode = mode
        self.store = FlatParamStore(self.model, fixed_param_prefix, compute_dtype, dev, channels_last,
                                   mode=mode if mode in ('rpn', 'rcnn') else None, x2=self.x2)
        # VGG16's fc6 / fc7 (120 M of 137 M weights): single process, their update runs inside their
        # weight gradient (below); under data parallelism the gradient must be summed first, so their
        # buckets take the update on the reducer's optimizer stream right after their all-reduce
        fc_names = ('fc6_weight', 'fc7_weight') if os.environ.get('MXR_FUSED_FC_SGD', '1') != '0' else ()
        self.reducer = BucketReducer(self.store, bucket_mb=bucket_mb, average=average_grads,
                                     comm_dtype=grad_comm_dtype, sgd_names=fc_names)
        if self.reducer.dp:
            self.store.broadcast_(0)  # identical starting weights on every rank
        self.momentum, self.wd, self.clip, self.rescale = momentum, wd, clip_gradient, rescale_grad
        self.base_lr = lr
        self.lr_scheduler = lr_scheduler
        if lr_scheduler is not None:
            lr_scheduler.base_lr = lr
        self.lr_t = torch.full((1,), float(lr), dtype=torch.float32, device=dev)
        # VGG16's FC weights take their update inside their weight-gradient kernel: the 120 M-element
        # gradient is never written, read or cleared (core/params.py enable_fused_sgd,
        # ops/vgg_fused.py); single process with the end-of-step optimizer only
        self.fused_fc_sgd = []
        if (dev.type == 'cuda' and not self.reducer.dp and not self.reducer.sgd_capable and
                os.environ.get('MXR_FUSED_FC_SGD', '1') != '0'):
            self.fused_fc_sgd = self.store.enable_fused_sgd(('fc6_weight', 'fc7_weight'), self.lr_t, momentum, wd,
                                                            rescale_grad, clip_gradient)
        self.num_update = 0
        # step counter of the counter-based dropout (ops/fc.py), advanced on the device at the end
        # of every step (inside the captured graph), so a replayed graph draws a fresh mask every
        # update with no host-side fill between replays
        self.rng_step = torch.zeros(1, dtype=torch.int64, device=dev)
        self._lr_set = float(lr)  # the value lr_t holds (filled again only when the schedule moves)
        from ..models.layers import Linear
        for m in self.model.modules():
            if isinstance(m, Linear):
                m.rng_step = self.rng_step
        self.nonfinite = torch.zeros((), dtype=torch.int32, device=dev)
        # fused gradient clear (SGD kernel zeroes what it read; MXR_FUSED_GRAD_CLEAR=0: a fill per
        # step); grads_dirty: a path left the flat gradients written (step API, monitored step,
        # an exception mid-step) -- the next step clears them first
        self.fused_clear = os.environ.get('MXR_FUSED_GRAD_CLEAR', '1') != '0'
        self.grads_dirty = False
        self.fault = torch.ones((), dtype=torch.float32, device=dev) if os.environ.get('MXR_FAULT_INJECT') else None
        # the loss-combine kernel bumps the counter (one launch for loss, objective and guard);
        # with fault injection the guard must see the poisoned objective, so the trainer keeps it
        self.model.nonfinite_counter = self.nonfinite if self.fault is None else None

    # ------------------------------------------------------------------
    def prepare_batch(self, batch):
        out = {}
        for k, v in batch.items():
            if k == 'pixel_means':  # raw-image batches: constants of the loader, kernel arguments
                out[k] = tuple(float(m) for m in (v.tolist() if torch.is_tensor(v) else v))
                continue
            if torch.is_tensor(v):
                v = v.to(self.device, non_blocking=True)
                if k == 'data' and v.dtype == torch.uint8:  # raw images: converted in forward (on device)
                    out[k] = v
                    continue
                if k == 'data':
                    v = v.to(self.compute_dtype)
                    if self.channels_last:
                        v = v.contiguous(memory_format=torch.channels_last)
            out[k] = v
        return out

    def forward(self, b):
        m = self.model
        if b['data'].dtype == torch.uint8:
            # raw uint8 BGR images (data/loader.py raw_images): RGB / means / pad on the device,
            # inside the captured step (ops/image.py)
            from ..ops.image import image_prep
            b = dict(b)
            b['data'] = image_prep(b['data'], b['im_info'], b.get('pixel_means'), self.compute_dtype,
                                   self.channels_last)
        if self.mode == 'e2e':
            return m.train_e2e(b['data'], b['im_info'], b['gt_boxes'], b['n_gt'])
        if self.mode == 'rpn':
            return m.train_rpn(b['data'], b['im_info'], b['gt_boxes'], b['n_gt'])
        if self.mode == 'rcnn':
            return m.train_rcnn(b['data'], b['rois'], b['label'], b['bbox_target'], b['bbox_inside_weight'],
                                b['bbox_outside_weight'])
        raise ValueError(self.mode)

    def step_body(self, b):
        """The device work of one step (capturable)."""
        from ..ops.precision import bump_generation, x2_mode
        bump_generation()  # the update below rewrites trainable weights in place
        with x2_mode(self.x2):
            return self._step_body(b)

    def _step_body(self, b):
        # the dgrad filter cache of the current weights, built beside the forward pass
        # (and the gradient clear), joined before the first backward kernel
        # gradient clear: the previous step's update kernels zeroed the buffers they consumed
        # (fused_clear), so only a step after a path that left them written clears them here
        dirty = self.grads_dirty or not self.fused_clear
        self.grads_dirty = True  # until this step's update has run
        zg_side = os.environ.get('MXR_ZERO_GRAD_SIDE', '1') != '0'
        cache_join = self.store.refresh_dgrad_cache_async(zero_grad=zg_side and dirty)
        if dirty and not zg_side:
            self.store.zero_grad()
        # the optimizer runs bucket by bucket under the backward pass (parallel/reducer.py)
        self.reducer.prepare(sgd=(self.lr_t, self.momentum, self.wd, self.rescale, self.clip),
                             clear=self.fused_clear)
        # a model that starts part of its backward inside forward (the e2e graph's early RPN
        # backward) joins the filter cache first
        self.model.pre_backward = cache_join
        # forward (the e2e graph's early RPN backward) and backward may apply fused FC updates
        with grad_sink.fused_sgd_scope(bool(self.fused_fc_sgd)):
            try:
                out = self.forward(b)
            finally:
                self.model.pre_backward = None
            if self.fault is not None:  # test hook: multiplies the loss by NaN on the armed step
                out['loss'] = out['loss'] * self.fault
                out['objective'] = out['objective'] * self.fault
            # device-side non-finite guard: no host sync, read every `frequent` steps;
            # counted by the model's loss-combine kernel unless fault injection is armed
            if self.model.nonfinite_counter is None:
                self.nonfinite.add_((~torch.isfinite(out['objective'])).to(torch.int32))
            cache_join()
            with prof.range('backward+allreduce'):
                from ..ops.fused import defer_reduces
                # no gradient hook reads the flat buffers mid-backward: split-K reduces may cross units
                with defer_reduces(not (self.reducer.overlap or self.reducer.sgd_capable)):
                    from ..ops._ext import unit_grad
                    out['loss'].backward(unit_grad(out['loss'].device))
        with prof.range('allreduce_wait'):
            self.reducer.finish()
        with prof.range('sgd'):
            if not self.reducer.sgd_applied:
                self.store.sgd_step(self.lr_t, self.momentum, self.wd, self.rescale, self.clip,
                                    grad_for=self.reducer.grad_for, refresh=False, clear=self.fused_clear)
        self.grads_dirty = not self.fused_clear
        self.advance_rng()
        # Return detached outputs: a caller holding the loss would otherwise keep this step's
        # autograd graph (and its AccumulateGrad nodes, bound to this step's stream) alive, and a
        # later hipGraph capture on a side stream then syncs against that stream and dies in
        # hipStreamEndCapture.
        return {k: (v.detach() if torch.is_tensor(v) else v) for k, v in out.items()}

    def check_finite(self, step=None):
        """Raise FloatingPointError if any step since the last check produced a non-finite loss --
        one host read of a device counter.  (A proposal NMS chain that gives up a poll is finished
        by the serial fallback and only counted in ``model.nms_gave_up``.)"""
        n = int(self.nonfinite.item())
        if n:
            self.nonfinite.zero_()
            raise FloatingPointError('non-finite loss in %d step(s) up to step %s'
                                     % (n, step))

    def arm_fault(self, kind='nan'):
        """Fault injection (``MXR_FAULT_INJECT=nan@STEP``): poison the next step's loss."""
        if self.fault is not None:
            self.fault.fill_(float('nan') if kind == 'nan' else float('inf'))

    def disarm_fault(self):
        if self.fault is not None:
            self.fault.fill_(1.0)

    # ------------------------------------------------------------------ state snapshot
    @torch.no_grad()
    def snapshot_state(self):
        """Copies of everything a step mutates: fp32 masters, momentum, low-precision shadows,
        model buffers (train-mode BN moving statistics), the non-finite counter and the RNG
        streams.  Used to make hipGraph warm-up runs side-effect free."""
        st = {'groups': [(g.master.clone(), g.mom.clone(), None if g.shadow is None else g.shadow.clone())
                         for g in self.store.groups],
              'buffers': [b.detach().clone() for b in self.model.buffers()],
              'nonfinite': self.nonfinite.clone(), 'rng_step': self.rng_step.clone(),
              'rng_cpu': torch.get_rng_state()}
        if self.device.type == 'cuda':
            st['rng_cuda'] = torch.cuda.get_rng_state(self.device)
        return st

    @torch.no_grad()
    def restore_state(self, st, rng=True):
        for g, (m, mo, sh) in zip(self.store.groups, st['groups']):
            g.master.copy_(m)
            g.mom.copy_(mo)
            if sh is not None:
                g.shadow.copy_(sh)
        for b, v in zip(self.model.buffers(), st['buffers']):
            b.copy_(v)
        self.nonfinite.copy_(st['nonfinite'])
        from ..ops.precision import bump_generation
        bump_generation()  # the masters were rewritten
        if 'rng_step' in st:
            self.rng_step.copy_(st['rng_step'])
        self.store.refresh_dgrad_cache()
        if rng:
            torch.set_rng_state(st['rng_cpu'])
            if 'rng_cuda' in st:
                torch.cuda.set_rng_state(st['rng_cuda'], self.device)

    def update_lr(self):
        self.num_update += 1
        if self.lr_scheduler is not None:
            lr = float(self.lr_scheduler(self.num_update))
            if lr != self._lr_set:  # a device fill only when the schedule moves
                self.lr_t.fill_(lr)
                self._lr_set = lr

    def advance_rng(self):
        """End of a step: the dropout counter moves on (on the device; captured with the step)."""
        if self.rng_step.is_cuda:
            from ..ops._ext import need_ext
            need_ext().counter_add_(self.rng_step, 1)
        else:
            self.rng_step.add_(1)

    def step(self, batch):
        self.model.train()
        b = self.prepare_batch(batch)
        self.update_lr()
        return self.step_body(b)


class GraphedStep:
    """Capture ``trainer.step_body`` for fixed input shapes into a hipGraph and replay it.

    Static input buffers are filled with copies of each new batch (D2D), the LR lives in a
    device tensor, RNG draws use PyTorch's graph-safe Philox offsets.  Falls back to eager
    if capture fails (reported, not silent).

    The warm-up runs (which allocate the kernels' workspaces and settle the allocator before
    capture) execute real steps on the example batch; every piece of state they touch --
    weights, momentum, shadows, BN moving statistics, the non-finite counter, the RNG -- is
    snapshotted first and restored before capture, so capturing a new shape never applies
    unscheduled updates (graphed and eager training give the same weights).
    """

    def __init__(self, trainer, example_batch, warmup=3):
        self.t = trainer
        trainer.model.train()
        self.static = trainer.prepare_batch(example_batch)
        self.static = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in self.static.items()}
        saved = trainer.snapshot_state() if warmup else None
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        try:
            with torch.cuda.stream(s):
                for _ in range(warmup):
                    trainer.step_body(self.static)
        finally:
            # a warm-up step that raised must not leave its updates behind (an eager fallback
            # would start from weights no schedule produced)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            if saved is not None:
                trainer.restore_state(saved)
                del saved
                torch.cuda.synchronize()
        # the conv autotune ran in the warm-up: under DP every rank captures rank 0's plan (the
        # K-split choices change summation order), and rank 0 persists it for the next run
        from ..ops import tune_plan
        self.plan_hash = tune_plan.sync_from_rank0(torch.device('cuda', torch.cuda.current_device()))
        if not (torch.distributed.is_available() and torch.distributed.is_initialized()) or \
                torch.distributed.get_rank() == 0:
            tune_plan.save()
        self.graph = torch.cuda.CUDAGraph()
        # thread_local: the loaders' prefetch threads keep staging the next batches (pinned host
        # buffers, H2D copies on their own streams) while a new shape is captured; in the default
        # global mode any such call from another thread invalidates the capture
        with torch.cuda.graph(self.graph, capture_error_mode='thread_local'):
            self.out = trainer.step_body(self.static)
        torch.cuda.synchronize()

    def __call__(self, batch=None):
        if batch is not None:
            for k, v in batch.items():
                if torch.is_tensor(v) and torch.is_tensor(self.static.get(k)):
                    self.static[k].copy_(v, non_blocking=True)
        self.t.update_lr()
        if self.t.grads_dirty:  # the graph holds no gradient clear (captured after a fused-clear step)
            self.t.store.zero_grad()
        from ..ops.precision import bump_generation
        bump_generation()  # the replayed update rewrites trainable weights in place
        self.graph.replay()
        self.t.grads_dirty = not self.t.fused_clear
        return self.out
