"""MutableModule: the reference's training driver API (`rcnn/module.py:13-199` plus the
inherited MXNet ``BaseModule.fit``) on top of :class:`Trainer`.

* ``symbol`` is a :class:`~mx_rcnn_amd.models.FasterRCNN` (or ``(model, mode)``); the mode
  (``'e2e'``, ``'rpn'``, ``'rcnn'``) selects the training graph like the reference's symbol
  builders do.
* Shape changes: the reference rebinds a new executor sharing memory when the input shape
  changes (`rcnn/module.py:155-175`).  Here every distinct input shape gets its own captured
  hipGraph (``use_graph=True``), cached by shape -- the same idea, replayed without any
  per-step launch overhead.
* ``fixed_param_prefix`` freezes parameters by SUBSTRING match, exactly like the reference
  (with a warning when a prefix also matches inside other names).
* Data parallel: one process per GPU (torch.distributed, RCCL); gradients are SUM-reduced
  in overlapped buckets; BN moving statistics are averaged across ranks only when params are
  fetched (checkpointing), mirroring MXNet's ``get_params``; rank 0 runs epoch-end callbacks.
"""
import logging
import os
import time
import zlib

import numpy as np
import torch

from ..parallel import dist as pdist
from ..parallel import watchdog
from .callback import BatchEndParam
from .lr_scheduler import FactorScheduler
from .trainer import GraphedStep, Trainer
from ..utils import profiler as prof


def sync_key(key):
    """The part of a step's input-shape key that every rank shares: the shapes without their
    leading (batch / RoI-count) dimension.  With an uneven ``work_load_list`` each rank's slice of
    the global batch has its own, fixed size (data/loader.py split_input_slice), so the ranks'
    full keys differ while their capture points -- a new padded image shape of the global step --
    still coincide."""
    return tuple((k, tuple(s[1:])) for k, s in key)


class MutableModule(object):
    def __init__(self, symbol, data_names=None, label_names=None, logger=logging, context=None, work_load_list=None,
                 max_data_shapes=None, max_label_shapes=None, fixed_param_prefix=None, mode=None, use_graph=None,
                 compute_dtype=None, precision=None):
        """precision: 'fp32' (default on the GPU: the reference's precision, exact fp32 triples on
        the bf16 MFMA, ops/precision.py), 'bf16x3' or 'bf16' (core/trainer.py); compute_dtype is the
        older spelling (bf16 -> 'bf16', fp32 -> 'fp32')."""
        if isinstance(symbol, tuple):
            symbol, mode = symbol
        self.symbol = symbol
        self.model = symbol
        self.mode = mode or getattr(symbol, 'train_mode', 'e2e')
        self._data_names = list(data_names or [])
        self._label_names = list(label_names or [])
        self.logger = logger
        ctx = context if context is not None else ('cuda' if torch.cuda.is_available() else 'cpu')
        if isinstance(ctx, (list, tuple)):
            ctx = ctx[0]
        self.context = torch.device(ctx) if not isinstance(ctx, torch.device) else ctx
        self.work_load_list = work_load_list
        self.max_data_shapes, self.max_label_shapes = max_data_shapes, max_label_shapes
        self.fixed_param_prefix = fixed_param_prefix or []
        self.use_graph = (self.context.type == 'cuda') and (use_graph is None or bool(use_graph))
        self.compute_dtype = compute_dtype
        if precision is None:
            from ..ops.precision import default_name
            precision = 'bf16' if compute_dtype == torch.bfloat16 else ('fp32' if compute_dtype == torch.float32
                                                                        else default_name())
        self.precision = precision
        self.binded = self.params_initialized = self.optimizer_initialized = False
        self.trainer = None
        self._graphs = {}
        self._outputs = None
        self._batch = None
        self._monitor = None
        self._hb = None  # heartbeat of the running fit(), paused across captures

    # ------------------------------------------------------------------ properties
    @property
    def data_names(self):
        return self._data_names

    @property
    def output_names(self):
        return ['loss', 'rpn_cls_loss', 'rpn_bbox_loss', 'cls_loss', 'bbox_loss', 'cls_prob', 'label']

    @property
    def data_shapes(self):
        return self.max_data_shapes

    @property
    def label_shapes(self):
        return self.max_label_shapes

    @property
    def output_shapes(self):
        if self._outputs is None:
            return []
        return [(k, tuple(v.shape)) for k, v in self._outputs.items() if torch.is_tensor(v)]

    # ------------------------------------------------------------------ setup
    def bind(self, data_shapes=None, label_shapes=None, for_training=True, inputs_need_grad=False,
             force_rebind=False, shared_module=None, grad_req='write'):
        if data_shapes is not None:
            self.max_data_shapes = data_shapes
        if label_shapes is not None:
            self.max_label_shapes = label_shapes
        self.for_training = for_training
        self.model.to(self.context)
        self.binded = True

    def init_params(self, initializer=None, arg_params=None, aux_params=None, allow_missing=True, force_init=False):
        """Load MXNet-named arrays into the model (missing names keep their initialisation)."""
        if self.params_initialized and not force_init:
            return
        if self.trainer is not None:
            arrays = dict(arg_params or {})
            self.trainer.store.load_arrays(arrays)
            self._load_aux(aux_params)
        else:
            self._load_model_arrays(arg_params, aux_params, allow_missing)
        self.params_initialized = True

    def _load_model_arrays(self, arg_params, aux_params, allow_missing=True):
        cur = self._model_args()
        missing = []
        with torch.no_grad():
            for k, t in cur.items():
                if arg_params and k in arg_params:
                    src = torch.as_tensor(np.asarray(arg_params[k]) if not torch.is_tensor(arg_params[k])
                                          else arg_params[k]).float()
                    t.copy_(src.reshape(t.shape).to(t.device, t.dtype))
                else:
                    missing.append(k)
        if missing and not allow_missing:
            raise KeyError('missing arg params: %s' % missing[:10])
        self._load_aux(aux_params)

    def _load_aux(self, aux_params):
        if not aux_params:
            return
        cur = self._model_aux()
        with torch.no_grad():
            for k, t in cur.items():
                if k in aux_params:
                    src = aux_params[k]
                    src = src if torch.is_tensor(src) else torch.as_tensor(np.asarray(src))
                    t.copy_(src.reshape(t.shape).to(t.device, t.dtype))

    def _graph_mode(self):
        return self.mode if self.mode in ('rpn', 'rcnn') else None

    def _model_args(self):
        try:
            return self.model.arg_params(self._graph_mode())
        except TypeError:
            return self.model.arg_params()

    def _model_arg_shapes(self):
        fn = getattr(self.model, 'arg_shapes', None)
        if fn is None:
            return {}
        try:
            return fn(self._graph_mode())
        except TypeError:
            return fn()

    def _model_aux(self):
        try:
            return self.model.aux_params(self._graph_mode())
        except TypeError:
            return self.model.aux_params()

    def init_optimizer(self, kvstore='device', optimizer='sgd', optimizer_params=None, force_init=False):
        if self.optimizer_initialized and not force_init:
            return
        assert optimizer == 'sgd', 'only SGD (the reference optimizer) is implemented'
        p = dict(optimizer_params or {})
        lr = p.get('learning_rate', 0.01)
        sched = p.get('lr_scheduler')
        self.trainer = Trainer(self.model, self.mode, fixed_param_prefix=self.fixed_param_prefix, lr=lr,
                               momentum=p.get('momentum', 0.0), wd=p.get('wd', 0.0),
                               clip_gradient=p.get('clip_gradient', -1.0) or -1.0,
                               rescale_grad=p.get('rescale_grad', 1.0), lr_scheduler=sched,
                               compute_dtype=self.compute_dtype, device=self.context,
                               bucket_mb=p.get('bucket_mb', 64),
                               precision=self.precision if self.context.type == 'cuda' else None)
        if self._monitor is not None:  # a norm monitor reads the gradients: no fused updates
            self.trainer.fused_fc_sgd = []
        self.optimizer_initialized = True

    def install_monitor(self, mon):
        self._monitor = mon
        mon.install(self.model)
        # the monitor reads gradients: no update may be fused into a weight-gradient kernel
        if self.trainer is not None:
            self.trainer.fused_fc_sgd = []

    # ------------------------------------------------------------------ step API
    def forward(self, data_batch, is_train=None):
        is_train = self.for_training if is_train is None else is_train
        b = self.trainer.prepare_batch(data_batch)
        self._batch = b
        self.model.train(is_train)
        from ..ops.precision import x2_mode
        # the step API runs in the trainer's precision mode, like step() / graph replay (the
        # multi-plane autograd functions read the mode at backward time too)
        with x2_mode(self.trainer.x2):
            if is_train:
                # step() leaves the strided convs' dgrad filter cache for the next step_body to rebuild
                # (sgd_step(refresh=False)); a backward through this API must see the updated filters
                self.trainer.store.refresh_dgrad_cache()
                self.trainer.store.zero_grad()
                self.trainer.grads_dirty = True  # update() leaves them written (the monitor reads them)
                self.trainer.reducer.prepare()
                self._outputs = self.trainer.forward(b)
            else:
                with torch.no_grad():
                    self._outputs = self.trainer.forward(b)

    def backward(self, out_grads=None):
        from ..ops.precision import x2_mode
        with x2_mode(self.trainer.x2):
            self._outputs['loss'].backward()
        # release the autograd graph (see Trainer.step_body: a live graph breaks later captures)
        self._outputs = {k: (v.detach() if torch.is_tensor(v) else v) for k, v in self._outputs.items()}

    def update(self):
        t = self.trainer
        t.reducer.finish()
        t.update_lr()
        t.store.sgd_step(t.lr_t, t.momentum, t.wd, t.rescale, t.clip, grad_for=t.reducer.grad_for)
        t.advance_rng()

    def step(self, data_batch):
        """forward + backward + update fused (graph-replayed per input shape when enabled).
        Steps watched by a norm monitor or the stage profiler run eagerly (hooks and timing
        events do not exist inside a replayed graph)."""
        eager = (not self.use_graph or prof.enabled() or
                 (self._monitor is not None and self._monitor.activated))
        if eager:
            t = self.trainer
            watched = self._monitor is not None and self._monitor.activated
            fused = t.fused_clear
            t.fused_clear = fused and not watched  # a norm monitor reads the gradients after the update
            try:
                self._outputs = t.step(data_batch)
            finally:
                t.fused_clear = fused
                if watched:
                    t.grads_dirty = True
            return self._outputs
        key = tuple((k, tuple(v.shape)) for k, v in sorted(data_batch.items()) if torch.is_tensor(v))
        g = self._graphs.get(key)
        if g is None:
            g = self._capture(key, data_batch)
        if g == 'eager':
            self._outputs = self.trainer.step(data_batch)
        else:
            self._outputs = g(data_batch)
        return self._outputs

    def _capture(self, key, data_batch):  # noqa: C901
        """Capture a hipGraph for a new input shape.  Under data parallelism every rank reaches
        this on the same step (the loaders pad every rank's batch to the global step's shape,
        data/loader.py), and the ranks agree on the outcome: if capture failed anywhere, all
        ranks run this shape eagerly (the captured step contains collectives, so a mixed
        graphed/eager step would mismatch them)."""
        ok, g = 1.0, None
        if self._hb is not None:
            self._hb.pause()
        try:
            g = GraphedStep(self.trainer, data_batch)
        except Exception as e:  # reported, never silent
            if pdist.is_distributed() and pdist.get_world_size() > 1:
                # the failed warm-up may have issued fewer bucket all-reduces than the peers' did:
                # negotiating an eager fallback would pair mismatched collectives -> job error
                raise RuntimeError('hipGraph capture failed on rank %d under data parallelism (%s: %s)'
                                   % (pdist.get_rank(), type(e).__name__, str(e)[:300]))
            ok = 0.0
            logging.warning('hipGraph capture failed for %s (%s: %s)', key, type(e).__name__, str(e)[:300])
            torch.cuda.synchronize()
        finally:
            if self._hb is not None:
                self._hb.resume()
        if pdist.is_distributed():
            if pdist.get_world_size() > 1:
                h = torch.tensor([float(zlib.crc32(repr(sync_key(key)).encode()))], dtype=torch.float64,
                                 device=self.context)
                lo, hi = h.clone(), h.clone()
                torch.distributed.all_reduce(lo, op=torch.distributed.ReduceOp.MIN)
                torch.distributed.all_reduce(hi, op=torch.distributed.ReduceOp.MAX)
                if float(lo.item()) != float(hi.item()):
                    raise RuntimeError('ranks reached different input shapes at a capture point (%s); the data '
                                       'loaders must pad every rank to the global step shape' % (key,))
            ok = -pdist.all_reduce_max(-ok, self.context)
        if ok < 1.0:
            g = 'eager'
            logging.warning('running input shape %s eagerly on every rank', key)
        else:
            logging.info('captured hipGraph for input shape %s (%d cached)', key, len(self._graphs) + 1)
        self._graphs[key] = g
        return g

    def get_outputs(self, merge_multi_context=True):
        return self._outputs

    def update_metric(self, eval_metric, labels=None):
        eval_metric.update(labels, self._outputs)

    def get_params(self):
        """-> (arg_params, aux_params) as fp32 numpy, BN moving stats averaged over ranks."""
        if self.trainer is not None:
            arg = {k: v.detach().float().cpu().numpy() for k, v in self.trainer.store.state_arrays().items()}
        else:
            arg = {k: v.detach().float().cpu().numpy() for k, v in self._model_args().items()}
        shapes = self._model_arg_shapes()
        arg = {k: (v.reshape(shapes[k]) if k in shapes else v) for k, v in arg.items()}  # checkpoint layout
        aux = {}
        for k, v in self._model_aux().items():
            t = v.detach().float().clone()
            if pdist.is_distributed():
                torch.distributed.all_reduce(t)
                t /= pdist.get_world_size()
            aux[k] = t.cpu().numpy()
        return arg, aux

    def save_optimizer_states(self, fname):
        """Momentum + update count (MXNet ``Module.save_optimizer_states``), MXNet .params codec."""
        from ..utils import ndarray_io
        st = {'mom:' + k: v.detach().cpu().numpy() for k, v in self.trainer.store.optimizer_state().items()}
        st['num_update'] = np.array([self.trainer.num_update], np.float32)
        st['rng_step'] = self.trainer.rng_step.detach().cpu().numpy().astype(np.float64)  # dropout counter
        st['rng_cpu'] = torch.get_rng_state().numpy()
        if self.context.type == 'cuda':
            st['rng_cuda'] = torch.cuda.get_rng_state(self.context).numpy()
        ndarray_io.save(fname, st)

    def load_optimizer_states(self, fname):
        from ..utils import ndarray_io
        st = ndarray_io.load(fname)
        moms = {k[4:]: v for k, v in st.items() if k.startswith('mom:')}
        missing = self.trainer.store.load_optimizer_state(moms)
        if 'num_update' in st:
            self.trainer.num_update = int(np.asarray(st['num_update']).reshape(-1)[0])
            self.trainer.num_update -= 1
            self.trainer.update_lr()  # lr tensor matches the schedule position
        if 'rng_step' in st:
            self.trainer.rng_step.fill_(int(np.asarray(st['rng_step']).reshape(-1)[0]))
        elif 'num_update' in st:
            # a states file from before the dropout counter was saved: the counter advanced once
            # per update, so re-derive it instead of replaying the first steps' dropout masks
            self.trainer.rng_step.fill_(int(np.asarray(st['num_update']).reshape(-1)[0]))
        if 'rng_cpu' in st:
            torch.set_rng_state(torch.from_numpy(np.ascontiguousarray(st['rng_cpu'], dtype=np.uint8)))
        if 'rng_cuda' in st and self.context.type == 'cuda':
            torch.cuda.set_rng_state(torch.from_numpy(np.ascontiguousarray(st['rng_cuda'], dtype=np.uint8)),
                                     self.context)
        if missing:
            logging.warning('optimizer state missing for %d params (e.g. %s)', len(missing), missing[0])

    def set_params(self, arg_params, aux_params, allow_missing=False, force_init=True):
        self.init_params(None, arg_params, aux_params, allow_missing=allow_missing, force_init=force_init)

    # ------------------------------------------------------------------ fit
    def fit(self, train_data, eval_data=None, eval_metric=None, epoch_end_callback=None, batch_end_callback=None,
            kvstore='device', optimizer='sgd', optimizer_params=None, eval_batch_end_callback=None,
            initializer=None, arg_params=None, aux_params=None, allow_missing=True, force_rebind=False,
            force_init=False, begin_epoch=0, num_epoch=None, validation_metric=None, monitor=None,
            max_steps=None, check_every=20, states_prefix=None, resume_states=None):
        """MXNet ``BaseModule.fit``.  Extras: ``max_steps`` (smoke runs), ``check_every`` (non-finite
        guard period), ``states_prefix`` (rank 0 writes ``<prefix>-%04d.states`` = momentum +
        update count at each epoch end) and ``resume_states`` (a .states file to restore after
        the optimizer is created; the data order also resumes at ``begin_epoch``)."""
        assert num_epoch is not None, 'please specify number of epochs'
        self.bind(for_training=True)
        if monitor is not None:
            self.install_monitor(monitor)
        self.init_params(initializer, arg_params, aux_params, allow_missing, force_init)
        self.init_optimizer(kvstore, optimizer, optimizer_params)
        if resume_states:
            self.load_optimizer_states(resume_states)
            logging.info('restored optimizer states from %s', resume_states)
        if begin_epoch > 0 and hasattr(train_data, 'epoch'):
            train_data.epoch = begin_epoch  # same shuffle as an uninterrupted run
            train_data.reset()
        rank = pdist.get_rank()
        cbs_b = batch_end_callback if isinstance(batch_end_callback, (list, tuple)) else \
            ([batch_end_callback] if batch_end_callback else [])
        cbs_e = epoch_end_callback if isinstance(epoch_end_callback, (list, tuple)) else \
            ([epoch_end_callback] if epoch_end_callback else [])
        hb = watchdog.from_env()
        self._hb = hb
        try:
            self._fit_loop(train_data, eval_metric, cbs_b, cbs_e, begin_epoch, num_epoch, max_steps, check_every,
                           states_prefix, rank, hb)
        finally:
            self._hb = None
            if hb is not None:
                hb.stop()
            if hasattr(train_data, 'close'):
                train_data.close()

    def _fit_loop(self, train_data, eval_metric, cbs_b, cbs_e, begin_epoch, num_epoch, max_steps, check_every,
                  states_prefix, rank, hb):
        import contextlib
        steps = 0
        fault_step, fault_kind = parse_fault(os.environ.get('MXR_FAULT_INJECT'))
        quiet = hb.paused if hb is not None else contextlib.nullcontext
        for epoch in range(begin_epoch, num_epoch):
            tic = time.time()
            if eval_metric is not None:
                eval_metric.reset()
            if hb is not None:
                hb.beat(steps)
            for nbatch, batch in enumerate(train_data):
                if self._monitor is not None:
                    self._monitor.tic()
                fault = fault_step is not None and steps == fault_step
                if fault:
                    self.trainer.arm_fault(fault_kind)
                self.step(batch)
                if fault:
                    self.trainer.disarm_fault()
                if hb is not None:
                    hb.beat(steps)
                if (steps + 1) % check_every == 0:
                    self.trainer.check_finite(steps)
                if eval_metric is not None:
                    self.update_metric(eval_metric)
                if self._monitor is not None:
                    self._monitor.toc_print()
                for cb in cbs_b:
                    cb(BatchEndParam(epoch, nbatch, eval_metric, locals()))
                steps += 1
                if max_steps is not None and steps >= max_steps:
                    break
            # epoch-end host phases (gather, checkpoint, reshuffle) are known to be long
            with quiet():
                self.trainer.check_finite(steps)
                if eval_metric is not None:
                    for name, val in eval_metric.get_name_value():
                        logging.info('Epoch[%d] Train-%s=%f', epoch, name, val)
                logging.info('Epoch[%d] Time cost=%.3f', epoch, time.time() - tic)
                arg, aux = self.get_params()
                if rank == 0:
                    for cb in cbs_e:
                        cb(epoch, self.symbol, arg, aux)
                    if states_prefix:
                        self.save_optimizer_states('%s-%04d.states' % (states_prefix, epoch + 1))
                if max_steps is not None and steps >= max_steps:
                    break
                train_data.reset()


def parse_fault(spec):
    """``MXR_FAULT_INJECT=nan@STEP`` (or ``inf@STEP``) -> (step, kind); None -> (None, None)."""
    if not spec:
        return None, None
    kind, _, at = spec.partition('@')
    return int(at), kind


def default_lr_scheduler(step, factor=0.1):
    return FactorScheduler(step, factor)
