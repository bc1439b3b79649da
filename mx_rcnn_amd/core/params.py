"""Flat parameter store: fp32 master weights + momentum, low-precision compute shadows and
flat gradient buffers (SURVEY §5.8 item 2, §2.9 SGD row).

Design (MI355X-first):
* Every trainable parameter lives in ONE flat buffer per (precision, weight-decay) group.
  The module's Parameter is re-pointed at a bf16 view of a flat "shadow" buffer, and its
  ``.grad`` is pre-set to a view of a flat gradient buffer, so autograd accumulates in
  place: zeroing grads is one memset, the all-reduce buckets are plain slices, and the
  fused SGD kernel (csrc/hip/sgd.hip) updates master + momentum and rewrites the bf16
  shadow in the same pass (no separate cast kernels per step).
* Buffers are ordered in REVERSE registration order (= roughly the order gradients become
  ready in backward) so bucket i can be all-reduced while backward still runs.
* BatchNorm affine parameters stay fp32 (the fused BN kernels take fp32 params).
* Frozen parameters (``fixed_param_prefix``, matched by SUBSTRING exactly like the
  reference `rcnn/module.py:50-55`) are cast once to the compute dtype and never updated.
* Weight decay follows MXNet's Optimizer.set_wd_mult: only names ending in ``_weight`` or
  ``_gamma`` are decayed.
"""
import logging
import os

import torch
import torch.nn as nn

from ..ops.sgd import sgd_momentum_
from ..ops import grad_sink
from ..ops import precision


def _is_bn_param(name):
    return name.endswith('_gamma') or name.endswith('_beta')


def match_fixed(name, prefixes):
    return any(p in name for p in (prefixes or []))


class ParamGroup:
    def __init__(self, key, entries, device, compute_dtype, x2=False):
        self.key = key  # (lowp: bool, decay: bool)
        lowp, decay = key
        self.decay = decay
        self.entries = entries  # list of (mx_name, module, attr, numel, shape, channels_last)
        self.numel = sum(e[3] for e in entries)
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.mom = torch.zeros(self.numel, dtype=torch.float32, device=device)
        # x2 = plane count of the fp32 modes (ops/precision.py: 2 bf16x3 pairs, 3 fp32 triples): the
        # parameters ARE the fp32 masters, gradients are fp32, and the shadow holds the bf16 planes
        # the MFMA kernels read -- plane k at [k * plane, k * plane + n), plane = n rounded up to a
        # multiple of 8 so every plane's rows stay 16-B aligned -- rewritten by the SGD kernel in
        # the same pass as the update
        self.x2 = (3 if x2 == 3 else 2) if (x2 and lowp) else 0
        self.plane = (self.numel + 7) // 8 * 8
        gd = compute_dtype if (lowp and not self.x2) else torch.float32
        if self.x2:
            self.shadow = torch.zeros(self.x2 * self.plane, dtype=torch.bfloat16, device=device)
        else:
            self.shadow = torch.zeros(self.numel, dtype=gd, device=device) if lowp else None
        self.grad = torch.zeros(self.numel, dtype=gd, device=device)
        self.offsets = []

    def sync_shadow(self):
        """Re-derive the shadow from the fp32 masters (after a load / broadcast)."""
        if self.shadow is None:
            return
        if self.x2:
            from ..ops import precision
            parts = precision.split(self.master, self.x2)
            n, pl = self.numel, self.plane
            for k in range(self.x2):
                self.shadow[k * pl:k * pl + n].copy_(parts[k * n:(k + 1) * n])
        else:
            self.shadow.copy_(self.master.to(self.shadow.dtype))


class FlatParamStore:
    def __init__(self, model, fixed_param_prefix=None, compute_dtype=torch.bfloat16, device=None,
                 channels_last=True, mode=None, x2=False):
        self.model = model
        self.compute_dtype = compute_dtype
        dev = torch.device(device) if device is not None else next(model.parameters()).device
        self.device = dev
        # x2: plane count of the fp32 training modes on the bf16 MFMA (ops/precision.py: 2 = bf16x3,
        # 3 = fp32); compute_dtype is then fp32
        self.x2 = (3 if x2 == 3 else 2) if x2 else 0
        lowp_enabled = compute_dtype != torch.float32 or self.x2
        fixed = fixed_param_prefix or []
        layers = list(model.mx_layers(mode)) if mode is not None else list(model.mx_layers())
        named = []  # (mx_name, module, attr, param)
        for m in layers:
            for attr, p in m._parameters.items():
                if p is None:
                    continue
                named.append(('%s_%s' % (m.mx_name, attr), m, attr, p))
        self.fixed_names = [n for n, _, _, _ in named if match_fixed(n, fixed)]
        for pfx in fixed:
            hits = [n for n in self.fixed_names if pfx in n and not n.startswith(pfx)]
            if hits:
                logging.warning('fixed_param_prefix %r also matches %d params by substring (e.g. %s)',
                                pfx, len(hits), hits[0])
        groups = {}
        for n, m, attr, p in reversed(named):
            if n in self.fixed_names:
                continue
            lowp = lowp_enabled and not _is_bn_param(n)
            decay = n.endswith('_weight') or n.endswith('_gamma')
            cl = channels_last and p.dim() == 4
            groups.setdefault((lowp, decay), []).append((n, m, attr, p.numel(), tuple(p.shape), cl))
        self.groups = [ParamGroup(k, v, dev, compute_dtype, self.x2) for k, v in sorted(groups.items())]
        self.params = {}
        self._fused = {}  # group index -> fused-update specs (enable_fused_sgd)
        with torch.no_grad():
            for g in self.groups:
                off = 0
                for n, m, attr, numel, shape, cl in g.entries:
                    src = m._parameters[attr].detach().to(dev, torch.float32)
                    g.offsets.append(off)
                    g.master[off:off + numel].copy_(self._flat_view(src, cl))
                    lowp = g.shadow is not None and not g.x2
                    storage = g.shadow if lowp else g.master
                    pv = self._shaped(storage[off:off + numel], shape, cl)
                    if lowp:
                        pv.copy_(src.to(compute_dtype))
                    param = nn.Parameter(pv, requires_grad=True)
                    param.grad = self._shaped(g.grad[off:off + numel], shape, cl)
                    grad_sink.enable_direct(param)
                    m._parameters[attr] = param
                    self.params[n] = param
                    if g.x2:  # the kernels' planes of this weight: plane-0 view + the group's plane spacing
                        precision.register_weight(param, self._shaped(g.shadow[off:off + numel], shape, cl),
                                                  g.plane, g.x2)
                    off += numel
                if g.x2:
                    g.sync_shadow()
            # frozen: cast once, no grad (the fp32 original is kept for checkpoints; the x2 mode
            # keeps them fp32 and the ops build their pairs once, ops/precision.py weight_pair)
            self.frozen_fp32 = {}
            for n, m, attr, p in named:
                if n in self.fixed_names:
                    self.frozen_fp32[n] = p.detach().to(dev, torch.float32).clone()
                    lowp = lowp_enabled and not _is_bn_param(n) and not self.x2
                    t = p.detach().to(dev, compute_dtype if lowp else torch.float32)
                    if channels_last and t.dim() == 4:
                        t = t.contiguous(memory_format=torch.channels_last)
                    m._parameters[attr] = nn.Parameter(t, requires_grad=False)
                    self.params[n] = m._parameters[attr]
        for b in model.buffers():
            b.data = b.data.to(dev)
        self._build_dgrad_cache()

    # ------------------------------------------------------------------ dgrad filter cache
    def _build_dgrad_cache(self):
        """Flipped/transposed bf16 copies of every trainable conv filter the MFMA dgrad path
        uses, refreshed by ONE multi-filter kernel after each update (ops/conv.py)."""
        self._wt_table = None
        if self.device.type != 'cuda' or (self.compute_dtype != torch.bfloat16 and not self.x2):
            return
        from ..ops import conv as conv_ops
        from ..ops._ext import need_ext
        ext = need_ext()
        srcs, dsts = [], []
        self._x2_entries = {}  # table entry -> (param, plane) of the x2 pair entries
        # stride-1 data gradients (and the FC's) read the forward filter transposed in-kernel
        # (ops/conv.py dgrad_args): only the strided k x k convs' parity sub-filters need the copy
        bt = conv_ops.dgrad_bt_enabled()
        for g in self.groups:
            if g.shadow is None:
                continue
            for (n, m, attr, numel, shape, cl), off in zip(g.entries, g.offsets):
                p = self.params[n]
                if bt and not (len(shape) == 4 and shape[2] > 1 and int(getattr(m, 'stride', 1)) > 1):
                    continue
                if getattr(m, 'in_shape', None) is not None:  # an FC held as a (C, H, W) filter: GEMM rows
                    continue
                if g.x2:
                    self._x2_dgrad_entry(g, p, off, numel, shape, cl, srcs, dsts)
                    continue
                if len(shape) == 2:  # FullyConnected (out, in): its transpose, for the FC data gradient
                    o, i = shape
                    if o % 64 != 0 or i % 64 != 0:
                        continue
                    buf = torch.empty((i, o, 1, 1), dtype=p.dtype, device=self.device,
                                      memory_format=torch.channels_last)
                    conv_ops.register_dgrad_weight(p, buf)
                    srcs.append(p.detach().view(o, i, 1, 1))
                    dsts.append(buf)
                    continue
                if len(shape) != 4 or not cl:
                    continue
                o, i, kh, kw = shape
                if o % 64 != 0 or i % 8 != 0 or kh != kw:
                    continue
                buf = torch.empty((i, o, kh, kw), dtype=p.dtype, device=self.device,
                                  memory_format=torch.channels_last)
                conv_ops.register_dgrad_weight(p, buf)
                srcs.append(p.detach())
                dsts.append(buf)
        self._wt_params = []
        if srcs:
            # the parameter (and, x2, the plane) behind each table entry: x2 entries are views of
            # the shadow, so they are recorded by _x2_dgrad_entry rather than found by pointer
            self._wt_params = [p for p in self._dgrad_params(srcs)]
            for k, (pp, pl) in self._x2_entries.items():
                self._wt_params[k] = pp
            self._wt_planes = [self._x2_entries.get(k, (None, -1))[1] for k in range(len(srcs))]
            self._wt_srcs, self._wt_dsts = srcs, dsts
            self._sub_in_table = set()
            n_ent, tiles = ext.wt_flip_table_info(srcs)
            self._wt_table = (ext.wt_flip_build(srcs, dsts), n_ent, tiles, dsts)
            self.refresh_dgrad_cache()

    def _x2_dgrad_entry(self, g, p, off, numel, shape, cl, srcs, dsts):
        """Multi-plane modes: the flipped / transposed filter of ``p`` as a planes buffer
        (P*I, O, kh, kw), filled by one flip-table entry per plane (from the shadow's plane views)."""
        from ..ops import conv as conv_ops
        P = g.x2
        starts = [k * g.plane for k in range(P)]
        if len(shape) == 2:
            o, i = shape
            if o % 64 != 0 or i % 64 != 0:
                return
            views = [g.shadow[pl + off:pl + off + numel].view(o, i, 1, 1) for pl in starts]
            buf = torch.empty((P * i, o, 1, 1), dtype=torch.bfloat16, device=self.device,
                              memory_format=torch.channels_last)
        else:
            if len(shape) != 4 or not cl:
                return
            o, i, kh, kw = shape
            if o % 64 != 0 or i % 8 != 0 or kh != kw:
                return
            views = [self._shaped(g.shadow[pl + off:pl + off + numel], shape, cl) for pl in starts]
            buf = torch.empty((P * i, o, kh, kw), dtype=torch.bfloat16, device=self.device,
                              memory_format=torch.channels_last)
        conv_ops.register_dgrad_weight(p, buf)
        for pl, (v, d) in enumerate(zip(views, [buf[k * i:(k + 1) * i] for k in range(P)])):
            self._x2_entries[len(srcs)] = (p, pl)
            srcs.append(v)
            dsts.append(d)

    def _dgrad_params(self, srcs):
        """The parameter behind each flip-table source (same order)."""
        by_ptr = {p.data_ptr(): p for p in self.params.values()}
        return [by_ptr.get(s.data_ptr()) for s in srcs]

    def _maybe_add_sub_filters(self):
        """Fold the parity sub-filters registered since the table was built (the strided data
        gradient registers them on its first backward) into the flip kernel's table, so they are
        written in the same pass instead of one copy kernel each.  Never while capturing: the
        table upload is a host-to-device copy."""
        from ..ops import conv as conv_ops
        if not conv_ops._SUBW or os.environ.get('MXR_SUBFILTER_FOLD', '1') == '0':
            return
        if torch.cuda.is_current_stream_capturing():
            return
        subs, have = [], set()
        for k, p in enumerate(self._wt_params):
            lst = conv_ops.sub_filters_of(p) if p is not None else []
            plane = self._wt_planes[k] if self.x2 else -1
            if plane >= 0 and lst:  # planes: this entry writes one plane of the (P*I, ...) sub-filters
                part = p.shape[1]
                lst = [(b[plane * part:(plane + 1) * part], r, c) for b, r, c in lst]
            rows = {tuple(r) for _, r, _ in lst}
            cols = {tuple(c) for _, _, c in lst}
            kh = p.shape[2] if (p is not None and p.dim() == 4) else 0
            full = (lst and len(lst) == len(rows) * len(cols) and len(rows) <= 2 and len(cols) <= 2 and
                    sum(len(r) for r in rows) == kh and sum(len(c) for c in cols) == p.shape[3])
            subs.append(lst if full else [])
            if full:
                have.add(id(p))
        if have == self._sub_in_table:
            return
        from ..ops._ext import need_ext
        _, n_ent, tiles, dsts = self._wt_table
        self._wt_table = (need_ext().wt_flip_build(self._wt_srcs, self._wt_dsts, subs), n_ent, tiles, dsts)
        self._sub_in_table = have

    def refresh_dgrad_cache(self):
        if self._wt_table is not None:
            from ..ops._ext import need_ext
            from ..ops.conv import refresh_sub_filters
            self._maybe_add_sub_filters()
            table, n_ent, tiles, _ = self._wt_table
            need_ext().wt_flip_run(table, n_ent, tiles)
            refresh_sub_filters(skip=self._sub_in_table)

    def refresh_dgrad_cache_async(self, zero_grad=False):
        """Rebuild the dgrad cache from the current weights on a side stream (concurrent with the
        forward pass, which does not read it); returns a callable that joins it into the compute
        stream (call before the backward pass).  ``zero_grad``: clear the flat gradient buffers on
        that side stream too, so the forward pass's first kernel depends on nothing issued in this
        step (the gradients are first written after the join)."""
        if self._wt_table is None or self.device.type != 'cuda' or os.environ.get('MXR_CACHE_SIDE', '1') == '0':
            if zero_grad:
                self.zero_grad()
            self.refresh_dgrad_cache()
            return lambda: None
        main = torch.cuda.current_stream(self.device)
        if getattr(self, '_cache_stream', None) is None:
            from ..models.faster_rcnn import _aux_stream
            self._cache_stream = _aux_stream(self.device, 'cache')
        side = self._cache_stream
        from ..models.faster_rcnn import fork
        fork(side, main)
        with torch.cuda.stream(side):
            if zero_grad:
                self.zero_grad()
            self.refresh_dgrad_cache()
        done = torch.cuda.Event()
        done.record(side)  # the join waits for this work only (the side stream may carry later roles)
        return lambda: main.wait_event(done)

    @staticmethod
    def _flat_view(t, cl):
        if cl:
            return t.permute(0, 2, 3, 1).reshape(-1)
        return t.reshape(-1)

    @staticmethod
    def _shaped(flat, shape, cl):
        if cl:
            o, i, kh, kw = shape
            return flat.view(o, kh, kw, i).permute(0, 3, 1, 2)
        return flat.view(shape)

    # ------------------------------------------------------------------ data parallel
    @torch.no_grad()
    def broadcast_(self, src=0):
        """Make every rank start from rank ``src``'s weights (the reference's ranks load one
        checkpoint; random-init or per-rank-calibrated models would otherwise train apart):
        the flat fp32 masters (bf16 shadows re-derived), the frozen parameters and the model
        buffers (BN moving statistics), then the dgrad filter cache."""
        import torch.distributed as dist
        for g in self.groups:
            dist.broadcast(g.master, src)
            g.sync_shadow()
        for n in self.fixed_names:
            dist.broadcast(self.frozen_fp32[n], src)
            self.params[n].data.copy_(self.frozen_fp32[n].to(self.params[n].dtype))
            precision.forget_weight(self.params[n])  # .data writes do not move the version counter
        for b in self.model.buffers():
            if b.is_floating_point() or b.dtype in (torch.int32, torch.int64):
                t = b.data if b.is_contiguous() else b.data.contiguous()
                dist.broadcast(t, src)
                if t is not b.data:
                    b.data.copy_(t)
        self.refresh_dgrad_cache()

    @torch.no_grad()
    def weights_digest(self):
        """A bit-sensitive checksum of every trainable fp32 master (int in [0, 2^31 - 1)): equal on
        data-parallel replicas exactly when their weights are bitwise equal (up to hash collisions).
        One device reduction per group; for checks outside the timed region."""
        mod = (1 << 31) - 1
        acc = 0
        for g in self.groups:
            v = g.master.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
            w = torch.arange(v.numel(), device=v.device, dtype=torch.int64) % 8191 + 1
            acc = (acc * 1000003 + int(((v * w) % mod).sum().item())) % mod
        return acc

    # ------------------------------------------------------------------ step pieces
    def zero_grad(self):
        for g in self.groups:
            g.grad.zero_()

    def grad_buffers(self):
        return [g.grad for g in self.groups]

    def sgd_step(self, lr, momentum=0.9, wd=0.0005, rescale=1.0, clip=-1.0, grad_for=None, refresh=True,
                 clear=False):
        """``lr``: 1-element fp32 device tensor.  ``grad_for(group)`` picks the gradient source
        (the reducer's fp32 all-reduce buffer under data parallelism; default ``group.grad``).
        ``refresh=False``: the caller rebuilds the dgrad cache itself (Trainer.step_body does, at
        the start of the next step, concurrently with its forward pass).  ``clear``: the update
        kernel zeroes each group's gradient buffer after reading it (replaces zero_grad).
        Parameters whose update ran fused into their weight gradient this step
        (enable_fused_sgd), and ranges the reducer already updated after their all-reduce
        (:meth:`mark_updated`), are skipped."""
        early = getattr(self, '_early', {})
        self._early = {}
        for gi, g in enumerate(self.groups):
            grad = grad_for(g) if grad_for is not None else g.grad
            skip = sorted([(sp['off'], sp['off'] + sp['numel']) for sp in self._fused.get(gi, ()) if sp['applied']] +
                          early.get(id(g), []))
            for sp in self._fused.get(gi, ()):
                sp['applied'] = False
            if not skip:
                sgd_momentum_(g.master, g.mom, grad, lr, momentum, wd if g.decay else 0.0, rescale, clip, g.shadow,
                              planes=g.x2 or 1, zero=g.grad if clear else None)
                continue
            cuts, at = [], 0
            for s0, e0 in skip:
                if s0 > at:
                    cuts.append((at, s0))
                at = max(at, e0)
            if at < g.numel:
                cuts.append((at, g.numel))
            for s0, e0 in cuts:  # the complement of the fused ranges
                if g.x2:
                    sh, pst = g.shadow[s0:], g.plane
                else:
                    sh, pst = (g.shadow[s0:e0] if g.shadow is not None else None), 0
                sgd_momentum_(g.master[s0:e0], g.mom[s0:e0], grad[s0:e0], lr, momentum, wd if g.decay else 0.0, rescale,
                              clip, sh, planes=g.x2 or 1, zero=g.grad[s0:e0] if clear else None, plane_stride=pst)
        if refresh:
            self.refresh_dgrad_cache()

    def mark_updated(self, group, start, end):
        """[start, end) of ``group`` got its SGD update this step already (the reducer's per-bucket
        update after the bucket's all-reduce, parallel/reducer.py): the next sgd_step skips it."""
        if not hasattr(self, '_early'):
            self._early = {}
        self._early.setdefault(id(group), []).append((int(start), int(end)))

    def enable_fused_sgd(self, names, lr, momentum=0.9, wd=0.0005, rescale=1.0, clip=-1.0):
        """Let the weight-gradient kernels of parameters ``names`` apply their SGD update in place
        (csrc conv_wgrad_sgd: the gradient is never stored; ops/vgg_fused.py).  Only parameters whose
        flat offset keeps the kernel's 16-B rows aligned qualify.  Returns the enabled names."""
        self.disable_fused_sgd()
        done = []
        if self.device.type != 'cuda':
            return done
        for gi, g in enumerate(self.groups):
            for (n, _, _, numel, shape, cl), off in zip(g.entries, g.offsets):
                if n not in names or off % 8 or numel % 8:
                    continue
                if g.x2:
                    sh, planes, pst = g.shadow[off:], g.x2, g.plane
                else:
                    sh, planes, pst = (g.shadow[off:off + numel] if g.shadow is not None else None), 1, 0
                spec = {'w': g.master[off:off + numel], 'mom': g.mom[off:off + numel], 'shadow': sh, 'planes': planes,
                        'plane_stride': pst, 'lr': lr, 'momentum': float(momentum),
                        'wd': float(wd) if g.decay else 0.0, 'rescale': float(rescale), 'clip': float(clip),
                        'grad_bf16': g.grad.dtype == torch.bfloat16, 'off': off, 'numel': numel, 'applied': False}
                grad_sink.set_fused_sgd(self.params[n], spec)
                self._fused.setdefault(gi, []).append(spec)
                done.append(n)
        return done

    def disable_fused_sgd(self):
        for specs in getattr(self, '_fused', {}).values():
            for sp in specs:
                sp['applied'] = False
        for p in self.params.values():
            grad_sink.set_fused_sgd(p, None)
        self._fused = {}

    def master_param(self, name):
        for g in self.groups:
            for (n, _, _, numel, shape, cl), off in zip(g.entries, g.offsets):
                if n == name:
                    return self._shaped(g.master[off:off + numel], shape, cl)
        if name in self.frozen_fp32:
            return self.frozen_fp32[name]
        return self.params[name].detach().float()

    def optimizer_state(self):
        """Momentum of every trainable parameter (fp32, parameter layout) for exact resume."""
        out = {}
        for g in self.groups:
            for (n, _, _, numel, shape, cl), off in zip(g.entries, g.offsets):
                out[n] = self._shaped(g.mom[off:off + numel], shape, cl).contiguous()
        return out

    def load_optimizer_state(self, arrays):
        missing = []
        with torch.no_grad():
            for g in self.groups:
                for (n, _, _, numel, shape, cl), off in zip(g.entries, g.offsets):
                    if n not in arrays:
                        missing.append(n)
                        continue
                    src = torch.as_tensor(arrays[n]).to(self.device, torch.float32).reshape(shape)
                    g.mom[off:off + numel].copy_(self._flat_view(src, cl))
        return missing

    def state_arrays(self):
        """fp32 copies of every parameter (trainable from master, frozen from the cast copy)."""
        return {n: self.master_param(n).contiguous() for n in self.params}

    def load_arrays(self, arrays, strict=False):
        """Copy fp32 arrays into master/shadow (trainable) or the frozen copies."""
        missing = []
        with torch.no_grad():
            for n, p in self.params.items():
                if n not in arrays:
                    missing.append(n)
                    continue
                src = torch.as_tensor(arrays[n]).to(self.device, torch.float32).reshape(p.shape)
                found = False
                for g in self.groups:
                    for (gn, _, _, numel, shape, cl), off in zip(g.entries, g.offsets):
                        if gn == n:
                            g.master[off:off + numel].copy_(self._flat_view(src, cl))
                            p.data.copy_(src.to(p.dtype))
                            precision.forget_weight(p)
                            found = True
                            if g.x2:
                                g.sync_shadow()
                if not found:
                    p.data.copy_(src.to(p.dtype))
                    precision.forget_weight(p)  # .data writes do not move the version counter
                    if n in self.frozen_fp32:
                        self.frozen_fp32[n].copy_(src)
        self.refresh_dgrad_cache()
        if strict and missing:
            raise KeyError('missing params: %s' % missing[:10])
        return missing
