"""Faster R-CNN / Fast R-CNN / RPN model (reference graph builders `rcnn/symbol.py:164-386`,
`rcnn/resnet.py:67-193`), one nn.Module per network with mode-specific entry points
instead of seven separate symbols:

* ``train_e2e``   approximate-joint end-to-end training (`get_faster_rcnn`, resnet is_train)
* ``train_rpn``   RPN-only training (`get_vgg_rpn`)
* ``train_rcnn``  Fast R-CNN on given RoIs (`get_vgg_rcnn`)
* ``rpn_test``    RPN proposals (`get_vgg_rpn_test`)
* ``detect``      Faster R-CNN test (`get_vgg_test`, resnet test) or, with ``rois``,
                  Fast R-CNN test (`get_vgg_rcnn_test`)

All detection stages run on the device with static shapes: anchor target, proposal,
proposal target and RoIPool are HIP kernels; no host synchronisation in a training step,
so the whole step can be captured in a hipGraph (core/graph.py).  Images per device may be
> 1 (the reference is limited to 1: `rcnn/rpn/proposal.py:194`).
"""
import math

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..config import config as _global_cfg, snapshot
from ..utils import profiler as prof
from ..ops import anchor_target, proposal, proposal_target, roi_pool
from ..ops._ext import unit_grad
from ..ops.head import rpn_head
from ..ops.roi_pool import roi_pool_bn_relu
from ..ops.losses import combine_losses, rpn_softmax_ce, smooth_l1, softmax_ce
from .layers import Conv
from .resnet import ResNetHead, ResNetTrunk
from .vgg import VGG16Trunk, VGGHead

VGG_SCALES = (8, 16, 32)
RESNET_SCALES = (4, 8, 16, 32)
RATIOS = (0.5, 1, 2)


class RPNHead(nn.Module):
    def __init__(self, in_channels, num_anchors, mid=512):
        super().__init__()
        self.rpn_conv_3x3 = Conv('rpn_conv_3x3', in_channels, mid, 3, 1, 1)
        self.rpn_cls_score = Conv('rpn_cls_score', mid, 2 * num_anchors, 1, 1, 0)
        self.rpn_bbox_pred = Conv('rpn_bbox_pred', mid, 4 * num_anchors, 1, 1, 0)
        # reference init for new layers (train_end2end.py:62-78): N(0,.01), N(0,.001) for bbox
        nn.init.normal_(self.rpn_conv_3x3.weight, 0, 0.01)
        nn.init.normal_(self.rpn_cls_score.weight, 0, 0.01)
        nn.init.normal_(self.rpn_bbox_pred.weight, 0, 0.001)

    def forward(self, feat):
        # conv + ReLU + both predictors as one op: its backward is one kernel for the two 1x1 heads
        # with the ReLU backward fused (ops/head.py); falls back to the three modules elsewhere
        return rpn_head(feat, self.rpn_conv_3x3, self.rpn_cls_score, self.rpn_bbox_pred)


class FasterRCNN(nn.Module):
    def __init__(self, network='vgg16', num_classes=21, cfg=None, bn_mom=0.99, num_anchors=None,
                 anchor_scales=None, anchor_ratios=RATIOS, resnet_spec=None, train_mode='e2e'):
        super().__init__()
        self.cfg = cfg if cfg is not None else snapshot()
        # the trainer's device-side non-finite step counter, bumped by the loss-combine kernel
        # (core/trainer.py hands it over; None = the caller checks the objective itself)
        self.nonfinite_counter = None
        # int32 device counter: images whose multi-workgroup NMS chain gave up a poll and were
        # redone by the serial fallback (csrc/hip/nms.hip); observability only, never a failure
        self.nms_gave_up = None
        self.network = network
        self.num_classes = num_classes
        if network == 'vgg16' or network == 'vgg':
            self.trunk = VGG16Trunk()
            self.head = VGGHead(num_classes)
            self.anchor_scales = tuple(anchor_scales or VGG_SCALES)
        elif network.startswith('resnet'):
            depth = resnet_spec if resnet_spec is not None else \
                int(network.replace('resnet', '').replace('-', '').replace('_', ''))
            self.trunk = ResNetTrunk(depth, bn_mom=bn_mom)
            self.head = ResNetHead(num_classes, depth, bn_mom=bn_mom)
            self.anchor_scales = tuple(anchor_scales or RESNET_SCALES)
            # random-init stand-in for pretrained weights: MSRA on the branch convs, small
            # residual-branch outputs (conv3 / shortcut) so 100+ pre-activation units stay bounded
            for mod in (self.trunk, self.head.stage4):
                for m in mod.modules():
                    if isinstance(m, Conv):
                        if m.mx_name.endswith('_conv3') or m.mx_name.endswith('_sc'):
                            nn.init.normal_(m.weight, 0, 0.01)
                        else:
                            nn.init.kaiming_normal_(m.weight, nonlinearity='relu')
        else:
            raise ValueError('unknown network %r' % network)
        self.anchor_ratios = tuple(anchor_ratios)
        self.train_mode = train_mode
        self.num_anchors = num_anchors or len(self.anchor_scales) * len(self.anchor_ratios)
        self.feat_stride = 16
        self.rpn = RPNHead(self.trunk.out_channels, self.num_anchors)
        nn.init.normal_(self.head.cls_score.weight, 0, 0.01)
        nn.init.normal_(self.head.bbox_pred.weight, 0, 0.01)
        if network.startswith('vgg'):
            nn.init.normal_(self.head.fc6.weight, 0, 0.005)
            nn.init.normal_(self.head.fc7.weight, 0, 0.005)

    # ------------------------------------------------------------------ naming / params
    GRAPH_PARTS = {'rpn': ('trunk', 'rpn'), 'rpn_test': ('trunk', 'rpn'), 'rcnn': ('trunk', 'head'),
                   'rcnn_test': ('trunk', 'head')}

    def mx_layers(self, mode=None):
        """Named layers of the graph ``mode`` builds: the RPN graphs (`rcnn/symbol.py` get_*_rpn)
        hold no Fast R-CNN head and the RCNN graphs no RPN, so their checkpoints / optimizers
        only see those parameters; every other mode (e2e, test) holds all of them."""
        parts = self.GRAPH_PARTS.get(mode)
        mods = self.modules() if parts is None else (m for p in parts for m in getattr(self, p).modules())
        for m in mods:
            if hasattr(m, 'mx_args'):
                yield m

    def arg_params(self, mode=None):
        out = {}
        for m in self.mx_layers(mode):
            out.update(m.mx_args())
        return out

    def arg_shapes(self, mode=None):
        """MXNet checkpoint shapes of arg_params() (Linear(in_shape=...) weights flattened)."""
        out = {}
        for m in self.mx_layers(mode):
            out.update(m.mx_arg_shapes())
        return out

    def aux_params(self, mode=None):
        out = {}
        for m in self.mx_layers(mode):
            out.update(m.mx_aux())
        return out

    @torch.no_grad()
    def calibrate_bn(self, data):
        """Set the trunk's frozen BN moving statistics from one fp32 forward over ``data`` (N,3,H,W).
        Random-init ResNets have no meaningful frozen statistics; without this their activations
        grow through 100+ pre-activation units.  Pretrained checkpoints carry real ones (load them
        after, or skip this)."""
        bns = [m for m in self.trunk.modules() if hasattr(m, 'moving_var')]
        was = self.training
        self.eval()
        for m in bns:
            m._calibrate = True
        try:
            self.trunk(data.float())
        finally:
            for m in bns:
                m._calibrate = False
            self.train(was)
        return len(bns)

    @torch.no_grad()
    def calibrate_vgg(self, data):
        """Data-dependent init of a random VGG16 trunk (the stand-in for the ImageNet weights the
        reference always loads, `train_end2end.py:56-78`): layer by layer, an MSRA-normal filter
        rescaled so the pre-activation over ``data`` (N,3,H,W) has unit standard deviation, zero
        bias (LSUV).  The N(0, 0.01) default leaves 13 plain conv layers with vanishing
        activations, a trunk that random-init training cannot move."""
        import torch.nn.functional as Fn
        from .layers import max_pool
        trunk = self.trunk
        x = data.float().cpu()
        g = torch.Generator().manual_seed(0)
        for i, c in enumerate(trunk.convs):
            w = torch.randn(c.weight.shape, generator=g) * (2.0 / c.weight[0].numel()) ** 0.5
            y = Fn.conv2d(x, w, None, 1, 1)
            w /= float(y.std()) + 1e-12
            c.weight.copy_(w.to(c.weight.device, c.weight.dtype))
            if c.bias is not None:
                c.bias.zero_()
            x = torch.relu(y / (float(y.std()) + 1e-12))
            if i in trunk.pool_after:
                x = max_pool(x, 2, 2)
        return len(trunk.convs)

    def feat_shape(self, h, w):
        return self.trunk.feat_shape(h, w)

    # ------------------------------------------------------------------ pieces
    def _proposal(self, rpn_cls, rpn_bbox, im_info, key, is_prob=False, after_mask=None):
        c = self.cfg[key]
        if rpn_cls.is_cuda and (self.nms_gave_up is None or self.nms_gave_up.device != rpn_cls.device):
            self.nms_gave_up = torch.zeros(1, dtype=torch.int32, device=rpn_cls.device)
        return proposal(rpn_cls.detach(), rpn_bbox.detach(), im_info, self.feat_stride, self.anchor_scales,
                        self.anchor_ratios, c.RPN_PRE_NMS_TOP_N, c.RPN_POST_NMS_TOP_N, c.RPN_NMS_THRESH,
                        c.RPN_MIN_SIZE, is_train=(key == 'TRAIN'), is_prob=is_prob, after_mask=after_mask,
                        gave_up=self.nms_gave_up if rpn_cls.is_cuda else None)

    def _anchor_target_async(self, data, im_info, gt_boxes, n_gt):
        """Start the RPN anchor-target assignment (which needs only the image shape and the gt
        boxes) on an auxiliary stream, concurrent with the trunk forward; returns a callable that
        joins it into the compute stream and yields the targets."""
        H, W = self.feat_shape(data.shape[2], data.shape[3])

        def run():
            return anchor_target((H, W), gt_boxes, n_gt, im_info, self.feat_stride, self.anchor_scales,
                                 self.anchor_ratios, allowed_border=0, cfg=self.cfg)
        if not data.is_cuda or os.environ.get('MXR_AUX_STREAM', '1') == '0':
            at = run()
            return lambda: at
        main = torch.cuda.current_stream()
        aux = _aux_stream(data.device)
        fork(aux, main)
        with torch.cuda.stream(aux):
            at = run()
        done = _mark(aux)  # the join waits for THIS work only (the side stream may carry later roles)

        def join():
            main.wait_event(done)
            for t in at.values():
                t.record_stream(main)
            return at
        join.stream, join.at = aux, at  # for _rpn_losses_async: the losses can stay on this stream
        return join

    def _rpn_losses_async(self, rpn_cls, rpn_bbox, im_info, gt_boxes, n_gt, at_join):
        """The RPN losses on the auxiliary stream that holds the anchor targets, issued right after
        the RPN forward: the proposal chain (decode, top-k, NMS -> sampling -> RoI pooling), the
        step's serial critical path, then starts without waiting for them.  Returns a callable that
        joins the stream and yields (cls_loss, bbox_loss, anchor targets)."""
        aux = getattr(at_join, 'stream', None)
        if aux is None:
            res = self._rpn_losses(rpn_cls, rpn_bbox, im_info, gt_boxes, n_gt, at_join())
            return lambda: res
        main = torch.cuda.current_stream()
        fork(aux, main)  # the RPN outputs (nothing later on main is waited for)
        rpn_cls.record_stream(aux)
        rpn_bbox.record_stream(aux)
        with torch.cuda.stream(aux):
            res = self._rpn_losses(rpn_cls, rpn_bbox, im_info, gt_boxes, n_gt, at_join.at)
        done = _mark(aux)

        def join():
            main.wait_event(done)
            for t in (res[0], res[1]) + tuple(res[2].values()):
                t.record_stream(main)
            return res
        return join

    def _rpn_losses(self, rpn_cls, rpn_bbox, im_info, gt_boxes, n_gt, at=None):
        H, W = rpn_cls.shape[2], rpn_cls.shape[3]
        if at is None:
            at = anchor_target((H, W), gt_boxes, n_gt, im_info, self.feat_stride, self.anchor_scales,
                               self.anchor_ratios, allowed_border=0, cfg=self.cfg)
        assert at['label'].shape[1] == rpn_cls.shape[1] // 2 * H * W, 'anchor grid / RPN map mismatch'
        cls_loss = rpn_softmax_ce(rpn_cls, at['label'], sample_meta=at.get('sample_meta'))
        bbox_loss = smooth_l1(rpn_bbox, at['bbox_target'], at['bbox_inside_weight'], at['bbox_outside_weight'],
                              sigma=3.0, grad_scale=1.0, slot=2)
        return cls_loss, bbox_loss, at

    def _head_losses(self, cls_score, bbox_pred, label, bbox_target, inside, outside, e2e=True):
        """e2e graph: SoftmaxOutput('batch') + MakeLoss(grad_scale=1/BATCH_SIZE) (`rcnn/symbol.py:372-378`);
        Fast R-CNN graph: normalization 'null', grad_scale 1, the optimizer's rescale_grad =
        1/BATCH_SIZE does the scaling (`rcnn/symbol.py:105-111`, `tools/train_rcnn.py`)."""
        cls_loss, cls_prob = softmax_ce(cls_score, label, 'batch' if e2e else 'null')
        bbox_loss = smooth_l1(bbox_pred, bbox_target, inside, outside, sigma=1.0,
                              grad_scale=1.0 / float(self.cfg.TRAIN.BATCH_SIZE) if e2e else 1.0, slot=3)
        return cls_loss, bbox_loss, cls_prob

    # ------------------------------------------------------------------ modes
    def _early_rpn_backward(self, data):
        """Run the RPN branch's backward before the proposal chain finishes (e2e training on the
        GPU).  The proposal chain -- decode, top-k, NMS, RoI sampling -- is a few hundred us of
        single-workgroup kernels with the rest of the chip idle, and nothing in the RPN losses'
        backward depends on it (proposals are not differentiable), so it runs on its own stream
        while the compute stream does the RPN head's backward; the head's feature gradient then
        enters the trunk through the RoI-pooling backward kernel (``grad_add``)."""
        return (data.is_cuda and torch.is_grad_enabled() and os.environ.get('MXR_EARLY_RPN_BWD', '1') != '0'
                and os.environ.get('MXR_AUX_STREAM', '1') != '0')

    def _proposal_target_async(self, rpn_cls, rpn_bbox, im_info, gt_boxes, n_gt):
        """Proposal + proposal target on the proposal stream; returns a join -> targets dict."""
        main = torch.cuda.current_stream()
        ps = _aux_stream(rpn_cls.device, 'proposal')
        fork(ps, main)

        def mask_done():
            # the compute stream resumes once the (all-CU) NMS bitmask is built: its RPN backward
            # then shares the chip only with the single-workgroup NMS reduce and RoI sampling
            main.wait_stream(ps)
        with torch.cuda.stream(ps):
            rois, _ = self._proposal(rpn_cls, rpn_bbox, im_info, 'TRAIN', after_mask=mask_done)
            pt = proposal_target(rois, gt_boxes, n_gt, self.num_classes, cfg=self.cfg, is_train=True)
        done = _mark(ps)

        def join():
            main.wait_event(done)
            for t in pt.values():
                if torch.is_tensor(t):
                    t.record_stream(main)
            return pt
        return join

    def train_e2e(self, data, im_info, gt_boxes, n_gt):
        """Approximate joint training step forward.  Returns dict with 'loss' (to backward)
        and the metric tensors of the reference's six metrics (rcnn/metric.py)."""
        at_join = self._anchor_target_async(data, im_info, gt_boxes, n_gt)
        early = self._early_rpn_backward(data)
        with prof.range('trunk'):
            feat = self.trunk(data)
        # early RPN backward: the RPN head reads a detached alias of the feature map, so the main
        # backward (from the R-CNN losses) does not revisit it
        feat_rpn = feat.detach().requires_grad_() if early else feat
        with prof.range('rpn'):
            rpn_cls, rpn_bbox = self.rpn(feat_rpn)
        with prof.range('anchor_target+rpn_loss'):
            rpn_losses = self._rpn_losses_async(rpn_cls, rpn_bbox, im_info, gt_boxes, n_gt, at_join)
        d_feat = None
        if early:
            with prof.range('proposal'):  # issue only: the chain runs on the proposal stream
                pt_join = self._proposal_target_async(rpn_cls, rpn_bbox, im_info, gt_boxes, n_gt)
            rpn_cls_loss, rpn_bbox_loss, at = rpn_losses()
            with prof.range('rpn_backward'):
                pre = getattr(self, 'pre_backward', None)
                if pre is not None:
                    pre()  # e.g. the trainer's dgrad filter-cache join
                one = unit_grad(data.device)  # recognised by the loss ops: no scale kernels
                torch.autograd.backward([rpn_cls_loss, rpn_bbox_loss], [one, one])
                d_feat = feat_rpn.grad
            pt = pt_join()
        else:
            with prof.range('proposal'):
                rois, _ = self._proposal(rpn_cls, rpn_bbox, im_info, 'TRAIN')
            with prof.range('proposal_target'):
                pt = proposal_target(rois, gt_boxes, n_gt, self.num_classes, cfg=self.cfg, is_train=True)
        with prof.range('roi_pool'):
            pooled = roi_pool(feat, pt['rois'], (7, 7), 1.0 / self.feat_stride, grad_add=d_feat)
        with prof.range('head'):
            cls_score, bbox_pred = self.head(pooled)
        with prof.range('head_loss'):
            cls_loss, bbox_loss, cls_prob = self._head_losses(cls_score, bbox_pred, pt['label'], pt['bbox_target'],
                                                              pt['bbox_inside_weight'], pt['bbox_outside_weight'])
        if not early:
            rpn_cls_loss, rpn_bbox_loss, at = rpn_losses()
        B = data.shape[0]
        R = cls_score.shape[0]
        # 'loss' carries the gradients (each loss applies its own grad_scale in backward); its value
        # mixes normalised and summed terms like the reference's outputs.  'objective' is the
        # value of the function actually being minimised.  One launch for both (+ the trainer's
        # non-finite counter when it handed one over).  After an early RPN backward the RPN terms
        # enter only the value.
        r_terms = [rpn_cls_loss.detach(), rpn_bbox_loss.detach()] if early else [rpn_cls_loss, rpn_bbox_loss]
        loss, obj = combine_losses(r_terms + [cls_loss, bbox_loss],
                                   [1.0, 1.0, 1.0, 1.0 / float(self.cfg.TRAIN.BATCH_SIZE)], self.nonfinite_counter)
        return {'loss': loss, 'objective': obj, 'rpn_cls_loss': rpn_cls_loss, 'rpn_bbox_loss': rpn_bbox_loss,
                'cls_loss': cls_loss, 'bbox_loss': bbox_loss, 'cls_prob': cls_prob, 'label': pt['label'],
                'rpn_cls_score': rpn_cls, 'rpn_label': at['label'], 'num_images': B, 'num_rois': R}

    def train_rpn(self, data, im_info, gt_boxes, n_gt):
        at_join = self._anchor_target_async(data, im_info, gt_boxes, n_gt)
        feat = self.trunk(data)
        rpn_cls, rpn_bbox = self.rpn(feat)
        cls_loss, bbox_loss, at = self._rpn_losses(rpn_cls, rpn_bbox, im_info, gt_boxes, n_gt, at_join())
        loss, obj = combine_losses([cls_loss, bbox_loss], [1.0, 1.0], self.nonfinite_counter)
        return {'loss': loss, 'objective': obj,
                'rpn_cls_loss': cls_loss, 'rpn_bbox_loss': bbox_loss, 'rpn_cls_score': rpn_cls, 'rpn_label': at['label'], 'num_images': data.shape[0]}

    def train_rcnn(self, data, rois, label, bbox_target, inside, outside):
        feat = self.trunk(data)
        pooled = roi_pool(feat, rois, (7, 7), 1.0 / self.feat_stride)
        cls_score, bbox_pred = self.head(pooled)
        cls_loss, bbox_loss, cls_prob = self._head_losses(cls_score, bbox_pred, label, bbox_target, inside, outside,
                                                          e2e=False)
        k = 1.0 / float(self.cfg.TRAIN.BATCH_SIZE)
        loss, obj = combine_losses([cls_loss, bbox_loss], [k, k], self.nonfinite_counter)
        return {'loss': loss, 'objective': obj,
                'cls_loss': cls_loss, 'bbox_loss': bbox_loss, 'cls_prob': cls_prob,
                'label': label, 'num_images': data.shape[0], 'num_rois': rois.shape[0]}

    @torch.no_grad()
    def rpn_test(self, data, im_info):
        feat = self.trunk(data)
        rpn_cls, rpn_bbox = self.rpn(feat)
        return self._proposal(rpn_cls, rpn_bbox, im_info, 'TEST')

    @torch.no_grad()
    def detect(self, data, im_info, rois=None):
        """Returns (rois (R, 5), cls_prob (R, C), bbox_pred (R, 4C)) with R = B * post (or given)."""
        feat = self.trunk(data)
        if rois is None:
            rpn_cls, rpn_bbox = self.rpn(feat)
            rois, _ = self._proposal(rpn_cls, rpn_bbox, im_info, 'TEST')
            rois = rois.reshape(-1, 5)
        bn = self.head.pool_bn(feat) if hasattr(self.head, 'pool_bn') else None
        if bn is not None:  # the head's first bn1 + ReLU in the pooling kernel (ops/roi_pool.py)
            act = roi_pool_bn_relu(feat, rois, (7, 7), 1.0 / self.feat_stride, bn)
            cls_score, bbox_pred = self.head(act, act1=act)
        else:
            pooled = roi_pool(feat, rois, (7, 7), 1.0 / self.feat_stride)
            cls_score, bbox_pred = self.head(pooled)
        return rois, torch.softmax(cls_score.float(), dim=1), bbox_pred.float()


_AUX = {}


def fork(side, main=None):
    """side.wait_stream(main), shaped for hipGraph replay: the runtime spreads a captured graph's
    parallel branches over its queues by walking the DAG depth-first, the FIRST child of a node
    continuing the node's queue.  A fork whose side kernel is captured before main's next kernel
    hands the main chain to a new queue (every later hop costs a cross-queue wait), so a no-op on
    main takes the first-child slot before the side branch starts (MXR_FORK_NOOP=0: plain fork)."""
    main = main if main is not None else torch.cuda.current_stream()
    if os.environ.get('MXR_FORK_NOOP', '1') == '0':
        side.wait_stream(main)
        return
    ev = torch.cuda.Event()
    ev.record(main)
    with torch.cuda.stream(main):
        torch.cuda._sleep(0)
    side.wait_event(ev)


def _mark(stream):
    """An event recorded on ``stream`` now: a join that waits on it depends on the work issued so
    far only, not on what a shared side stream (MXR_SIDE_STREAMS=1) carries for later roles."""
    ev = torch.cuda.Event()
    ev.record(stream)
    return ev


def _aux_stream(device, role='aux'):
    """Per-device side stream of a role ('aux': anchor targets / RPN losses, 'proposal': the
    proposal chain, 'cache': the dgrad filter cache + gradient clear).  MXR_SIDE_STREAMS=1 (the
    default under the runtime's own graph-queue count) puts every role on ONE side stream: fewer
    parallel branches in the captured step's DAG, fewer cross-queue waits (mx_rcnn_amd/__init__.py);
    with the opt-in MXR_GRAPH_QUEUES=2 one stream per role measured better (default 0 there)."""
    dflt = '0' if os.environ.get('DEBUG_HIP_FORCE_GRAPH_QUEUES') else '1'
    if os.environ.get('MXR_SIDE_STREAMS', dflt) == '1':
        role = 'aux'
    s = _AUX.get((device.index, role))
    if s is None:
        s = torch.cuda.Stream(device=device)
        _AUX[(device.index, role)] = s
    return s


def build_model(network='vgg16', num_classes=21, cfg=None, **kw):
    return FasterRCNN(network, num_classes, cfg=cfg, **kw)
