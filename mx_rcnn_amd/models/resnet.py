"""Pre-activation ResNet-18/34/50/101/152/200 in the C4 detection layout (reference
`rcnn/resnet.py:5-223`): stages 1-3 with frozen BN (use_global_stats) form the trunk,
RPN + RoIPool sit after the last unit of stage 3, stage 4 runs per RoI with batch-statistics
BN (the reference's ``bn_global_`` switch), then bn1 -> relu -> global avg-pool -> cls/bbox.
"""
import os

import torch
import torch.nn as nn

from ..ops.conv import igemm_eligible, weight_ok
from ..ops.fused import conv_add, conv_add_bn_relu, conv_bn_relu, fused_unit
from ..ops.head import fc_pair
from ..ops.pool import global_avg_pool, kernel_path, max_pool_bn_relu, post_bn_ok
from ..ops.stem import stem_fusable, stem_conv
from .layers import BatchNorm, Conv, Linear, max_pool


def fusion_enabled():
    return os.environ.get('MXR_FUSE', '1') != '0'


def _frozen(bn):
    return bn.use_global_stats or not bn.training

DEPTHS = {
    18: ([2, 2, 2, 2], [64, 64, 128, 256, 512], False),
    34: ([3, 4, 6, 3], [64, 64, 128, 256, 512], False),
    50: ([3, 4, 6, 3], [64, 256, 512, 1024, 2048], True),
    101: ([3, 4, 23, 3], [64, 256, 512, 1024, 2048], True),
    152: ([3, 8, 36, 3], [64, 256, 512, 1024, 2048], True),
    200: ([3, 24, 36, 3], [64, 256, 512, 1024, 2048], True),
}


class ResidualUnit(nn.Module):
    """BN->ReLU->conv pre-activation unit; the projection shortcut reads act1."""

    def __init__(self, name, cin, cout, stride, dim_match, bottle_neck, bn_mom, bn_global):
        super().__init__()
        self.dim_match, self.bottle_neck = dim_match, bottle_neck
        self.bn1 = BatchNorm(name + '_bn1', cin, momentum=bn_mom, use_global_stats=bn_global)
        if bottle_neck:
            mid = int(cout * 0.25)
            self.conv1 = Conv(name + '_conv1', cin, mid, 1, 1, 0, bias=False)
            self.bn2 = BatchNorm(name + '_bn2', mid, momentum=bn_mom, use_global_stats=bn_global)
            self.conv2 = Conv(name + '_conv2', mid, mid, 3, stride, 1, bias=False)
            self.bn3 = BatchNorm(name + '_bn3', mid, momentum=bn_mom, use_global_stats=bn_global)
            self.conv3 = Conv(name + '_conv3', mid, cout, 1, 1, 0, bias=False)
        else:
            self.conv1 = Conv(name + '_conv1', cin, cout, 3, stride, 1, bias=False)
            self.bn2 = BatchNorm(name + '_bn2', cout, momentum=bn_mom, use_global_stats=bn_global)
            self.conv2 = Conv(name + '_conv2', cout, cout, 3, 1, 1, bias=False)
        if not dim_match:
            self.sc = Conv(name + '_sc', cin, cout, 1, stride, 0, bias=False)

    def forward(self, x):
        act1 = self.bn1(x)
        if self.bottle_neck:
            a, last = self.bn3(self.conv2(self.bn2(self.conv1(act1)))), self.conv3
        else:
            a, last = self.bn2(self.conv1(act1)), self.conv2
        sc = x if self.dim_match else self.sc(act1)
        if fusion_enabled() and igemm_eligible(a, last.weight, last.stride, last.pad) and weight_ok(a, last.weight):
            return conv_add(a, last, sc)  # residual add in the conv epilogue (train-mode BN head units)
        return last(a) + sc

    def can_fuse(self, x):
        """Frozen BNs and MFMA-eligible convs: run the unit as fused conv+BN+ReLU(+residual) ops."""
        if not (fusion_enabled() and _frozen(self.bn1) and _frozen(self.bn2) and
                (not self.bottle_neck or _frozen(self.bn3))):
            return False
        c1 = self.conv1
        return igemm_eligible(x, c1.weight, c1.stride, c1.pad) and weight_ok(x, c1.weight)

    def frozen_bns(self):
        return _frozen(self.bn1) and _frozen(self.bn2) and (not self.bottle_neck or _frozen(self.bn3))

    def unit_op_ok(self, x, next_bn):
        """The whole-unit fused op needs MFMA-eligible 1x1/3x3 shapes (any M) and frozen BNs."""
        if not fusion_enabled() or os.environ.get('MXR_FUSE_UNIT', '1') == '0' or not self.frozen_bns():
            return False
        if not (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and x.is_contiguous(memory_format=torch.channels_last)):
            return False
        # forward-only units with large-M 1x1 convs (frozen stages 1-2) run faster on hipBLASLt
        needs_grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters()))
        from ..ops import precision
        if not needs_grad and not self.can_fuse(x) and not precision.x2_enabled():
            return False
        if next_bn is not None and not (_frozen(next_bn) and next_bn.relu):
            return False
        convs = [self.conv1, self.conv2] + ([self.conv3] if self.bottle_neck else [])
        if not all(weight_ok(x, c.weight) and c.weight.shape[0] % 64 == 0 and c.weight.shape[1] % 64 == 0
                   for c in convs):
            return False
        if not self.dim_match and not (self.sc.weight.shape[0] % 64 == 0 and weight_ok(x, self.sc.weight)):
            return False
        return x.shape[1] % 64 == 0 and x.shape[1] % 8 == 0

    def train_unit_ok(self, x, next_bn):
        """Batch-statistics unit (the RoI head in training): one fused op whose convs produce the
        statistics of their outputs in the epilogue (ops/fused.py _forward_train)."""
        if not fusion_enabled() or os.environ.get('MXR_TRAIN_UNIT', '1') == '0':
            return False
        if any(_frozen(b) for b in ([self.bn1, self.bn2] + ([self.bn3] if self.bottle_neck else []))):
            return False
        if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and
                x.is_contiguous(memory_format=torch.channels_last) and x.shape[1] % 64 == 0):
            return False
        if next_bn is not None and not _train_bn_ok(next_bn):
            return False
        convs = [self.conv1, self.conv2] + ([self.conv3] if self.bottle_neck else [])
        if not self.dim_match:
            convs.append(self.sc)  # the strided 1x1 projection reads act1 directly (no subsampled copy)
        return igemm_eligible(x, self.conv1.weight, self.conv1.stride, self.conv1.pad) and all(
            weight_ok(x, c.weight) and c.weight.shape[0] % 64 == 0 and c.weight.shape[1] % 64 == 0 for c in convs)

    def forward_fused(self, x, act1=None, next_bn=None):
        """-> (unit output, next unit's act1 or None).  act1: this unit's bn1(x) if already
        produced by the previous unit's epilogue."""
        if self.unit_op_ok(x, next_bn):
            return fused_unit(self, x, act1, next_bn)
        if act1 is None:
            act1 = self.bn1(x)
        a = conv_bn_relu(act1, self.conv1, self.bn2)
        if self.bottle_neck:
            c2 = self.conv2
            if igemm_eligible(a, c2.weight, c2.stride, c2.pad):
                a = conv_bn_relu(a, c2, self.bn3)
            else:
                a = self.bn3(c2(a))
            last = self.conv3
        else:
            last = self.conv2
        sc = x if self.dim_match else self.sc(act1)
        if not igemm_eligible(a, last.weight, last.stride, last.pad):
            out = last(a) + sc
            return out, (next_bn(out) if next_bn is not None else None)
        if next_bn is not None and _frozen(next_bn) and next_bn.relu:
            return conv_add_bn_relu(a, last, sc, next_bn)
        out = conv_add(a, last, sc)
        return out, (next_bn(out) if next_bn is not None else None)


def _train_bn_ok(bn):
    return not _frozen(bn) and bn.relu and bn.gamma.shape[0] % 64 == 0


def run_stage_parts(stage, x, tail_bn=None, tail_act=False, act1_in=None):
    """Run a stage (nn.Sequential of ResidualUnit) unit by unit through the fused ops where they
    apply, chaining each unit's last epilogue into the next unit's bn1; units that cannot fuse run
    as plain modules.  Frozen-BN units hand the next unit its bn1 activation; batch-statistics
    units (the RoI head in training) hand it the statistics partials of their output, and the last
    one those of ``tail_bn``'s input -> (x, partials for tail_bn or None).  ``tail_act``: a frozen
    ``tail_bn`` (+ReLU) is applied in the last unit's epilogue as well (the RoI head at test time:
    no separate BN pass over the stage-4 output, or the next stage's first bn1 in the trunk) -> (x,
    None, relu(tail_bn(x)) or None).  ``act1_in``: the first unit's bn1 activation when the previous
    stage's last epilogue produced it."""
    units = list(stage)
    act1, parts, nxt, nbn = act1_in, None, None, None
    for i, u in enumerate(units):
        nxt = units[i + 1] if i + 1 < len(units) else None
        nbn = None
        tbn = nxt.bn1 if nxt is not None else tail_bn
        tbn = tbn if (tbn is not None and fusion_enabled() and _train_bn_ok(tbn)) else None
        if u.train_unit_ok(x, tbn):
            x, parts = fused_unit(u, x, parts, tbn, train=True)
            parts = parts if tbn is not None else None
            act1 = None
            continue
        parts = None
        nbn = nxt.bn1 if (nxt is not None and _frozen(nxt.bn1) and fusion_enabled()) else None
        if nxt is None and tail_act and tail_bn is not None and _frozen(tail_bn) and tail_bn.relu and \
                fusion_enabled():
            nbn = tail_bn
        if u.unit_op_ok(x, nbn) and u.frozen_bns():
            x, act1 = fused_unit(u, x, act1, nbn)
        elif act1 is None and not u.can_fuse(x):
            x, act1 = u(x), None
        else:
            x, act1 = u.forward_fused(x, act1, nbn)
    if tail_act:
        return x, parts, (act1 if (nxt is None and nbn is tail_bn) else None)
    return x, parts


def run_stage(stage, x):
    return run_stage_parts(stage, x)[0]


def _stage(idx, n_units, cin, cout, bottle_neck, bn_mom, bn_global):
    units = []
    stride = 1 if idx == 1 else 2
    units.append(ResidualUnit('stage%d_unit1' % idx, cin, cout, stride, False, bottle_neck, bn_mom, bn_global))
    for j in range(n_units - 1):
        units.append(ResidualUnit('stage%d_unit%d' % (idx, j + 2), cout, cout, 1, True, bottle_neck, bn_mom,
                                  bn_global))
    return nn.Sequential(*units)


def resolve_depth(depth):
    """int depth (18..200) or an explicit (units, filter_list, bottle_neck) spec
    (the reference's generic ``resnet(units, num_stage, filter_list, ...)`` builder)."""
    if isinstance(depth, (tuple, list)):
        units, filters, bottle = depth
        assert len(units) == 4 and len(filters) == 5, 'C4 layout needs 4 stages / 5 filter sizes'
        return list(units), list(filters), bool(bottle)
    return DEPTHS[int(depth)]


class ResNetTrunk(nn.Module):
    """bn_data -> conv0 -> bn0/relu -> maxpool -> stages 1..3 (stride 16)."""
    feat_stride = 16

    def __init__(self, depth=101, bn_mom=0.99, bn_global=True):
        super().__init__()
        units, filters, bottle = resolve_depth(depth)
        self.out_channels = filters[3]
        self.bn_data = BatchNorm('bn_data', 3, momentum=bn_mom, fix_gamma=True, use_global_stats=bn_global,
                                 relu=False)
        self.conv0 = Conv('conv0', 3, filters[0], 7, 2, 3, bias=False)
        self.bn0 = BatchNorm('bn0', filters[0], momentum=bn_mom, use_global_stats=bn_global)
        self.stage1 = _stage(1, units[0], filters[0], filters[1], bottle, bn_mom, bn_global)
        self.stage2 = _stage(2, units[1], filters[1], filters[2], bottle, bn_mom, bn_global)
        self.stage3 = _stage(3, units[2], filters[2], filters[3], bottle, bn_mom, bn_global)

    def _stem_fused(self, x):
        bd, b0 = self.bn_data, self.bn0
        if getattr(bd, '_calibrate', False) or getattr(b0, '_calibrate', False):
            return False
        if self.training and not (bd.use_global_stats and b0.use_global_stats):
            return False
        return stem_fusable(x, self.conv0.weight, bd.gamma, bd.beta, b0.gamma, b0.beta)

    def forward(self, x):
        if self._stem_fused(x):  # one HIP launch (ops/stem.py)
            x = stem_conv(x, self.conv0.weight, 2, 3, in_bn=self.bn_data, out_bn=self.bn0, relu=True)
        else:
            x = self.bn0(self.conv0(self.bn_data(x)))
        u1 = self.stage1[0]
        act = None
        if kernel_path(x) and fusion_enabled() and not u1.dim_match and post_bn_ok(u1.bn1):
            # inference: stage1_unit1's bn1 + ReLU in the max-pool kernel; the projection unit reads
            # only that activation (x stays as the shape carrier)
            x = act = max_pool_bn_relu(x, 3, 2, 1, u1.bn1)
        else:
            x = max_pool(x, 3, 2, 1)
        # each stage's last unit also produces the next stage's first bn1 activation in its epilogue
        # (no separate BN + ReLU pass at the stage boundaries)
        stages = (self.stage1, self.stage2, self.stage3)
        for i, st in enumerate(stages):
            nxt_bn = stages[i + 1][0].bn1 if i + 1 < len(stages) else None
            x, _, act = run_stage_parts(st, x, nxt_bn, tail_act=True, act1_in=act)
        return x

    def feat_shape(self, h, w):
        h, w = (h + 6 - 7) // 2 + 1, (w + 6 - 7) // 2 + 1  # conv0
        h, w = (h + 2 - 3) // 2 + 1, (w + 2 - 3) // 2 + 1  # maxpool
        for _ in range(2):                                   # stage2/3 stride-2 3x3 (pad 1)
            h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        return h, w


class ResNetHead(nn.Module):
    """Stage 4 over pooled RoIs (batch-stat BN) -> bn1 -> relu -> global avg pool -> cls/bbox."""

    def __init__(self, num_classes, depth=101, bn_mom=0.99):
        super().__init__()
        units, filters, bottle = resolve_depth(depth)
        self.stage4 = _stage(4, units[3], filters[3], filters[4], bottle, bn_mom, False)
        self.bn1 = BatchNorm('bn1', filters[4], momentum=bn_mom, use_global_stats=False)
        self.cls_score = Linear('cls_score', filters[4], num_classes)
        self.bbox_pred = Linear('bbox_pred', filters[4], 4 * num_classes)

    def pool_bn(self, feat):
        """stage4_unit1's bn1 when the RoI pooling kernel may apply it (inference on the HIP path:
        16-bit or plane maps, frozen BN, a projection unit that reads only bn1's output) -> the
        BatchNorm or None."""
        u = self.stage4[0]
        return u.bn1 if (kernel_path(feat) and fusion_enabled() and not u.dim_match and post_bn_ok(u.bn1)) else None

    def forward(self, pooled, act1=None):
        """act1: relu(bn1(pooled)) of the first unit when the pooling produced it (pool_bn)."""
        # fused units either way: frozen BNs (test time) or batch statistics (training), where the
        # last unit's conv epilogue also produces bn1's statistics partials
        x, parts, act = run_stage_parts(self.stage4, pooled, self.bn1, tail_act=True, act1_in=act1)
        x = act if act is not None else self.bn1(x, parts=parts)
        x = global_avg_pool(x)
        return fc_pair(x, self.cls_score, self.bbox_pred)
