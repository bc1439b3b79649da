"""VGG16 trunk and Fast R-CNN head (reference `rcnn/symbol.py:6-119`).

13 conv3x3+ReLU layers, 4 max-pool 2x2/2 (floor), stride-16 relu5_3 (512 ch); the head is
RoIPool 7x7 @ 1/16 -> fc6 4096 -> ReLU -> Dropout .5 -> fc7 -> ReLU -> Dropout -> cls/bbox.
"""
import torch
import torch.nn as nn

from .layers import Conv, Linear, max_pool
from ..ops.head import fc_pair
from ..ops.stem import stem_fusable, stem_conv
from ..ops import vgg_fused

VGG_CFG = [(1, 2, 3, 64), (2, 2, 64, 128), (3, 3, 128, 256), (4, 3, 256, 512), (5, 3, 512, 512)]


class VGG16Trunk(nn.Module):
    out_channels = 512
    feat_stride = 16

    def __init__(self):
        super().__init__()
        self.convs = nn.ModuleList()
        self.pool_after = []
        for g, n, cin, cout in VGG_CFG:
            for i in range(1, n + 1):
                self.convs.append(Conv('conv%d_%d' % (g, i), cin if i == 1 else cout, cout, 3, 1, 1))
            self.pool_after.append(len(self.convs) - 1 if g < 5 else -1)

    def forward(self, x):
        if vgg_fused.trunk_ok(x, self.convs):  # one autograd node, ReLU backward in the dgrad epilogues
            return vgg_fused.vgg_trunk(x, self.convs, self.pool_after)
        for i, c in enumerate(self.convs):
            if i == 0 and stem_fusable(x, c.weight, c.bias):  # one HIP launch (ops/stem.py)
                x = stem_conv(x, c.weight, 1, 1, bias=c.bias, relu=True)
            else:
                x = c(x, relu=True)
            if i in self.pool_after:
                x = max_pool(x, 2, 2)
        return x

    def feat_shape(self, h, w):
        for _ in range(4):
            h, w = h // 2, w // 2
        return h, w


class VGGHead(nn.Module):
    """fc6/fc7 (+dropout) and the cls/bbox predictors on 7x7x512 pooled RoIs."""

    def __init__(self, num_classes, in_channels=512, pooled=7, dropout=0.5):
        super().__init__()
        self.fc6 = Linear('fc6', in_channels * pooled * pooled, 4096, in_shape=(in_channels, pooled, pooled))
        self.fc7 = Linear('fc7', 4096, 4096)
        self.cls_score = Linear('cls_score', 4096, num_classes)
        self.bbox_pred = Linear('bbox_pred', 4096, 4 * num_classes)
        self.dropout = dropout

    def forward(self, pooled):
        if pooled.is_cuda and pooled.dim() == 4 and pooled.is_contiguous(memory_format=torch.channels_last):
            # the pooled map's channels_last rows, (h, w, c) order: a free view, matching fc6's
            # channels_last filter (Linear in_shape) -- no Flatten copy forward or backward
            rows = pooled.permute(0, 2, 3, 1).reshape(pooled.shape[0], -1)
            if vgg_fused.head_ok(rows, self):
                return vgg_fused.vgg_head(rows, self)
        x = pooled.reshape(pooled.shape[0], -1)  # MXNet Flatten: (C, H, W) order
        # relu6/drop6 and relu7/drop7 run in the FC kernel's epilogue (ops/fc.py)
        x = self.fc6(x, relu=True, drop_p=self.dropout)
        x = self.fc7(x, relu=True, drop_p=self.dropout)
        return fc_pair(x, self.cls_score, self.bbox_pred)
