"""Device operators.  GPU tensors run hand-written gfx950 HIP kernels from
``mx_rcnn_amd/csrc/hip``; CPU tensors run the PyTorch reference implementations."""
from ._ext import ext_available, need_ext  # noqa: F401
from .anchors import base_anchors, all_anchors  # noqa: F401
from .boxes import bbox_transform, bbox_pred, clip_boxes, box_iou, iou_max  # noqa: F401
from .nms import nms, batched_nms  # noqa: F401
from .proposal import proposal  # noqa: F401
from .anchor_target import anchor_target  # noqa: F401
from .proposal_target import proposal_target  # noqa: F401
from .roi_pool import roi_pool, roi_pool_bn_relu  # noqa: F401
from .losses import rpn_softmax_ce, softmax_ce, smooth_l1  # noqa: F401
from .bn import frozen_bn_relu  # noqa: F401
from .sgd import sgd_momentum_  # noqa: F401
