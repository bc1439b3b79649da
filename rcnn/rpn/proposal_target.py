"""'proposal_target' op (reference `rcnn/rpn/proposal_target.py`)."""
from mx_rcnn_amd.config import config
from mx_rcnn_amd.ops.proposal_target import proposal_target  # noqa: F401


class ProposalTargetOperator(object):
    def __init__(self, num_classes, is_train=False):
        self._num_classes = int(num_classes)
        self._is_train = is_train

    def forward(self, rpn_roi, gt_boxes, n_gt=None):
        """rpn_roi (P, 5) or (B, P, 5); gt_boxes (G, 5) / (B, G, 5) padded with -1 rows."""
        import torch
        if rpn_roi.dim() == 2:
            rpn_roi, gt_boxes = rpn_roi[None], gt_boxes.reshape(1, -1, 5)
        if n_gt is None:
            n_gt = (gt_boxes[..., :5].mean(-1) != -1).sum(-1).to(torch.int32)
        out = proposal_target(rpn_roi, gt_boxes, n_gt, self._num_classes, config, self._is_train)
        return (out['rois'], out['label'], out['bbox_target'], out['bbox_inside_weight'],
                out['bbox_outside_weight'])
