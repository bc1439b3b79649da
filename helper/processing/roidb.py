from mx_rcnn_amd.data.roidb import prepare_roidb, add_bbox_regression_targets  # noqa: F401
