from mx_rcnn_amd.processing.bbox_regression import *  # noqa: F401,F403
