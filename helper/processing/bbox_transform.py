from mx_rcnn_amd.processing.bbox_transform import *  # noqa: F401,F403
