from mx_rcnn_amd.processing.nms import *  # noqa: F401,F403
