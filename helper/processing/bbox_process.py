from mx_rcnn_amd.processing.bbox_process import *  # noqa: F401,F403
