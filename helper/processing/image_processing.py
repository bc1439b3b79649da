from mx_rcnn_amd.processing.image_processing import *  # noqa: F401,F403
