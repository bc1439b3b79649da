from mx_rcnn_amd.processing.generate_anchor import *  # noqa: F401,F403
