from mx_rcnn_amd.data.load_data import *  # noqa: F401,F403
