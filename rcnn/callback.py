from mx_rcnn_amd.core.callback import Speedometer, BatchEndParam  # noqa: F401
