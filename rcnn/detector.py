from mx_rcnn_amd.core.detector import Detector  # noqa: F401
