from mx_rcnn_amd.core.generate import Detector, generate_detections, vis_detection  # noqa: F401
