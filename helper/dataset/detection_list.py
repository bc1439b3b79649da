from mx_rcnn_amd.data.detection_list import DetectionList  # noqa: F401
