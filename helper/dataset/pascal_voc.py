from mx_rcnn_amd.data.pascal_voc import PascalVOC  # noqa: F401
