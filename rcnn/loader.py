from mx_rcnn_amd.data.loader import AnchorLoader, ROIIter  # noqa: F401
