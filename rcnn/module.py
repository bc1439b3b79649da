from mx_rcnn_amd.core.module import MutableModule  # noqa: F401
