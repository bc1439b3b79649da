from mx_rcnn_amd.utils.combine_model import combine_model  # noqa: F401
