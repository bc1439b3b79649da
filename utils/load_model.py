from mx_rcnn_amd.utils.load_model import load_checkpoint, load_param, do_checkpoint, convert_context  # noqa: F401,E501
