from mx_rcnn_amd.utils.load_model import save_checkpoint  # noqa: F401
