from mx_rcnn_amd.utils.caffe_convert import load_model  # noqa: F401
