from mx_rcnn_amd.data.minibatch import get_minibatch, get_image_array, sample_rois, assign_anchor  # noqa: F401
