from mx_rcnn_amd.data.voc_eval import voc_eval, voc_ap, parse_voc_rec  # noqa: F401
