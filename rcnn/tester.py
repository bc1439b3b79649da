from mx_rcnn_amd.core.tester import pred_eval, vis_all_detection, save_all_detection  # noqa: F401
