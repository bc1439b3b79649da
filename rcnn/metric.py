from mx_rcnn_amd.core.metric import AccuracyMetric, LogLossMetric, SmoothL1LossMetric, CompositeEvalMetric, e2e_metrics  # noqa: F401,E501
