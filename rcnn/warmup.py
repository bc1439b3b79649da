from mx_rcnn_amd.core.lr_scheduler import WarmupScheduler, FactorScheduler  # noqa: F401
