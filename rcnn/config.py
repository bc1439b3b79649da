from mx_rcnn_amd.config import config, snapshot, restore, reset, override, parse_cfg_overrides  # noqa: F401
