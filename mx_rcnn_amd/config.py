"""Global detection configuration.

Same key names and defaults as the reference's process-global EasyDict
(`rcnn/config.py:1-70` of walkoncross/mx-rcnn), so scripts written against
`from rcnn.config import config` keep working.  Additions over the reference:

* ``AttrDict`` replaces the external ``easydict`` dependency.
* ``snapshot()`` / ``restore()`` give an immutable per-run copy, so the
  import-time / run-time mutation the reference relies on
  (`train_end2end.py:25-38`, `tools/train_rpn.py:16-18`) can be scoped.
* ``override({'TRAIN.RPN_MIN_SIZE': 10})`` and ``parse_cfg_overrides`` back
  the ``--cfg key=value`` CLI flag.
* ``ims_per_gpu`` knobs for batched proposal / target kernels (the reference
  hard-fails on more than one image per device, `rcnn/rpn/proposal.py:194`).
"""
import ast
import copy

import numpy as np


class AttrDict(dict):
    """dict with attribute access (recursive), the subset of EasyDict we need."""

    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError:
            raise AttributeError(name)

    def __setattr__(self, name, value):
        if isinstance(value, dict) and not isinstance(value, AttrDict):
            value = AttrDict(value)
        self[name] = value

    def __delattr__(self, name):
        del self[name]

    def __deepcopy__(self, memo):
        out = AttrDict()
        for k, v in self.items():
            dict.__setitem__(out, k, copy.deepcopy(v, memo))
        return out


def _default_config():
    c = AttrDict()
    # image processing config (rcnn/config.py:7-10)
    c.EPS = 1e-14
    c.PIXEL_MEANS = np.array([[[123.68, 116.779, 103.939]]])
    c.SCALES = (600,)
    c.MAX_SIZE = 1000
    # nms config (dead in the reference, kept for API parity; rcnn/config.py:13-14)
    c.USE_GPU_NMS = True
    c.GPU_ID = 0

    c.TRAIN = AttrDict()
    c.TRAIN.FINETUNE = False
    c.TRAIN.BATCH_SIZE = 128
    # R-CNN
    c.TRAIN.HAS_RPN = False
    c.TRAIN.ASPECT_GROUPING = True
    c.TRAIN.BATCH_IMAGES = 2
    c.TRAIN.FG_FRACTION = 0.25
    c.TRAIN.FG_THRESH = 0.5
    c.TRAIN.BG_THRESH_HI = 0.5
    c.TRAIN.BG_THRESH_LO = 0.1
    # R-CNN bounding box regression
    c.TRAIN.BBOX_REGRESSION_THRESH = 0.5
    c.TRAIN.BBOX_INSIDE_WEIGHTS = np.array([1.0, 1.0, 1.0, 1.0])
    # RPN anchor loader
    c.TRAIN.RPN_BATCH_SIZE = 256
    c.TRAIN.RPN_FG_FRACTION = 0.5
    c.TRAIN.RPN_POSITIVE_OVERLAP = 0.7
    c.TRAIN.RPN_NEGATIVE_OVERLAP = 0.3
    c.TRAIN.RPN_CLOBBER_POSITIVES = False
    c.TRAIN.RPN_BBOX_INSIDE_WEIGHTS = (1.0, 1.0, 1.0, 1.0)
    c.TRAIN.RPN_POSITIVE_WEIGHT = -1.0
    # end2end RPN proposal
    c.END2END = 0
    c.TRAIN.RPN_NMS_THRESH = 0.7
    c.TRAIN.RPN_PRE_NMS_TOP_N = 12000
    c.TRAIN.RPN_POST_NMS_TOP_N = 6000
    c.TRAIN.RPN_MIN_SIZE = 16
    # approximate bounding box regression
    c.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = False
    c.TRAIN.BBOX_MEANS = (0.0, 0.0, 0.0, 0.0)
    c.TRAIN.BBOX_STDS = (0.1, 0.1, 0.2, 0.2)
    c.TRAIN.BBOX_MEANS_INV = (0.0, 0.0, 0.0, 0.0)
    c.TRAIN.BBOX_STDS_INV = (10.0, 10.0, 5.0, 5.0)
    c.TRAIN.IMS_PER_BATCH = 1

    c.TEST = AttrDict()
    c.TEST.HAS_RPN = False
    c.TEST.BATCH_IMAGES = 1
    c.TEST.NMS = 0.3
    c.TEST.DEDUP_BOXES = 1.0 / 16.0
    c.TEST.RPN_NMS_THRESH = 0.7
    c.TEST.RPN_PRE_NMS_TOP_N = 6000
    c.TEST.RPN_POST_NMS_TOP_N = 300
    c.TEST.RPN_MIN_SIZE = 16
    return c


config = _default_config()


def snapshot():
    """Deep copy of the current global config (an immutable per-run view)."""
    return copy.deepcopy(config)


def restore(snap):
    """Restore the global config in place from a snapshot (keeps identity)."""
    config.clear()
    for k, v in copy.deepcopy(snap).items():
        dict.__setitem__(config, k, v)


def reset():
    """Reset the global config to the reference defaults."""
    restore(_default_config())


def _parse_value(text):
    try:
        return ast.literal_eval(text)
    except (ValueError, SyntaxError):
        return text


def override(updates, cfg=None):
    """Apply ``{'TRAIN.RPN_MIN_SIZE': 10, 'SCALES': (640,)}`` style updates."""
    cfg = config if cfg is None else cfg
    for key, value in updates.items():
        node = cfg
        parts = key.split('.')
        for p in parts[:-1]:
            if p not in node:
                raise KeyError('unknown config section %r in %r' % (p, key))
            node = node[p]
        if parts[-1] not in node:
            raise KeyError('unknown config key %r' % key)
        old = node[parts[-1]]
        if isinstance(value, str):
            value = _parse_value(value)
        if isinstance(old, np.ndarray):
            value = np.array(value, dtype=old.dtype)
        node[parts[-1]] = value
    return cfg


def parse_cfg_overrides(items):
    """Turn ``['TRAIN.RPN_MIN_SIZE=10', ...]`` (the ``--cfg`` flag) into a dict."""
    out = {}
    for item in items or []:
        if '=' not in item:
            raise ValueError('--cfg expects key=value, got %r' % item)
        k, v = item.split('=', 1)
        out[k.strip()] = v.strip()
    return out
