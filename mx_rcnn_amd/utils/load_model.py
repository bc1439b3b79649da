"""Checkpoint load/save with the reference's layout and bbox-normalisation fold
(`utils/load_model.py:6-94`, `utils/save_model.py:4-18`).

``<prefix>-%04d.params`` holds ``arg:<name>`` / ``aux:<name>`` arrays.  When
``TRAIN.BBOX_NORMALIZATION_PRECOMPUTED`` is set, saved ``bbox_pred`` weights are folded
into pixel-delta space (W <- diag(stds) W, b <- b*stds + means) and unfolded on load with
the *_INV constants.  ``load_param`` returns 3 values (arg, aux, num_classes) -- the
reference's own tools unpack 2 and crash; every caller here uses 3.
Optional sidecar ``<prefix>-%04d.states`` (momentum, update count, RNG) enables exact resume.
"""
import logging
import os

import numpy as np

from ..config import config
from . import ndarray_io


def params_file(prefix, epoch):
    return '%s-%04d.params' % (prefix, epoch)


def load_checkpoint(prefix, epoch):
    save_dict = ndarray_io.load(params_file(prefix, epoch))
    arg_params, aux_params = {}, {}
    for k, v in save_dict.items():
        tp, name = k.split(':', 1)
        if tp == 'arg':
            arg_params[name] = v
        elif tp == 'aux':
            aux_params[name] = v
    return arg_params, aux_params


def save_checkpoint(prefix, epoch, arg_params, aux_params):
    d = {'arg:%s' % k: v for k, v in arg_params.items()}
    d.update({'aux:%s' % k: v for k, v in aux_params.items()})
    os.makedirs(os.path.dirname(os.path.abspath(params_file(prefix, epoch))), exist_ok=True)
    ndarray_io.save(params_file(prefix, epoch), d)


def _np(v):
    return ndarray_io._to_numpy(v).astype(np.float32)


def fold_bbox_pred(arg, means=None, stds=None, cfg=None):
    """Fold target normalisation into bbox_pred (save direction)."""
    cfg = cfg or config
    if 'bbox_pred_bias' not in arg:
        return arg
    arg = dict(arg)
    nc = _np(arg['bbox_pred_bias']).size // 4
    means = np.array(cfg.TRAIN.BBOX_MEANS if means is None else means, dtype=np.float32).ravel()
    stds = np.array(cfg.TRAIN.BBOX_STDS if stds is None else stds, dtype=np.float32).ravel()
    if means.size == 4:
        means = np.tile(means, nc)
    if stds.size == 4:
        stds = np.tile(stds, nc)
    arg['bbox_pred_weight'] = _np(arg['bbox_pred_weight']) * stds[:, None]
    arg['bbox_pred_bias'] = _np(arg['bbox_pred_bias']) * stds + means
    return arg


def unfold_bbox_pred(arg, cfg=None):
    """Inverse fold (load direction) with BBOX_MEANS_INV / BBOX_STDS_INV."""
    cfg = cfg or config
    if 'bbox_pred_bias' not in arg:
        return arg
    arg = dict(arg)
    nc = _np(arg['bbox_pred_bias']).size // 4
    means = np.tile(np.array(cfg.TRAIN.BBOX_MEANS_INV, dtype=np.float32), nc)
    stds = np.tile(np.array(cfg.TRAIN.BBOX_STDS_INV, dtype=np.float32), nc)
    arg['bbox_pred_weight'] = _np(arg['bbox_pred_weight']) * stds[:, None]
    arg['bbox_pred_bias'] = (_np(arg['bbox_pred_bias']) - means) * stds
    return arg


def convert_context(params, ctx):
    """Move every array to a torch device (the reference's NDArray.as_in_context)."""
    import torch
    return {k: torch.as_tensor(np.asarray(v)).to(ctx) for k, v in params.items()}


def load_param(prefix, epoch, convert=False, ctx=None, cfg=None):
    """-> (arg_params, aux_params, num_classes); num_classes = len(bbox_pred_bias)/4 or 1000."""
    cfg = cfg or config
    arg_params, aux_params = load_checkpoint(prefix, epoch)
    num_classes = 1000
    if 'bbox_pred_bias' in arg_params:
        num_classes = int(np.asarray(arg_params['bbox_pred_bias']).size // 4)
        if cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED:
            logging.info('load model with mean/std (unfold bbox_pred)')
            arg_params = unfold_bbox_pred(arg_params, cfg)
    if convert:
        ctx = ctx if ctx is not None else 'cpu'
        arg_params = convert_context(arg_params, ctx)
        aux_params = convert_context(aux_params, ctx)
    return arg_params, aux_params, num_classes


def do_checkpoint(prefix, cfg=None, means=None, stds=None):
    """Epoch-end callback ``cb(iter_no, model_or_arg, arg, aux)`` saving ``prefix-(iter_no+1)``."""
    def _callback(iter_no, sym, arg, aux):
        c = cfg or config
        a = dict(arg)
        if c.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED or means is not None:
            a = fold_bbox_pred(a, means, stds, c)
        save_checkpoint(prefix, iter_no + 1, a, aux)
        logging.info('Saved checkpoint to "%s"', params_file(prefix, iter_no + 1))
    return _callback


def save_states(prefix, epoch, states):
    """Optimizer/momentum sidecar for exact resume."""
    ndarray_io.save('%s-%04d.states' % (prefix, epoch), states)


def states_file(prefix, epoch):
    """Path of the optimizer-state sidecar if it exists, else None."""
    path = '%s-%04d.states' % (prefix, epoch)
    return path if os.path.exists(path) else None


def load_states(prefix, epoch):
    path = '%s-%04d.states' % (prefix, epoch)
    return ndarray_io.load(path) if os.path.exists(path) else None
