"""MXNet .params codec round trip, legacy/V1 records, fold/unfold, combine_model, trainer
state export/import."""
import struct

import numpy as np
import torch

from mx_rcnn_amd.config import snapshot
from mx_rcnn_amd.utils import ndarray_io
from mx_rcnn_amd.utils.load_model import (save_checkpoint, load_checkpoint, load_param, fold_bbox_pred,
                                          unfold_bbox_pred, do_checkpoint)
from mx_rcnn_amd.utils.combine_model import combine_model


def test_roundtrip_v2(tmp_path):
    d = {'arg:w': np.arange(12, dtype=np.float32).reshape(3, 4), 'aux:m': np.ones(5, np.float64),
         'arg:i': np.array([1, 2, 3], np.int32), 'arg:h': np.zeros((2, 2), np.float16),
         'arg:t': torch.arange(6).float().reshape(2, 3)}
    f = str(tmp_path / 'x-0001.params')
    ndarray_io.save(f, d)
    out = ndarray_io.load(f)
    assert set(out) == set(d)
    np.testing.assert_array_equal(out['arg:w'], d['arg:w'])
    assert out['aux:m'].dtype == np.float64 and out['arg:i'].dtype == np.int32
    np.testing.assert_array_equal(out['arg:t'], d['arg:t'].numpy())
    # header layout
    raw = open(f, 'rb').read()
    assert struct.unpack_from('<QQQ', raw, 0) == (0x112, 0, 5)
    assert struct.unpack_from('<I', raw, 24)[0] == 0xF993FAC9


def _legacy_bytes(arr, magic=None):
    out = b''
    if magic is not None:
        out += struct.pack('<I', magic)
    out += struct.pack('<I', arr.ndim) + struct.pack('<%dI' % arr.ndim, *arr.shape)
    out += struct.pack('<iii', 1, 0, 0) + arr.astype('<f4').tobytes()
    return out


def test_reads_v1_and_legacy(tmp_path):
    a = np.random.RandomState(0).rand(2, 3).astype(np.float32)
    b = np.random.RandomState(1).rand(4).astype(np.float32)
    body = struct.pack('<QQQ', 0x112, 0, 2) + _legacy_bytes(a, 0xF993FAC8) + _legacy_bytes(b)
    body += struct.pack('<Q', 2)
    for n in (b'arg:a', b'aux:b'):
        body += struct.pack('<Q', len(n)) + n
    f = tmp_path / 'old-0000.params'
    f.write_bytes(body)
    out = ndarray_io.load(str(f))
    np.testing.assert_array_equal(out['arg:a'], a)
    np.testing.assert_array_equal(out['aux:b'], b)


def test_fold_unfold_inverse():
    cfg = snapshot()
    rng = np.random.RandomState(2)
    arg = {'bbox_pred_weight': rng.rand(84, 16).astype(np.float32), 'bbox_pred_bias': rng.rand(84).astype(np.float32)}
    back = unfold_bbox_pred(fold_bbox_pred(arg, cfg=cfg), cfg=cfg)
    np.testing.assert_allclose(back['bbox_pred_weight'], arg['bbox_pred_weight'], rtol=1e-5)
    np.testing.assert_allclose(back['bbox_pred_bias'], arg['bbox_pred_bias'], rtol=1e-5, atol=1e-6)
    f = fold_bbox_pred(arg, cfg=cfg)
    np.testing.assert_allclose(f['bbox_pred_weight'][2], arg['bbox_pred_weight'][2] * 0.2, rtol=1e-6)


def test_checkpoint_load_param_and_combine(tmp_path):
    cfg = snapshot()
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    from mx_rcnn_amd import config as cm
    cm.restore(cfg)
    arg = {'conv_weight': np.ones((2, 2), np.float32), 'bbox_pred_weight': np.ones((8, 3), np.float32),
           'bbox_pred_bias': np.zeros(8, np.float32)}
    aux = {'bn_moving_mean': np.zeros(3, np.float32)}
    cb = do_checkpoint(str(tmp_path / 'm'))
    cb(0, None, arg, aux)
    a2, x2, nc = load_param(str(tmp_path / 'm'), 1)
    assert nc == 2
    np.testing.assert_allclose(a2['bbox_pred_weight'], arg['bbox_pred_weight'], rtol=1e-5)
    save_checkpoint(str(tmp_path / 'n'), 3, {'conv_weight': np.zeros((2, 2), np.float32), 'x': np.ones(1)}, {})
    args, auxs = combine_model(str(tmp_path / 'm'), 1, str(tmp_path / 'n'), 3, str(tmp_path / 'c'), 0)
    c_arg, c_aux = load_checkpoint(str(tmp_path / 'c'), 0)
    assert np.all(c_arg['conv_weight'] == 1) and 'x' in c_arg and 'bn_moving_mean' in c_aux
