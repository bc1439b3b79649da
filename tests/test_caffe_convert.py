"""Caffe .caffemodel reader / converter (utils/caffe_convert.py) against blobs we encode
ourselves (no caffe model ships in the reference: parity with a real file is unpinned)."""
import numpy as np
import pytest

from mx_rcnn_amd.utils import caffe_convert as cc
from mx_rcnn_amd.utils.load_model import load_checkpoint


def _net(rng):
    return [('data', 'Input', []),
            ('conv1_1', 'Convolution', [rng.standard_normal((4, 3, 3, 3)).astype(np.float32),
                                        rng.standard_normal(4).astype(np.float32)]),
            ('relu1_1', 'ReLU', []),
            ('conv1_2', 'Convolution', [rng.standard_normal((4, 4, 3, 3)).astype(np.float32),
                                        rng.standard_normal(4).astype(np.float32)]),
            ('fc6', 'InnerProduct', [rng.standard_normal((8, 4 * 2 * 2)).astype(np.float32),
                                     rng.standard_normal(8).astype(np.float32)]),
            ('cls/score', 'InnerProduct', [rng.standard_normal((3, 8)).astype(np.float32),
                                           rng.standard_normal(3).astype(np.float32)])]


@pytest.mark.parametrize('v1', [False, True])
def test_caffemodel_roundtrip_and_conversion(tmp_path, v1):
    rng = np.random.default_rng(0)
    net = _net(rng)
    types = {'Convolution': 4, 'InnerProduct': 14, 'Input': 5, 'ReLU': 18}
    layers = [(n, types[t] if v1 else t, b) for n, t, b in net]
    path = str(tmp_path / 'm.caffemodel')
    cc.write_caffemodel(path, layers, v1=v1)
    back = cc.read_caffemodel(path)
    assert [n for n, _, _ in back] == [n for n, _, _ in net]
    for (_, _, b0), (_, _, b1) in zip(net, back):
        assert len(b0) == len(b1)
        for x, y in zip(b0, b1):
            np.testing.assert_array_equal(x.reshape(-1), np.asarray(y).reshape(-1))
    shapes = {'conv1_1_weight': (4, 3, 3, 3), 'conv1_1_bias': (4,), 'conv1_2_weight': (4, 4, 3, 3),
              'conv1_2_bias': (4,), 'fc6_weight': (8, 16), 'fc6_bias': (8,)}  # no cls_score: skipped
    arg = cc.load_model(path, str(tmp_path / 'out'), 0, arg_shapes=shapes)
    assert set(arg) == set(shapes)
    np.testing.assert_array_equal(arg['conv1_1_weight'], net[1][2][0][:, ::-1])  # BGR -> RGB
    np.testing.assert_array_equal(arg['conv1_2_weight'], net[3][2][0])  # only the first conv swapped
    np.testing.assert_array_equal(arg['fc6_bias'], net[4][2][1])
    saved, _ = load_checkpoint(str(tmp_path / 'out'), 0)
    assert set(saved) == set(shapes)


def test_slash_names_and_unshaped_conversion():
    rng = np.random.default_rng(1)
    arg = cc.convert_layers(_net(rng))
    assert 'cls_score_weight' in arg and arg['cls_score_weight'].shape == (3, 8)


def test_vgg_test_arg_shapes_cover_the_reference_layers():
    shapes = cc.vgg_test_arg_shapes(21)
    assert shapes['conv1_1_weight'] == (64, 3, 3, 3) and shapes['fc6_weight'] == (4096, 25088)
    assert shapes['cls_score_weight'] == (21, 4096) and shapes['bbox_pred_weight'] == (84, 4096)
