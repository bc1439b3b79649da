"""Dataset / roidb / minibatch / loader tests on synthetic and on-disk fixtures."""
import os

import numpy as np
import pytest

from mx_rcnn_amd.config import config
from mx_rcnn_amd.data import cache as cache_io
from mx_rcnn_amd.data.detection_list import DetectionList
from mx_rcnn_amd.data.load_data import load_synthetic_roidb
from mx_rcnn_amd.data.loader import AnchorLoader, ROIIter, aspect_grouped_order
from mx_rcnn_amd.data.minibatch import sample_rois, assign_anchor
from mx_rcnn_amd.data.pascal_voc import PascalVOC
from mx_rcnn_amd.data.roidb import prepare_roidb, add_bbox_regression_targets
from mx_rcnn_amd.data.voc_eval import voc_ap, voc_eval
from mx_rcnn_amd.processing.image_processing import imwrite

REF_LST = '/root/reference/data/test.lst'


def test_synthetic_roidb_and_anchor_loader():
    imdb, roidb = load_synthetic_roidb(6, 120, 200, 5, flip=True)
    assert len(roidb) == 12 and roidb[6]['flipped']
    w = roidb[0]['width']
    np.testing.assert_array_equal(roidb[6]['boxes'][:, 0], w - roidb[0]['boxes'][:, 2] - 1)
    config.SCALES = (120,)
    config.MAX_SIZE = 200
    ld = AnchorLoader(None, roidb, batch_size=2, shuffle=True, prefetch=2, workers=2)
    n = 0
    for b in ld:
        assert b['data'].shape[:2] == (2, 3) and b['im_info'].shape == (2, 3)
        assert b['gt_boxes'].shape[0] == 2 and b['gt_boxes'].shape[2] == 5
        for k in range(2):
            g = b['gt_boxes'][k, :int(b['n_gt'][k])]
            assert (g[:, 4] > 0).all()
        n += 1
    assert n == 6
    # sharding: 2 ranks see disjoint equal-length shards
    a0 = AnchorLoader(None, roidb, 1, True, rank=0, world_size=2, prefetch=1, workers=1)
    a1 = AnchorLoader(None, roidb, 1, True, rank=1, world_size=2, prefetch=1, workers=1)
    s0 = {int(x[0]) for x in a0._batches}
    s1 = {int(x[0]) for x in a1._batches}
    assert len(a0) == len(a1) == 6 and not (s0 & s1)


def test_aspect_grouping_pairs():
    roidb = [{'width': 10 if i % 3 else 5, 'height': 7} for i in range(10)]
    order = aspect_grouped_order(roidb, np.random.RandomState(0))
    assert sorted(order.tolist()) == list(range(10))
    horz = [roidb[i]['width'] >= roidb[i]['height'] for i in order]
    pairs = [(horz[i], horz[i + 1]) for i in range(0, 10, 2)]
    assert sum(a != b for a, b in pairs) <= 1


def test_sample_rois_and_roiiter():
    imdb, roidb = load_synthetic_roidb(4, 100, 160, 4)
    rng = np.random.RandomState(0)
    for r in roidb:  # add jittered proposals around gt as offline proposals
        props = np.vstack([r['boxes'] + rng.randint(-5, 5, size=r['boxes'].shape) for _ in range(20)])
        props = np.clip(props, 0, 99)
        props[:, 2] = np.maximum(props[:, 2], props[:, 0] + 1)
        props[:, 3] = np.maximum(props[:, 3], props[:, 1] + 1)
        r['box_list'] = props
    rpn_roidb = imdb.create_roidb_from_box_list([r['box_list'] for r in roidb], roidb)
    merged = imdb.merge_roidbs(roidb, rpn_roidb)
    prepare_roidb(imdb, merged)
    means, stds = add_bbox_regression_targets(merged)
    assert means.shape == (16,) and stds.shape == (16,)
    rois, labels, tgt, inw, ov = sample_rois(merged[0], 8, 32, 4)
    assert rois.shape == (32, 4) and tgt.shape == (32, 16)
    nfg = int((labels > 0).sum())
    assert np.all(labels[nfg:] == 0) and np.all(ov[:nfg] >= 0.5)
    config.SCALES = (100,)
    config.MAX_SIZE = 160
    config.TRAIN.BATCH_SIZE = 32
    config.TRAIN.BATCH_IMAGES = 2
    it = ROIIter(merged, batch_size=2, shuffle=True)
    b = next(it)
    assert b['rois'].shape == (32, 5) and b['label'].shape == (32,) and b['bbox_target'].shape == (32, 16)
    assert set(np.unique(b['rois'][:, 0].numpy()).tolist()) <= {0.0, 1.0}
    t = ROIIter(merged, batch_size=1, mode='test')
    tb = next(t)
    assert tb['rois'].shape[1] == 5 and tb['im_info'].shape == (1, 3)


def test_assign_anchor_api():
    out = assign_anchor((1, 512, 10, 14), np.array([[10, 10, 90, 80, 1]], np.float32), [[160, 224, 1.0]])
    assert out['label'].shape == (1, 9 * 10 * 14)
    assert out['bbox_target'].shape == (1, 36, 10, 14)


@pytest.mark.skipif(not os.path.exists(REF_LST), reason='reference list file not mounted')
def test_detection_list_reference_file(tmp_path):
    d = DetectionList('wider_test', REF_LST, str(tmp_path), str(tmp_path))
    assert d.num_classes == 2 and d.classes == ['__background__', 'face'] and d.num_images == 100
    e = d.load_annotation(1)
    assert e['boxes'].shape == (2, 4) and e['boxes'][0].tolist() == [281, 56, 281 + 87 - 1, 56 + 122 - 1]
    roidb = d.gt_roidb()
    assert os.path.exists(os.path.join(str(tmp_path), 'cache', 'wider_test_gt_roidb.npz'))
    again = d.gt_roidb()
    np.testing.assert_array_equal(again[5]['boxes'], roidb[5]['boxes'])


def _make_voc(root):
    dp = os.path.join(root, 'VOCdevkit', 'VOC2007')
    for sub in ('ImageSets/Main', 'Annotations', 'JPEGImages'):
        os.makedirs(os.path.join(dp, sub), exist_ok=True)
    names = ['000001', '000002']
    boxes = {'000001': [('dog', 10, 20, 60, 80, 0), ('person', 30, 5, 50, 40, 1)],
             '000002': [('car', 5, 5, 70, 50, 0)]}
    for n in names:
        objs = ''.join('<object><name>%s</name><difficult>%d</difficult><bndbox><xmin>%d</xmin><ymin>%d</ymin>'
                       '<xmax>%d</xmax><ymax>%d</ymax></bndbox></object>' % (c, d, a, b, x, y)
                       for c, a, b, x, y, d in boxes[n])
        with open(os.path.join(dp, 'Annotations', n + '.xml'), 'w') as f:
            f.write('<annotation>%s</annotation>' % objs)
        imwrite(os.path.join(dp, 'JPEGImages', n + '.jpg'), np.zeros((90, 100, 3), np.uint8))
    with open(os.path.join(dp, 'ImageSets', 'Main', 'test.txt'), 'w') as f:
        f.write('\n'.join(names) + '\n')
    return os.path.join(root, 'VOCdevkit'), boxes


def test_pascal_voc_roundtrip_and_map(tmp_path):
    devkit, boxes = _make_voc(str(tmp_path))
    voc = PascalVOC('test', '2007', str(tmp_path), devkit)
    roidb = voc.gt_roidb()
    assert roidb[0]['boxes'].tolist() == [[9, 19, 59, 79]]  # difficult excluded, 0-based
    assert voc.image_size_from_index('000001') == (90, 100)
    # perfect detections -> AP 1 for present classes
    dets = [[np.zeros((0, 5)) for _ in range(2)] for _ in range(21)]
    dets[voc.classes.index('dog')][0] = np.array([[9, 19, 59, 79, 0.9]])
    dets[voc.classes.index('car')][1] = np.array([[4, 4, 69, 49, 0.8]])
    voc.evaluate_detections(dets)
    f = voc.get_result_file_template().format('dog')
    rec, prec, ap = voc_eval(f, os.path.join(voc.data_path, 'Annotations', '{0!s}.xml'),
                             os.path.join(voc.data_path, 'ImageSets', 'Main', 'test.txt'), 'dog',
                             str(tmp_path / 'c'), 0.5, True)
    assert ap == pytest.approx(1.0)
    cache_io.save_box_list(str(tmp_path / 'props.npz'), [np.ones((3, 4)), np.zeros((0, 4))])
    bl = cache_io.load_box_list(str(tmp_path / 'props.npz'))
    assert bl[0].shape == (3, 4) and bl[1].shape == (0, 4)


def test_voc_ap_fixed_branch():
    rec = np.array([0.5, 1.0])
    prec = np.array([1.0, 0.5])
    assert voc_ap(rec, prec, False) == pytest.approx(0.75)
    assert voc_ap(rec, prec, True) == pytest.approx((6 * 1.0 + 5 * 0.5) / 11)


def test_split_input_slice_and_work_load_list():
    from mx_rcnn_amd.data.loader import split_input_slice
    assert split_input_slice(4, [1, 1]) == [(0, 2), (2, 4)]
    assert split_input_slice(6, [1, 2]) == [(0, 2), (2, 6)]
    assert split_input_slice(5, [1, 1, 1]) == [(0, 2), (2, 4), (4, 5)]
    with pytest.raises(ValueError):
        split_input_slice(2, [1, 1, 1])
    imdb, roidb = load_synthetic_roidb(12, 96, 128, 4)
    config.SCALES = (96,)
    config.MAX_SIZE = 128
    # global batch 2 x 2 = 4 images split 1:3 between the ranks; same steps on every rank
    r0 = AnchorLoader(None, roidb, 2, True, rank=0, world_size=2, work_load_list='1,3', prefetch=1, workers=1)
    r1 = AnchorLoader(None, roidb, 2, True, rank=1, world_size=2, work_load_list=[1, 3], prefetch=1, workers=1)
    assert len(r0) == len(r1) == 3
    assert all(len(b) == 1 for b in r0._batches) and all(len(b) == 3 for b in r1._batches)
    for b0, b1, g in zip(r0._batches, r1._batches, r0._global):
        assert list(b0) + list(b1) == list(g)


def test_dp_loaders_agree_on_step_shape():
    """Every rank pads its batch to the global step's (bucketed) shape and gt count, computed
    from roidb metadata without communication, so all ranks reach each hipGraph capture on the
    same step (reference: AnchorLoader pads across devices, rcnn/loader.py:283-286)."""
    rng = np.random.RandomState(3)
    imdb, roidb = load_synthetic_roidb(16, 96, 128, 4)
    for k, r in enumerate(roidb):  # mixed sizes and gt counts
        r['height'], r['width'] = int(rng.randint(80, 200)), int(rng.randint(80, 200))
        n = int(rng.randint(1, 6))
        r['boxes'] = np.tile(np.array([[2, 2, 40, 40]], np.uint16), (n, 1))
        r['gt_classes'] = np.ones(n, np.int32)
        r['synthetic_seed'] = k
    config.SCALES = (100, 120)
    config.MAX_SIZE = 180
    ld = [AnchorLoader(None, roidb, 1, True, rank=r, world_size=2, prefetch=1, workers=1) for r in range(2)]
    shapes = []
    for b0, b1 in zip(ld[0], ld[1]):
        assert b0['data'].shape == b1['data'].shape and b0['gt_boxes'].shape == b1['gt_boxes'].shape
        assert b0['data'].shape[2] % 64 == 0 and b0['data'].shape[3] % 64 == 0
        G = b0['gt_boxes'].shape[1]
        assert G >= 8 and (G & (G - 1)) == 0
        for b in (b0, b1):  # the real image sits inside the padding
            h, w = b['im_info'][0, :2].tolist()
            assert h <= b['data'].shape[2] and w <= b['data'].shape[3]
        shapes.append(tuple(b0['data'].shape))
    assert len(shapes) == 8
    config.SCALES = (600,)
    config.MAX_SIZE = 1000


def _greedy_loop(ov):
    """Repeated global-argmax matching (oracle for the pair-sorted version)."""
    ov = ov.copy()
    out = np.zeros(ov.shape[1])
    for _ in range(min(ov.shape)):
        b, g = np.unravel_index(np.argmax(ov), ov.shape)
        out[g] = ov[b, g]
        ov[b, :] = -1
        ov[:, g] = -1
    return out


def test_evaluate_recall_greedy_matching():
    import scipy.sparse
    from mx_rcnn_amd.data.imdb import IMDB
    rng = np.random.RandomState(9)
    for _ in range(20):
        ov = rng.rand(rng.randint(1, 12), rng.randint(1, 6))
        np.testing.assert_allclose(np.sort(IMDB.greedy_gt_coverage(ov)), np.sort(_greedy_loop(ov)))
    # toy image: 2 gts, proposals hitting one exactly and the other at IoU 0.8
    gt = np.array([[0, 0, 9, 9], [20, 20, 39, 39]], np.float32)
    props = np.array([[0, 0, 9, 9], [20, 20, 35, 39], [50, 50, 60, 60]], np.float32)
    boxes = np.vstack([gt, props])
    ovl = np.zeros((5, 2), np.float32)
    ovl[0, 1] = ovl[1, 1] = 1.0
    roidb = [{'boxes': boxes, 'gt_classes': np.array([1, 1, 0, 0, 0], np.int32),
              'gt_overlaps': scipy.sparse.csr_matrix(ovl)}]
    ar, rec, th = IMDB('t').evaluate_recall(roidb, thresholds=[0.5, 0.7, 0.9])
    np.testing.assert_allclose(rec, [1.0, 1.0, 0.5])  # IoU 1.0 and 0.8
    ar, rec, th = IMDB('t').evaluate_recall(roidb, thresholds=[0.5], area='large')
    assert rec[0] == 0.0  # no gt of area >= 96^2
