"""The reference-compatible namespace: every public module path / name of
mx-rcnn's rcnn / helper / utils packages imports here, and the graph builders and custom-op
functions behave like the reference's (CPU)."""
import importlib

import pytest
import torch

API = {
    'rcnn.config': ['config'],
    'rcnn.symbol': ['get_vgg_conv', 'get_vgg_rcnn', 'get_vgg_rcnn_test', 'get_vgg_rpn', 'get_vgg_rpn_test',
                    'get_vgg_test', 'get_faster_rcnn'],
    'rcnn.resnet': ['residual_unit', 'rpn', 'resnet', 'resnet_18', 'resnet_34', 'resnet_50', 'resnet_101',
                    'resnet_152', 'resnet_200'],
    'rcnn.rpn.proposal': ['proposal', 'ProposalOperator'],
    'rcnn.rpn.proposal_target': ['proposal_target', 'ProposalTargetOperator'],
    'rcnn.rpn.generate': ['Detector', 'generate_detections', 'vis_detection'],
    'rcnn.loader': ['ROIIter', 'AnchorLoader'],
    'rcnn.minibatch': ['get_minibatch', 'get_image_array', 'sample_rois', 'assign_anchor'],
    'rcnn.module': ['MutableModule'],
    'rcnn.metric': ['AccuracyMetric', 'LogLossMetric', 'SmoothL1LossMetric'],
    'rcnn.callback': ['Speedometer'],
    'rcnn.warmup': ['WarmupScheduler'],
    'rcnn.detector': ['Detector'],
    'rcnn.tester': ['pred_eval', 'vis_all_detection', 'save_all_detection'],
    'helper.processing.bbox_transform': ['bbox_transform', 'bbox_pred', 'clip_boxes', 'clip_pad'],
    'helper.processing.bbox_regression': ['bbox_overlaps', 'compute_bbox_regression_targets',
                                          'expand_bbox_regression_targets'],
    'helper.processing.bbox_process': ['unique_boxes', 'filter_small_boxes'],
    'helper.processing.generate_anchor': ['generate_anchors'],
    'helper.processing.image_processing': ['resize', 'transform', 'transform_inverse', 'tensor_vstack'],
    'helper.processing.nms': ['nms', 'nest'],
    'helper.processing.roidb': ['prepare_roidb', 'add_bbox_regression_targets'],
    'helper.dataset.imdb': ['IMDB'],
    'helper.dataset.pascal_voc': ['PascalVOC'],
    'helper.dataset.detection_list': ['DetectionList'],
    'helper.dataset.voc_eval': ['voc_eval', 'voc_ap', 'parse_voc_rec'],
    'utils.load_model': ['load_checkpoint', 'load_param', 'convert_context'],
    'utils.save_model': ['save_checkpoint'],
    'utils.combine_model': ['combine_model'],
    'utils.load_data': ['load_gt_roidb', 'load_rpn_roidb', 'load_ss_roidb'],
    'utils.caffe_convert': ['load_model'],
}


@pytest.mark.parametrize('mod', sorted(API))
def test_reference_names_import(mod):
    m = importlib.import_module(mod)
    for name in API[mod]:
        assert hasattr(m, name), '%s.%s missing' % (mod, name)


def test_vgg_graph_builders_declare_the_reference_params():
    from rcnn import symbol
    rpn = set(symbol.get_vgg_rpn().arg_params('rpn'))
    rcnn = set(symbol.get_vgg_rcnn().arg_params('rcnn'))
    full = set(symbol.get_vgg_test().arg_params())
    assert 'rpn_conv_3x3_weight' in rpn and 'fc6_weight' not in rpn
    assert 'fc6_weight' in rcnn and 'rpn_conv_3x3_weight' not in rcnn
    assert rpn | rcnn == full
    assert symbol.get_faster_rcnn(num_classes=21).train_mode == 'e2e'
    assert set(symbol.get_vgg_rcnn_test().arg_params('rcnn_test')) == rcnn


def test_resnet_builders():
    from rcnn import resnet
    m = resnet.resnet_50(num_class=21, is_train=True)
    assert m.train_mode == 'e2e' and m.num_anchors == 12
    m = resnet.resnet([3, 4, 23, 3], 4, [64, 256, 512, 1024, 2048], num_class=81)
    names = set(m.arg_params())
    assert 'stage3_unit23_conv3_weight' in names and 'stage3_unit24_conv3_weight' not in names


def test_proposal_and_proposal_target_ops():
    from rcnn.config import config
    from rcnn.rpn.proposal import ProposalOperator
    from rcnn.rpn.proposal_target import ProposalTargetOperator
    g = torch.Generator().manual_seed(0)
    A, H, W = 9, 10, 14
    prob = torch.softmax(torch.randn(1, 2, A * H, W, generator=g), dim=1).reshape(1, 2 * A, H, W)
    deltas = torch.randn(1, 4 * A, H, W, generator=g) * 0.1
    info = torch.tensor([[160.0, 224.0, 1.0]])
    out, score = ProposalOperator(feat_stride=16, is_train=False, output_score=True).forward(prob, deltas, info)
    assert out.shape == (config.TEST.RPN_POST_NMS_TOP_N, 5) and score.shape == (out.shape[0], 1)
    assert torch.all(out[:, 3] <= 223) and torch.all(out[:, 4] <= 159)
    gt = torch.tensor([[10.0, 20.0, 100.0, 120.0, 3.0]])
    roi, label, tgt, iw, ow = ProposalTargetOperator(num_classes=21, is_train=True).forward(out, gt)
    R = config.TRAIN.BATCH_SIZE
    assert roi.shape == (R, 5) and label.shape[0] == R and tgt.shape == (R, 84) == iw.shape == ow.shape
