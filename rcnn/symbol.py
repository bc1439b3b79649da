"""VGG16 graph builders (reference `rcnn/symbol.py`).  Each returns a FasterRCNN model whose
``train_mode`` selects the graph the reference symbol represented."""
from mx_rcnn_amd.models import FasterRCNN
from mx_rcnn_amd.models.vgg import VGG16Trunk


def get_vgg_conv(data=None):
    return VGG16Trunk()


def get_vgg_rcnn(num_classes=21):
    return FasterRCNN('vgg16', num_classes, train_mode='rcnn')


def get_vgg_rcnn_test(num_classes=21):
    return FasterRCNN('vgg16', num_classes, train_mode='rcnn_test')


def get_vgg_rpn(num_classes=21, num_anchors=9):
    return FasterRCNN('vgg16', num_classes, num_anchors=num_anchors, train_mode='rpn')


def get_vgg_rpn_test(num_classes=21, num_anchors=9):
    return FasterRCNN('vgg16', num_classes, num_anchors=num_anchors, train_mode='rpn_test')


def get_vgg_test(num_classes=21, num_anchors=9):
    return FasterRCNN('vgg16', num_classes, num_anchors=num_anchors, train_mode='test')


def get_faster_rcnn(num_classes=21, num_anchors=9):
    return FasterRCNN('vgg16', num_classes, num_anchors=num_anchors, train_mode='e2e')
