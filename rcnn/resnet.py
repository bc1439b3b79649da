"""Pre-activation ResNet C4 builders (reference `rcnn/resnet.py:5-223`)."""
from mx_rcnn_amd.models import FasterRCNN, RPNHead
from mx_rcnn_amd.models.resnet import ResidualUnit


def residual_unit(data=None, num_filter=256, stride=(1, 1), dim_match=True, name='unit', bottle_neck=True,
                  bn_mom=0.9, workspace=512, bn_global=True, in_channels=None):
    s = stride[0] if isinstance(stride, (tuple, list)) else stride
    cin = in_channels if in_channels is not None else num_filter
    return ResidualUnit(name, cin, num_filter, s, dim_match, bottle_neck, bn_mom, bn_global)


def rpn(data=None, num_class=2, num_anchor=12, is_train=False, in_channels=1024):
    return RPNHead(in_channels, num_anchor)


def resnet(units, num_stage, filter_list, num_class=2, num_anchor=12, bottle_neck=True, bn_mom=0.9,
           bn_global=True, workspace=512, is_train=False):
    assert num_stage == 4 == len(units)
    return FasterRCNN('resnet', num_class, bn_mom=bn_mom, num_anchors=num_anchor,
                      resnet_spec=(units, filter_list, bottle_neck), train_mode='e2e' if is_train else 'test')


def _mk(depth):
    def f(num_class=2, bn_mom=0.99, bn_global=True, is_train=False):
        return FasterRCNN('resnet%d' % depth, num_class, bn_mom=bn_mom, train_mode='e2e' if is_train else 'test')
    f.__name__ = 'resnet_%d' % depth
    return f


resnet_18, resnet_34, resnet_50 = _mk(18), _mk(34), _mk(50)
resnet_101, resnet_152, resnet_200 = _mk(101), _mk(152), _mk(200)
