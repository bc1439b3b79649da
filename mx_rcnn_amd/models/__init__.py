"""Model families: VGG16 and pre-activation ResNet-18..200 (C4) Faster R-CNN."""
from .faster_rcnn import FasterRCNN, RPNHead, build_model  # noqa: F401
from .resnet import ResNetTrunk, ResNetHead, DEPTHS  # noqa: F401
from .vgg import VGG16Trunk, VGGHead  # noqa: F401
