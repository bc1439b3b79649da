#!/usr/bin/env python
"""WIDER FACE training with ResNet-18 (reference `train_widerface_resnet18.py`)."""
import train_widerface

if __name__ == '__main__':
    train_widerface.main(train_widerface.parse_args(default_network='resnet18'), default_network='resnet18')
