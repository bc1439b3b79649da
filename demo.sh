#!/bin/bash
# Single-image demo (reference demo.sh; RCNN_SYNC=1 is the NaiveEngine-style synchronous debug mode).
RCNN_SYNC=1 python demo.py --prefix model/final --epoch 0 --image "${1:-data/demo/000001.jpg}"
