#!/bin/bash
# WIDER FACE training on 4 GPUs (reference face.sh called a non-existent train.py).
torchrun --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 train_widerface.py \
  --lr 0.0001 --num_epoch 20 --resume --load-epoch 13 "$@"
