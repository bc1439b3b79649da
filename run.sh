#!/bin/bash
# End-to-end VOC training on 2 GPUs (reference run.sh): one process per GPU over RCCL.
torchrun --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 train_end2end.py \
  --image_set 2007_trainval --lr 0.001 --factor-step 20000 --num_epoch 10 --prefix model/e2e "$@"
