#!/bin/bash
# BASELINE config 4 end to end on one GPU at the reference precision (fp32): RPN1 -> proposal dump at
# PRE_NMS_TOP_N = -1 (every anchor) -> RCNN1 -> RPN2 -> dump -> combine -> RCNN2 -> combine; the
# final checkpoint round-trips through load_param.  ResNet-50, synthetic 600x1000 images.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/alt4; export TMPDIR=/tmp
W="$PWD/gpurun_out/alt4"
timeout -k 10 900 python -u train_alternate.py --network resnet50 --synthetic 64 --synthetic-shape 600x1000 \
  --rpn_epoch 1 --rcnn_epoch 1 --frequent 16 --dtype fp32 --pretrained none --model-dir "$W/model" \
  --root_path "$W" > "$W/alt4.log" 2>&1 || { tail -30 "$W/alt4.log"; exit 1; }
grep -E "######|Speed|samples/sec|recall|Epoch\[0\] Time" "$W/alt4.log" | cut -c1-200 | tail -40
timeout -k 10 120 python - <<'PY'
import os
from mx_rcnn_amd.utils.load_model import load_param
W = os.path.join(os.environ.get('GRAFT_REPO_ROOT', '.'), 'gpurun_out/alt4/model')
arg, aux = load_param(os.path.join(W, 'final'), 0, convert=True)[:2]
print('final-0000.params: %d arg arrays, %d aux arrays, %d elements' % (len(arg), len(aux), sum(int(__import__("numpy").asarray(v).size) for v in arg.values())))
PY
rm -rf "$W/model" "$W/rpn_data"
