#!/bin/bash
# The CLI entry points on one MI355X with synthetic data: 4-step alternate training (ResNet-50,
# BASELINE config 4 at N=1: exercises the proposal dump / load path), end2end training with a
# checkpoint, then test.py evaluation of that checkpoint.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/cli; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
W=$(mktemp -d)
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; (cd "$W" && timeout -k 10 "$t" "$@") > "$OUT/cli/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -4 "$OUT/cli/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
R=$PWD
SYN="--synthetic 8 --synthetic-shape 600x1000"
run alternate_r50 500 python -u $R/train_alternate.py $SYN --network resnet50 --rpn_epoch 1 --rcnn_epoch 1 \
    --model-dir $W/alt --root_path $W --pretrained none --frequent 2 --max-steps 8
run end2end_r50 400 python -u $R/train_end2end.py $SYN --network resnet50 --num_epoch 1 --prefix $W/e2e \
    --pretrained none --frequent 2
run test_r50 400 python -u $R/test.py --network resnet50 --prefix $W/e2e --epoch 1 $SYN
ls -la $W $W/alt > "$OUT/cli/files.txt" 2>&1
