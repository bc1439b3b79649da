#!/bin/bash
# BASELINE config 4 (alternate-training stages, ResNet-50 / ResNet-101, 1 GPU) and the
# 2-images-per-GPU e2e step, at the fp32-class default with the bf16 extra field.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-160; if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi; }
for net in resnet50 resnet101; do
  for m in rpn rcnn; do
    run alt_${net}_$m 400 python bench.py --network $net --train-mode $m --steps 50 --warmup 5
  done
done
run e2e_r101_ims2 400 python bench.py --ims-per-gpu 2 --steps 50 --warmup 5
grep -h '^{' $OUT/alt_*.log $OUT/e2e_r101_ims2.log > $OUT/alt_lines.jsonl
