#!/bin/bash
# BASELINE config 4 (alternate-training stages) and the multi-image length axis on one GPU.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/cfg2; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/cfg2"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; grep '^{' "$OUT/$name.log" | cut -c1-260; tail -2 "$OUT/$name.log" | grep -v '^{' | cut -c1-300;
  if [ $rc -ne 0 ]; then exit $rc; fi; }
run alt_rpn_r50 300 python bench.py --network resnet50 --train-mode rpn --steps 100 --warmup 10
run alt_rcnn_r50 300 python bench.py --network resnet50 --train-mode rcnn --steps 100 --warmup 10
run alt_rpn_r101 300 python bench.py --train-mode rpn --steps 100 --warmup 10
run alt_rcnn_r101 300 python bench.py --train-mode rcnn --steps 100 --warmup 10
run e2e_r101_ims2 300 python bench.py --ims-per-gpu 2 --steps 50 --warmup 5
