#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/loss_curve.py --steps 200 --images 8 --dtype fp32 --out gpurun_out/r4_loss_curve_e2e_fp32.jsonl > gpurun_out/loss_fp32.log 2>&1 || { tail -20 gpurun_out/loss_fp32.log; exit 1; }
tail -3 gpurun_out/loss_fp32.log | cut -c1-300
timeout -k 10 400 python -u tools/loss_curve.py --steps 200 --images 8 --dtype fp32 --train-mode rcnn --out gpurun_out/r4_loss_curve_rcnn_fixed_rois_fp32.jsonl > gpurun_out/loss_rcnn_fp32.log 2>&1 || { tail -20 gpurun_out/loss_rcnn_fp32.log; exit 1; }
tail -3 gpurun_out/loss_rcnn_fp32.log | cut -c1-300
