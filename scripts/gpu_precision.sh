#!/bin/bash
# Precision evidence: per-layer parity probe (incl. the bf16-storage floor and the fp32-class arm),
# fixed-RoI R-CNN loss curves (fp32-class and bf16) and the e2e fp32-class curve.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -4 "$OUT/$name.log" | cut -c1-700; if [ $rc -ne 0 ]; then exit $rc; fi; }
run probe_rpn 300 python tools/parity_probe.py --mode rpn
run probe_rcnn 300 python tools/parity_probe.py --mode rcnn
run curve_rcnn_fp32 300 python tools/loss_curve.py --train-mode rcnn --dtype fp32 --steps 200 --out "$OUT/curve_rcnn_fp32.jsonl"
run curve_rcnn_bf16 300 python tools/loss_curve.py --train-mode rcnn --dtype bf16 --steps 200 --out "$OUT/curve_rcnn_bf16.jsonl"
run curve_e2e_fp32 400 python tools/loss_curve.py --dtype fp32 --steps 200 --out "$OUT/curve_e2e_fp32.jsonl"
