#!/bin/bash
# Round-6 (late) secondary numbers: VGG16 (BASELINE config 2) at the three precisions, alternate-training
# stages (config 4), 2 images per GPU, test FPS (config 5, batch 1 / 8, bf16 / fp16).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/cfg6; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/cfg6"
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc $(grep '^{' "$OUT/$name.log" | python -c 'import json,sys
d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d.get("dtype"), {k: c[k]["value"] for k in ("bf16x3","bf16") if k in c})' 2>/dev/null)";
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log"; exit $rc; fi; }
run vgg16 300 python bench.py --network vgg16 --image 600x1000 --num-classes 21 --steps 50 --warmup 5
run alt_rpn_r50 300 python bench.py --network resnet50 --train-mode rpn --steps 50 --warmup 5
run alt_rcnn_r50 300 python bench.py --network resnet50 --train-mode rcnn --steps 50 --warmup 5
run e2e_r101_ims2 300 python bench.py --ims-per-gpu 2 --steps 30 --warmup 5
run test_b1 300 python bench_test.py --steps 50 --warmup 5
run test_b8 300 python bench_test.py --batch 8 --steps 30 --warmup 5
run test_b8_fp16 300 python bench_test.py --batch 8 --dtype fp16 --steps 30 --warmup 5
run headline 300 python bench.py --steps 50 --warmup 5
run test_b1_fp32 300 python bench_test.py --dtype fp32 --steps 50 --warmup 5
run test_b8_fp32 300 python bench_test.py --batch 8 --dtype fp32 --steps 20 --warmup 3
