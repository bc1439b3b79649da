#!/bin/bash
# Conv autotune plan for the benchmark configurations (ops/tune_plan.py): every bench shape tuned
# once into gpurun_out/r5/plan.json (shipped as mx_rcnn_amd/tune/gfx950.json); then the glue
# attribution of the fp32 ResNet-101 and bf16 VGG16 steps (tools/glue_trace.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r5; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r5"
export MXR_TUNE_FILE=$OUT/plan.json
rm -f $MXR_TUNE_FILE
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/plan_$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc $(grep -c . $MXR_TUNE_FILE 2>/dev/null)"; grep '^{' "$OUT/plan_$name.log" | cut -c1-160; if [ $rc -ne 0 ]; then tail -5 "$OUT/plan_$name.log"; exit $rc; fi; }
run r101 300 python bench.py --steps 10 --warmup 3
run r101_ims2 300 python bench.py --steps 10 --warmup 3 --ims-per-gpu 2
run vgg16 300 python bench.py --steps 10 --warmup 3 --network vgg16 --image 600x1000 --num-classes 21
run r101_600 300 python bench.py --steps 10 --warmup 3 --image 600x1000 --num-classes 8
run vgg16_600_c8 300 python bench.py --steps 10 --warmup 3 --network vgg16 --image 600x1000 --num-classes 8
run r50_rpn 300 python bench.py --steps 10 --warmup 3 --network resnet50 --train-mode rpn --image 600x1000 --num-classes 21
run r50_rcnn 300 python bench.py --steps 10 --warmup 3 --network resnet50 --train-mode rcnn --image 600x1000 --num-classes 21
run test_b1 300 python bench_test.py --steps 10 --warmup 3
run test_b8 300 python bench_test.py --steps 5 --warmup 2 --batch 8
run test_b8_f16 300 python bench_test.py --steps 5 --warmup 2 --batch 8 --dtype fp16
unset MXR_TUNE_FILE
timeout -k 10 300 python tools/glue_trace.py --steps 3 > $OUT/glue_r101_fp32.txt 2>&1 || { tail -20 $OUT/glue_r101_fp32.txt; exit 1; }
head -40 $OUT/glue_r101_fp32.txt
