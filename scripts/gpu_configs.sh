#!/bin/bash
# The other BASELINE.json configurations on one MI355X: VGG16 e2e training 600x1000 (config 2) and
# ResNet-101 inference at batch 8 (config 5), plus the batch-1 test FPS.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -2 "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run bench_vgg16 400 python bench.py --network vgg16 --image 600x1000 --num-classes 21 --steps 20 --warmup 5
run bench_test_b1 300 python bench_test.py --steps 50 --warmup 5
run bench_test_b8 400 python bench_test.py --steps 20 --warmup 3 --batch 8
