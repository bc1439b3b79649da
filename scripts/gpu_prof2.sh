#!/bin/bash
# Full GPU test tier, then kernel traces of the fp32 ResNet-101 step and the bf16 VGG16 step.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
fi
run prof_fp32 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_fp32" -o run -- \
    python bench.py --steps 10 --warmup 3 --no-bf16-extra
run prof_vgg 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_vgg" -o run -- \
    python bench.py --network vgg16 --image 600x1000 --num-classes 21 --dtype bf16 --steps 10 --warmup 3
