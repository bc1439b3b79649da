#!/bin/bash
# Round evidence run: full GPU test tier, smoke, headline bench (200 steps), the other BASELINE
# configs (VGG16 600x1000 training, test FPS bf16 / fp16 at batch 1 and 8) and a kernel trace of
# the headline step (profiles/ summaries are derived from it).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
  run smoke 300 python __graft_entry__.py smoke
fi
run bench 400 python bench.py --steps 200 --warmup 10
run bench_vgg16 400 python bench.py --network vgg16 --image 600x1000 --num-classes 21 --steps 100 --warmup 10
run bench_test_b1 300 python bench_test.py --steps 100 --warmup 5
run bench_test_b8 400 python bench_test.py --steps 30 --warmup 3 --batch 8
run bench_test_f16_b8 400 python bench_test.py --steps 30 --warmup 3 --batch 8 --dtype fp16
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_round" -o run -- \
    python bench.py --steps 10 --warmup 3 --no-bf16-extra
