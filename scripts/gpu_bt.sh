#!/bin/bash
# bt dgrad / rmask / fused VGG tests, the x2 + kernel + parity tiers, the 1-rank RCCL step test, a short bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-1500; if [ $rc -ne 0 ]; then exit $rc; fi; }
run bt_tests 300 python -u -m pytest tests/test_dgrad_bt.py -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread

run dist_gpu 700 python -u -m pytest tests/test_dist_gpu.py -m gpu -v -s -x -p no:cacheprovider --timeout 600 --timeout-method thread
run bench 400 python bench.py --steps 20 --warmup 5
run bench_vgg 400 python bench.py --network vgg16 --image 600x1000 --num-classes 21 --steps 20 --warmup 5
