#!/bin/bash
# NMS correctness session: the large-P NMS / repeatability tests (with the MXR_NMS_CHECK device
# oracle on the proposal path), then the whole GPU tier, smoke and the headline bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -4 "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
MXR_NMS_CHECK=1 run nms_tests 300 python -u -m pytest tests/test_detection_ops.py tests/test_repeatability.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run smoke 300 python __graft_entry__.py smoke
run bench_graph 400 python bench.py --steps 20 --warmup 5
