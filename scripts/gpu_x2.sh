#!/bin/bash
# fp32-class (x2) kernel tests + the NMS tests, each step time-limited; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -6 "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run x2_tests 400 python -u -m pytest tests/test_fp32x2.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread
run nms_tests 300 python -u -m pytest tests/test_detection_ops.py tests/test_repeatability.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run parity_fp32 500 python -u -m pytest tests/test_parity.py -m gpu -v -k fp32 -p no:cacheprovider --timeout 200 --timeout-method thread
