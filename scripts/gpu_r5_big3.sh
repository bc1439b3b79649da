#!/bin/bash
# conv_big 3-deep tiles 204 / 205: numerics, then batch-8 test FPS with / without them in the
# autotune (fresh tuning: MXR_TUNE_PLAN=0), interleaved twice
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r5; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r5"
timeout -k 10 300 python -u -m pytest tests/test_kernels.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k conv_big > $OUT/big3_tests.log 2>&1 || { tail -30 $OUT/big3_tests.log; exit 1; }
tail -1 $OUT/big3_tests.log
ab() {  # name env...
  local name=$1; shift
  env "$@" MXR_TUNE_PLAN=0 timeout -k 10 300 python bench_test.py --steps 30 --warmup 3 --batch 8 > $OUT/big3_$name.log 2>&1 || { tail -5 $OUT/big3_$name.log; return 1; }
  echo "$name $(grep '^{' $OUT/big3_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for r in 1 2; do
  ab big3_$r X=1 || exit 1
  ab nobig3_$r MXR_NO_BIG3=1 || exit 1
done
