#!/bin/bash
# two data-parallel ranks on the box's one GPU (gloo between the ranks; tests/test_dist_gpu.py
# test_two_ranks_on_one_gpu_*) -> gpurun_out/r5/dp2_tests.log
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r5; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r5"
timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py -k two_ranks -m gpu -x -v -p no:cacheprovider \
  --timeout 600 --timeout-method thread > $OUT/dp2_tests.log 2>&1 || { tail -60 $OUT/dp2_tests.log; exit 1; }
tail -8 $OUT/dp2_tests.log
