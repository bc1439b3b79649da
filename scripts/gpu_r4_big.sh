#!/bin/bash
# conv_big 128-row tiles (202 / 203): numerics, batch-8 GEMM sweep, batch-8 test FPS
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels.py \
  -k "conv_big" > gpurun_out/big_tests.log 2>&1 || { tail -40 gpurun_out/big_tests.log; exit 1; }
tail -2 gpurun_out/big_tests.log
timeout -k 10 300 python tools/microbench/conv_tiles.py --shapes b8_s3_1x1a,b8_s3_3x3,b8_s3_1x1b,b8_rpn_3x3,vgg_c3 \
  --tiles 23,200,201,202,203 --splits 1 > gpurun_out/big_sweep.log 2>&1 || { tail -20 gpurun_out/big_sweep.log; exit 1; }
cat gpurun_out/big_sweep.log | cut -c1-220
timeout -k 10 300 python bench_test.py --batch 8 --steps 30 --warmup 5 > gpurun_out/big_test_b8.log 2>&1 || { tail -20 gpurun_out/big_test_b8.log; exit 1; }
grep '^{' gpurun_out/big_test_b8.log | cut -c1-400
