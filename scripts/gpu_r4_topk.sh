#!/bin/bash
# grid radix top-k: correctness (B=8, N=50400, P in {6000, 12000}, graph replay) and timing vs torch.sort
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_detection_ops.py \
  -k "topk" > gpurun_out/topk_tests.log 2>&1 || { tail -40 gpurun_out/topk_tests.log; exit 1; }
tail -3 gpurun_out/topk_tests.log
timeout -k 10 200 python tools/microbench/topk_bench.py > gpurun_out/topk_bench.log 2>&1 || { tail -20 gpurun_out/topk_bench.log; exit 1; }
cat gpurun_out/topk_bench.log
