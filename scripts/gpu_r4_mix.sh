#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels.py tests/test_repeatability.py \
  tests/test_fp32x2.py -k roi -m gpu > gpurun_out/mix_roi.log 2>&1 || { tail -30 gpurun_out/mix_roi.log; exit 1; }
tail -1 gpurun_out/mix_roi.log
timeout -k 10 300 python bench_test.py --batch 8 --steps 30 --warmup 5 > gpurun_out/mix_b8.log 2>&1 || { tail -20 gpurun_out/mix_b8.log; exit 1; }
grep '^{' gpurun_out/mix_b8.log | cut -c1-200
bash scripts/gpu_r4_ab.sh
