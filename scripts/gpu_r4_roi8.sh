#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels.py tests/test_repeatability.py \
  tests/test_fp32x2.py tests/test_model.py -k "roi or fp16 or detect" -m gpu > gpurun_out/roi8_tests.log 2>&1 || { tail -40 gpurun_out/roi8_tests.log; exit 1; }
tail -1 gpurun_out/roi8_tests.log
for b in 8 1; do
  timeout -k 10 300 python bench_test.py --batch $b --steps 30 --warmup 5 > gpurun_out/roi8_b$b.log 2>&1 || { tail -20 gpurun_out/roi8_b$b.log; exit 1; }
  grep '^{' gpurun_out/roi8_b$b.log | cut -c1-140
done
