#!/bin/bash
# fp32 (x3 triple) mode: kernel numerics, step parity, smoke, headline bench with the extra modes.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_fp32x2.py tests/test_conv_kg.py tests/test_parity.py tests/test_dgrad_bt.py -m gpu -v -s \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/x3_tests.log 2>&1 || { tail -60 gpurun_out/x3_tests.log; exit 1; }
grep -E "passed|failed|median cos|worst cosine" gpurun_out/x3_tests.log | tail -20
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/x3_smoke.log 2>&1 || { tail -20 gpurun_out/x3_smoke.log; exit 1; }
tail -1 gpurun_out/x3_smoke.log
timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/x3_bench.log 2>&1 || { tail -20 gpurun_out/x3_bench.log; exit 1; }
grep '^{' gpurun_out/x3_bench.log
