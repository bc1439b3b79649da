#!/bin/bash
# determinism probe + K-order (MXR_TAP_INNER) numerics and same-box A/B of the training step
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/det_check.py ${DET:-bf16,bf16,bf16} > gpurun_out/det.log 2>&1 || { tail -5 gpurun_out/det.log; exit 1; }
grep -v amdgpu.ids gpurun_out/det.log | head -40
MXR_TAP_INNER=1 timeout -k 10 400 python -u -m pytest tests/test_kernels.py tests/test_fp32x2.py -m gpu -x -q -k 'not wide_stage_equals_narrow' --timeout 120 --timeout-method thread > gpurun_out/tap_tests.log 2>&1 || { tail -30 gpurun_out/tap_tests.log; exit 1; }
tail -2 gpurun_out/tap_tests.log
for rep in 1 2; do
  for t in 0 1; do
    MXR_TAP_INNER=$t timeout -k 10 200 python bench.py --steps 40 --warmup 5 > gpurun_out/tap_ab_$t.log 2>&1 || { tail -5 gpurun_out/tap_ab_$t.log; exit 1; }
    echo "tap_inner=$t rep$rep $(grep '^{' gpurun_out/tap_ab_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c.get("bf16x3"), c.get("bf16"))')"
  done
done
