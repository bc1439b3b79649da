#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels.py tests/test_fused.py tests/test_model.py tests/test_observability.py tests/test_detection_ops.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/loss_tests.log 2>&1 || { tail -40 gpurun_out/loss_tests.log; exit 1; }
tail -2 gpurun_out/loss_tests.log
AB_REPS=2 AB_ENVS="X=0" bash scripts/gpu_ab3.sh
