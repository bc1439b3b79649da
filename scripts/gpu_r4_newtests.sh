#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_detection_ops.py tests/test_repeatability.py \
  -k "topk or fold" -m gpu > gpurun_out/newtests.log 2>&1 || { tail -40 gpurun_out/newtests.log; exit 1; }
tail -1 gpurun_out/newtests.log
