#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
timeout -k 5 60 tools/microbench/nms_bench_A && timeout -k 5 60 tools/microbench/nms_bench_A 6000 300 && timeout -k 5 60 tools/microbench/nms_bench_A 16384 6000 && timeout -k 10 300 python -u -m pytest tests/test_detection_ops.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
