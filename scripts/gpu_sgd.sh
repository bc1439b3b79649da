#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_model.py tests/test_observability.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/sgd_tests.log 2>&1 || { tail -40 gpurun_out/sgd_tests.log; exit 1; }
tail -2 gpurun_out/sgd_tests.log
MXR_OVERLAP_SGD=1 MXR_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/sgd_dist1.log 2>&1 || { tail -30 gpurun_out/sgd_dist1.log; exit 1; }
echo "dist1 $(grep -o '"value": [0-9.]*' gpurun_out/sgd_dist1.log)"
AB_ENVS="MXR_OVERLAP_SGD=1 MXR_OVERLAP_SGD=0" bash scripts/gpu_ab3.sh
