#!/bin/bash
# Large-tile kernel evidence: batch-8 test trace, VGG16 training A/B (MXR_NO_BIG=1 disables the
# 256-row tiles in the conv autotune), conv_big numerics tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels.py -k "conv_big or conv_igemm_fwd_vs_fp32" > gpurun_out/t_big.log 2>&1 || { tail -20 gpurun_out/t_big.log; exit 1; }
tail -1 gpurun_out/t_big.log
for e in MXR_NO_BIG=1 MXR_NONE=1 MXR_NO_BIG=1 MXR_NONE=1; do
  timeout -k 10 300 env $e python bench.py --network vgg16 --image 600x1000 --num-classes 21 --steps 30 --warmup 5 > gpurun_out/vgg.log 2>&1 || { tail -5 gpurun_out/vgg.log; exit 1; }
  echo "vgg $e $(grep -o '"value": [0-9.]*' gpurun_out/vgg.log | head -2 | tr '\n' ' ')"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b8big -o run -- \
  python bench_test.py --steps 10 --warmup 3 --batch 8 > gpurun_out/prof_b8big.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' gpurun_out/prof_b8big.log
