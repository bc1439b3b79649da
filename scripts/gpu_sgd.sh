#!/bin/bash
# SGD kernel variants (bandwidth), then the SGD GPU tests and an interleaved VGG16 / ResNet-101 A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 2 1; do
  MXR_SGD=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels.py tests/test_fp32x2.py -k sgd > gpurun_out/t_sgd.log 2>&1 || { tail -30 gpurun_out/t_sgd.log; exit 1; }
  echo "MXR_SGD=$v tests: $(tail -1 gpurun_out/t_sgd.log)"
done
for i in 1 2; do
  for v in 0 1 2; do
    MXR_SGD=$v timeout -k 10 120 python tools/microbench/sgd_bench.py >> gpurun_out/sgd_bench.jsonl 2> gpurun_out/sgd_bench.err || { tail -20 gpurun_out/sgd_bench.err; exit 1; }
  done
done
cat gpurun_out/sgd_bench.jsonl

for i in 1 2; do
  for v in 0 2; do
    MXR_SGD=$v timeout -k 10 300 python bench.py --network vgg16 --image 600x1000 --num-classes 21 --steps 50 --warmup 5 --no-bf16-extra > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "vgg MXR_SGD=$v $i $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
    MXR_SGD=$v timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-bf16-extra > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "r101 MXR_SGD=$v $i $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
  done
done
