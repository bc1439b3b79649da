#!/bin/bash
# Detector GPU tests + test FPS (head tail-BN fused), then interleaved A/B of env knobs on the
# fp32-class headline (AB_ENVS).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_detection_ops.py tests/test_model.py tests/test_fused.py > gpurun_out/t_det.log 2>&1 || { tail -30 gpurun_out/t_det.log; exit 1; }
tail -1 gpurun_out/t_det.log
for b in 1 8; do
  timeout -k 10 300 python bench_test.py --steps 30 --warmup 3 --batch $b > gpurun_out/bt$b.log 2>&1 || { tail -5 gpurun_out/bt$b.log; exit 1; }
  echo "test b$b $(grep -o '"value": [0-9.]*' gpurun_out/bt$b.log)"
done
for i in 1 2; do
  for e in $AB_ENVS; do
    timeout -k 10 300 env $e python bench.py --steps 30 --warmup 5 --no-bf16-extra > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "$e $i $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
  done
done
