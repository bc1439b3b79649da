#!/bin/bash
# Determinism round: the new bitwise tests, the RoI-pool / BN numerics tests, the DP bitwise test,
# then the fp32 bench with and without the deterministic frozen-BN sums.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_repeatability.py \
  tests/test_fp32x2.py -k "roi or bitwise or partial or repeatable" > gpurun_out/det_tests.log 2>&1 \
  || { tail -40 gpurun_out/det_tests.log; exit 1; }
tail -3 gpurun_out/det_tests.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels.py -k "roi or sgd" \
  tests/test_dist_gpu.py > gpurun_out/det_dist.log 2>&1 || { tail -40 gpurun_out/det_dist.log; exit 1; }
tail -3 gpurun_out/det_dist.log
ab() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-bf16-extra > gpurun_out/det_$name.log 2>&1 || { tail -5 gpurun_out/det_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/det_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
ab det X=1 && ab nondet MXR_NONDETERMINISTIC=1 && ab det2 X=1
