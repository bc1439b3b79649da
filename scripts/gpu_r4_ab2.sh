#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_kg.py -m gpu \
  > gpurun_out/ab2_kg.log 2>&1 || { tail -30 gpurun_out/ab2_kg.log; exit 1; }
tail -1 gpurun_out/ab2_kg.log
ab() {
  local name=$1 d=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --steps 40 --warmup 5 --dtype $d --no-bf16-extra > gpurun_out/ab2_$name.log 2>&1 || { tail -5 gpurun_out/ab2_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/ab2_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
ab fp32 fp32 X=1 && ab fp32_s3 fp32 MXR_GROUPED_X3S=3 && ab fp32_ms16 fp32 MXR_WGRAD_MIN_STEPS=16 && \
ab bf16 bf16 X=1 && ab bf16_ms16 bf16 MXR_WGRAD_MIN_STEPS=16 && ab bf16x3 bf16x3 X=1 && \
ab bf16x3_ms16 bf16x3 MXR_WGRAD_MIN_STEPS=16 && ab fp32_2 fp32 X=1 || exit 1
