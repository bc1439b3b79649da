#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() {
  local name=$1 d=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --steps 40 --warmup 5 --dtype $d --no-bf16-extra > gpurun_out/ab4_$name.log 2>&1 || { tail -5 gpurun_out/ab4_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/ab4_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
ab fp32 fp32 X=1 && ab fp32_m95 fp32 MXR_TUNE_MARGIN=0.95 && ab fp32_m100 fp32 MXR_TUNE_MARGIN=1.0 && \
ab bf16 bf16 X=1 && ab bf16_m95 bf16 MXR_TUNE_MARGIN=0.95 && ab bf16x3 bf16x3 X=1 && ab bf16x3_m95 bf16x3 MXR_TUNE_MARGIN=0.95 && \
ab fp32_b fp32 X=1 && ab fp32_m95b fp32 MXR_TUNE_MARGIN=0.95 || exit 1
