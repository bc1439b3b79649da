#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() {
  local name=$1 d=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --steps 40 --warmup 5 --dtype $d --no-bf16-extra > gpurun_out/ab5_$name.log 2>&1 || { tail -8 gpurun_out/ab5_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/ab5_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["objective_first_last"])')"
}
ab fp32 fp32 X=1 && ab fp32_osgd fp32 MXR_OVERLAP_SGD=1 && ab bf16x3 bf16x3 X=1 && ab bf16x3_osgd bf16x3 MXR_OVERLAP_SGD=1 && \
ab fp32_b fp32 X=1 && ab fp32_osgd_b fp32 MXR_OVERLAP_SGD=1 || exit 1
