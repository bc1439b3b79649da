#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() {
  local name=$1 d=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --steps 40 --warmup 5 --dtype $d --no-bf16-extra > gpurun_out/ab7_$name.log 2>&1 || { tail -8 gpurun_out/ab7_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/ab7_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["hip_runtime"])')"
}
ab fp32_q2 fp32 X=1 && ab fp32_q0 fp32 MXR_GRAPH_QUEUES=0 && ab fp32_q1 fp32 MXR_GRAPH_QUEUES=1 && ab fp32_q3 fp32 MXR_GRAPH_QUEUES=3 && \
ab bf16_q2 bf16 X=1 && ab bf16_q0 bf16 MXR_GRAPH_QUEUES=0 && ab bf16_q1 bf16 MXR_GRAPH_QUEUES=1 && \
ab bf16_s4 bf16 MXR_GROUPED_S=4 && ab bf16x3_s4 bf16x3 MXR_GROUPED_S=4 && ab bf16x3 bf16x3 X=1 || exit 1
