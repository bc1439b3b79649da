#!/bin/bash
# determinism probe under configurations that change the graph's queue / stream layout
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/det; export TMPDIR=/tmp
run() {  # label, precisions, extra args, env...
  local l=$1 p=$2 x=$3; shift 3
  env "$@" timeout -k 10 300 python tools/det_check.py $p $x > gpurun_out/det/$l.log 2>&1 || { tail -5 gpurun_out/det/$l.log; return 1; }
  echo "$l: $(grep 'arrays differ' gpurun_out/det/$l.log | tr '\n' ' ')"
}
run base bf16,bf16 "" MXR_NONE=1 || exit 1
run gq2 bf16,bf16 "" MXR_GRAPH_QUEUES=2 || exit 1
run sides0 bf16,bf16 "" MXR_SIDE_STREAMS=0 || exit 1
run e2e bf16,fp32 "--mode e2e" MXR_NONE=1 || exit 1
run e2e_gq2 bf16 "--mode e2e" MXR_GRAPH_QUEUES=2 MXR_SIDE_STREAMS=0 || exit 1
