#!/bin/bash
# DP bitwise test (three precisions), then the fp32 step regression A/B (KG tiles, grid top-k,
# fused gradient clear), then a kernel trace of the top-k microbench
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_dist_gpu.py \
  > gpurun_out/reg_dist.log 2>&1 || { tail -40 gpurun_out/reg_dist.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/reg_dist.log | cut -c1-160
ab() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-bf16-extra > gpurun_out/reg_$name.log 2>&1 || { tail -5 gpurun_out/reg_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/reg_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
ab base X=1 && ab nokg MXR_NO_KG=1 && ab notopk MXR_TOPK=0 && ab noclear MXR_FUSED_GRAD_CLEAR=0 && ab base2 X=1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/topk_prof -o topk -- python tools/microbench/topk_bench.py > gpurun_out/topk_prof.log 2>&1 || { tail -20 gpurun_out/topk_prof.log; exit 1; }
find gpurun_out/topk_prof -name "*kernel_stats.csv" | head -3
