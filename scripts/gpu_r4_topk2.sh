#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_detection_ops.py tests/test_repeatability.py \
  -k "topk or proposal" -m gpu > gpurun_out/topk2_tests.log 2>&1 || { tail -40 gpurun_out/topk2_tests.log; exit 1; }
tail -1 gpurun_out/topk2_tests.log
timeout -k 10 200 python tools/microbench/topk_bench.py > gpurun_out/topk2_bench.log 2>&1 || { tail -20 gpurun_out/topk2_bench.log; exit 1; }
grep "us" gpurun_out/topk2_bench.log
ab() {
  local name=$1 d=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --steps 40 --warmup 5 --dtype $d --no-bf16-extra > gpurun_out/tk_$name.log 2>&1 || { tail -5 gpurun_out/tk_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/tk_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
ab bf16 bf16 X=1 && ab bf16_sort bf16 MXR_TOPK=0 && ab fp32 fp32 X=1 && ab fp32_sort fp32 MXR_TOPK=0 && ab bf16_b bf16 X=1 || exit 1
