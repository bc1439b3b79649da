#!/bin/bash
# fp32 (x3) A/B: grouped backward ring depth (MXR_GROUPED_X3S=2) and the wgrad split plan.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-bf16-extra > gpurun_out/ab_$name.log 2>&1 || { tail -5 gpurun_out/ab_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/ab_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for r in 1 2; do
  ab base_$r X=1 || exit 1
  ab x3s2_$r MXR_GROUPED_X3S=2 || exit 1
  ab ms8_$r MXR_WGRAD_MIN_STEPS=8 || exit 1
  ab ms32_$r MXR_WGRAD_MIN_STEPS=32 || exit 1
done
