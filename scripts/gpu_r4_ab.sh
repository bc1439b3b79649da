#!/bin/bash
# fp32 (x3) A/B: the x3 K-group forward tiles in the autotune (vs MXR_NO_KG=1), grouped backward ring depth (MXR_GROUPED_X3S=2), the wgrad split plan, forward split-K
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-bf16-extra > gpurun_out/ab_$name.log 2>&1 || { tail -5 gpurun_out/ab_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/ab_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
ab base_1 X=1 || exit 1
ab nokg MXR_NO_KG=1 || exit 1
ab x3s2 MXR_GROUPED_X3S=2 || exit 1
ab ms8 MXR_WGRAD_MIN_STEPS=8 || exit 1
ab splitk2 MXR_X2_SPLITK=2 || exit 1
ab base_2 X=1 || exit 1
