#!/bin/bash
# run-to-run determinism of the bf16 Fast R-CNN step (tools/det_check.py) under stream knobs: only
# meaningful on a box where the baseline differs, so the baseline runs first and ends the script
# when it is clean
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/det; export TMPDIR=/tmp
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python tools/det_check.py bf16,bf16 > gpurun_out/det/$l.log 2>&1 || { tail -5 gpurun_out/det/$l.log; return 1; }
  echo "$l: $(grep 'arrays differ' gpurun_out/det/$l.log | tr '\n' ' ')"
}
run base MXR_NONE=1 || exit 1
grep -q ' 0 of ' gpurun_out/det/base.log && grep -c ' 0 of ' gpurun_out/det/base.log | grep -q 2 && { echo "baseline clean on this box"; exit 0; }
for k in MXR_WGRAD_STREAM=0 MXR_CACHE_SIDE=0 MXR_FORK_NOOP=0 MXR_SIDE_STREAMS=0 MXR_GROUPED_BWD=0 MXR_GROUPED_CONV=0 MXR_ZERO_GRAD_SIDE=0; do
  run ${k%%=*} $k || exit 1
done
