#!/bin/bash
# A/B of the round-2 op switches on the headline bench (each arm its own process and time limit).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
NET=${NET:-resnet101}
EXTRA=${EXTRA:-}
for arm in "base:" "nostrided:MXR_STRIDED_DGRAD=0" "nofc:MXR_FC_KERNEL=0" "nopool:MXR_POOL_KERNEL=0" "base2:"; do
  name=${arm%%:*}; envs=${arm#*:}
  env $envs timeout -k 10 300 python bench.py --network $NET $EXTRA --steps 200 --warmup 10 > gpurun_out/ab_$name.log 2>&1
  rc=$?
  echo "$name rc=$rc $(tail -1 gpurun_out/ab_$name.log | cut -c1-110)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
