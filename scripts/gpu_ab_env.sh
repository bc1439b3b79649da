#!/bin/bash
# A/B of runtime environment knobs on the headline bench: each arm "name:VAR=val,VAR2=val" runs in
# its own process under its own time limit; the first failing arm ends the script.
#   ARMS="base: q1:DEBUG_HIP_FORCE_GRAPH_QUEUES=1" bash scripts/gpu_ab_env.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
NET=${NET:-resnet101}
EXTRA=${EXTRA:-}
STEPS=${STEPS:-200}
for arm in $ARMS; do
  name=${arm%%:*}; envs=${arm#*:}
  envs=${envs//,/ }
  env $envs timeout -k 10 300 python bench.py --network $NET $EXTRA --steps $STEPS --warmup 10 > gpurun_out/ab_$name.log 2>&1
  rc=$?
  echo "$name [$envs] rc=$rc $(tail -1 gpurun_out/ab_$name.log | cut -c1-110)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
