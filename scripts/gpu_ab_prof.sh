#!/bin/bash
# A/B with kernel traces: for each arm "name:VAR=val,..." a 200-step bench and a rocprofv3 kernel
# trace (10 steps) on the same box, so per-kernel times compare without box-to-box variance.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
NET=${NET:-resnet101}
for arm in $ARMS; do
  name=${arm%%:*}; envs=${arm#*:}; envs=${envs//,/ }
  env $envs timeout -k 10 300 python bench.py --network $NET --steps 200 --warmup 10 > gpurun_out/abp_$name.log 2>&1
  rc=$?; echo "$name [$envs] rc=$rc $(tail -1 gpurun_out/abp_$name.log | cut -c1-120)"; [ $rc -ne 0 ] && exit $rc
  env $envs timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/abp_prof_$name -o run -- \
      python bench.py --network $NET --steps 10 --warmup 3 > gpurun_out/abp_prof_$name.log 2>&1
  rc=$?; echo "$name prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
