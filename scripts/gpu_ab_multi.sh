#!/bin/bash
# Interleaved A/B of env settings on the headline bench; variants separated by ';', each a
# space-separated list of VAR=value (AB_VARIANTS="A=1 B=2;A=2")
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
IFS=';' read -ra VS <<< "$AB_VARIANTS"
for i in $(seq ${AB_REPS:-2}); do
  for v in "${VS[@]}"; do
    timeout -k 10 300 env $v python bench.py --steps ${AB_STEPS:-30} --warmup 5 $BENCH_ARGS > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "[$v] $i $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
  done
done
