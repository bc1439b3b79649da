#!/bin/bash
# Interleaved A/B of the headline bench: A = default, B = with env $AB_ENV (e.g. "MXR_X=1"),
# ${AB_REPS:-3} rounds of A then B on the same box (box-to-box DVFS variance is ~3 %).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for i in $(seq ${AB_REPS:-3}); do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 $BENCH_ARGS > gpurun_out/ab_A$i.log 2>&1 || exit $?
  echo "A$i $(grep -o '"value": [0-9.]*' gpurun_out/ab_A$i.log)"
  timeout -k 10 300 env $AB_ENV python bench.py --steps 30 --warmup 5 $BENCH_ARGS > gpurun_out/ab_B$i.log 2>&1 || exit $?
  echo "B$i $(grep -o '"value": [0-9.]*' gpurun_out/ab_B$i.log)"
done
