#!/bin/bash
# A/B/C of env settings on the headline bench, interleaved: AB_ENVS="X=1 X=2 X=3" (one per variant)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for i in $(seq ${AB_REPS:-2}); do
  for e in $AB_ENVS; do
    timeout -k 10 300 env $e python bench.py --steps 30 --warmup 5 $BENCH_ARGS > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "$e $i $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
  done
done
