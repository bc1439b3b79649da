#!/bin/bash
# round-6 iteration check: the touched GPU tests (TESTS), then optional interleaved A/B bench runs
# (AB="name:ENV=V,ENV2=V2 name2:..." each run as `python bench.py` with those variables)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r6; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r6"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 200 \
    --timeout-method thread > $OUT/check_tests.log 2>&1 || { tail -60 $OUT/check_tests.log; exit 1; }
  tail -3 $OUT/check_tests.log
fi
for rep in $(seq 1 ${REPS:-1}); do
  for spec in ${AB:-}; do
    name=${spec%%:*}; envs=${spec#*:}
    [ "$envs" = "$spec" ] && envs=""
    timeout -k 10 ${BENCH_LIMIT:-300} env $(echo "$envs" | tr ',' ' ') python ${BENCH_SCRIPT:-bench.py} ${BENCH_ARGS:---steps 40 --warmup 5 --no-bf16-extra} \
      > $OUT/ab_${name}_$rep.log 2>&1 || { tail -20 $OUT/ab_${name}_$rep.log; exit 1; }
    echo "$name rep$rep $(grep '^{' $OUT/ab_${name}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_runtime"))')"
  done
done
