#!/bin/bash
# Iteration loop: selected GPU tests (TESTS), headline bench, optional rocprof (PROF=1).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -3 "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
if [ -n "$TESTS" ]; then
  run tests 600 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
fi
if [ "${BENCH:-1}" = 1 ]; then
  run bench 400 python bench.py --steps 20 --warmup 5 $BENCH_ARGS
fi
if [ "${BENCH_TEST:-0}" = 1 ]; then
  run bench_test 400 python bench_test.py --steps 50 --warmup 5
fi
if [ "${PROF:-0}" = 1 ]; then
  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${PROF_NAME:-prof_iter}" -o run -- \
      python bench.py --steps 10 --warmup 3 $BENCH_ARGS
fi
