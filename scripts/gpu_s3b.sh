#!/bin/bash
# Smoke + benches first, then the graph-capture test in isolation and a stage bisect of the capture
# (one stage per process; stops at the first crash).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -3 "$OUT/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run smoke 300 python __graft_entry__.py smoke
run bench_graph 400 python bench.py --steps 20 --warmup 5
run bench_test 400 python bench_test.py --steps 50 --warmup 5
run graphtest 200 python -u -m pytest tests/test_model.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for s in trunk_fwd trunk_fwdbwd rpn_fwdbwd e2e_fwd e2e_fwdbwd step; do run bisect_$s 120 python tools/capture_bisect.py $s; done
