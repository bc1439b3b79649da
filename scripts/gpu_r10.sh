#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -4 "$OUT/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest_k 600 python -m pytest tests/test_kernels.py tests/test_fused.py -q -p no:cacheprovider -x
run bench_graph 400 python bench.py --steps 20 --warmup 5
run bench_test 400 python bench_test.py --steps 50 --warmup 5
cd /tmp && run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_r10" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3
