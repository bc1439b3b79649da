#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-1500; if [ $rc -ne 0 ]; then exit $rc; fi; }
run dist_gpu 700 python -u -m pytest tests/test_dist_gpu.py -m gpu -v -s -x -p no:cacheprovider --timeout 600 --timeout-method thread
run bench 400 python bench.py --steps 20 --warmup 5
