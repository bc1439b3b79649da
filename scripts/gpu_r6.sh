#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -3 "gpurun_out/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider -k "not graph"
run bench_graph 400 python bench.py --steps 20 --warmup 5
OUT=prof_graph2 run prof 600 bash scripts/gpu_prof.sh
