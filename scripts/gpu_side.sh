#!/bin/bash
# side-stream change check: GPU tests touching backward, headline bench, forced 1-rank RCCL graph bench
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -3 "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run side_tests 600 python -u -m pytest tests/test_fused.py tests/test_kernels.py tests/test_model.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run side_bench 300 python bench.py --steps 30 --warmup 5
MXR_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 run side_dist1 300 python bench.py --steps 20 --warmup 5
run side_bench_eager 300 python bench.py --steps 10 --warmup 3 --mode eager
