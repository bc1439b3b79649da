#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -3 "gpurun_out/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider -k "not graph"
MXR_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 run bench_dist1_graph 400 python bench.py --steps 10 --warmup 3
run torchrun1 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 1 --steps 10 --warmup 3
run bench_graph 400 python bench.py --steps 20 --warmup 5
