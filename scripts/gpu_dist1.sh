#!/bin/bash
# RCCL code paths on one GPU: a forced 1-rank NCCL(=RCCL) process group with the bucketed
# all-reduce captured inside the hipGraph, plus the driver's torchrun launch shape at N=1.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -3 "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
MXR_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 run bench_dist1_graph 400 python bench.py --steps 20 --warmup 5
run torchrun1 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 1 --steps 20 --warmup 5
