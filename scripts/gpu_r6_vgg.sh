#!/bin/bash
# round 6: VGG16 600x1000 training throughput (fp32 + bf16x3 + bf16 extras), single process (fc6 / fc7
# update fused into their weight gradient) vs a 1-rank RCCL group (MXR_FORCE_DIST=1: every bucket
# all-reduced in the captured step, fc6 / fc7 updated right after their buckets' all-reduce)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r6; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r6"
A="--network vgg16 --image 600x1000 --num-classes 21 --steps ${STEPS:-40} --warmup 5"
for rep in 1 2; do
  timeout -k 10 400 python bench.py $A > $OUT/vgg_plain_$rep.log 2>&1 || { tail -20 $OUT/vgg_plain_$rep.log; exit 1; }
  grep '^{' $OUT/vgg_plain_$rep.log | cut -c1-120
  MXR_FORCE_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $((29700 + rep)) bench.py $A > $OUT/vgg_dp1_$rep.log 2>&1 || { tail -20 $OUT/vgg_dp1_$rep.log; exit 1; }
  grep '^{' $OUT/vgg_dp1_$rep.log | cut -c1-120
done
