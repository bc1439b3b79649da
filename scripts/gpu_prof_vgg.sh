#!/bin/bash
# rocprofv3 kernel traces of the VGG16 e2e step (BASELINE config 2) at both precisions.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for p in fp32 bf16; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_vgg_$p -o run -- \
    python bench.py --network vgg16 --image 600x1000 --num-classes 21 --dtype $p --no-bf16-extra --steps 10 --warmup 3 \
    > gpurun_out/prof_vgg_$p.log 2>&1 || exit $?
  tail -1 gpurun_out/prof_vgg_$p.log | cut -c1-200
done
