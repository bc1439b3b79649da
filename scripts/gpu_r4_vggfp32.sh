#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
V="--network vgg16 --image 600x1000 --num-classes 21"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_vgg32 -o run -- \
  python bench.py $V --steps 10 --warmup 3 --no-bf16-extra > gpurun_out/prof_vgg32.log 2>&1 || exit $?
T=$(find gpurun_out/prof_vgg32 -name '*kernel_trace.csv' | head -1)
python tools/trace_groups.py "$T" --steps 10 --top 60 > gpurun_out/r4_vgg16_fp32_groups.txt 2>&1
head -30 gpurun_out/r4_vgg16_fp32_groups.txt | cut -c1-150
grep -n "at::native\|rocclr\|rocprim" gpurun_out/r4_vgg16_fp32_groups.txt | cut -c1-170
