#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for d in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f_$d -o run -- \
    python bench.py --steps 10 --warmup 3 --dtype $d --no-bf16-extra > gpurun_out/prof_f_$d.log 2>&1 || exit $?
  T=$(find gpurun_out/prof_f_$d -name '*kernel_trace.csv' | head -1)
  python tools/trace_groups.py "$T" --steps 10 --top 60 > gpurun_out/r4_final_${d}_groups.txt 2>&1
  python tools/trace_shapes.py "$T" 10 nms_reduce > gpurun_out/r4_final_${d}_launch_shapes.txt 2>&1
  python tools/stream_overlap.py "$T" --steps 5 > gpurun_out/r4_final_${d}_stream_overlap.txt 2>&1
  grep -E "roi_pool|steps=|sgd|topk|stem" gpurun_out/r4_final_${d}_groups.txt | cut -c1-130
done
