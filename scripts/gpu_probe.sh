#!/bin/bash
# Host-vs-GPU probe of the graphed ResNet-101 step (tools/launch_probe.py) at both precisions,
# then interleaved A/B of the graph queue count on the fp32-class headline.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for p in fp32 bf16; do
  timeout -k 10 300 python -u tools/launch_probe.py --precision $p --steps 50 > gpurun_out/probe_$p.log 2>&1 || { tail -20 gpurun_out/probe_$p.log; exit 1; }
  tail -1 gpurun_out/probe_$p.log
done
for i in 1 2; do
  for q in 1 2 3; do
    timeout -k 10 300 env DEBUG_HIP_FORCE_GRAPH_QUEUES=$q python bench.py --steps 50 --warmup 5 --no-bf16-extra > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "queues=$q $i $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
  done
done
