#!/bin/bash
# DP interference probe: the graphed ResNet-101 step with k CUs held by a side-stream kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for dt in fp32 bf16; do
  timeout -k 10 400 python -u tools/dp_interference.py --dtype $dt --steps 30 --us 1100 --ks 0,8,16,32,64 \
    > gpurun_out/dpi_$dt.jsonl 2> gpurun_out/dpi_$dt.err || { tail -20 gpurun_out/dpi_$dt.err; exit 1; }
  cat gpurun_out/dpi_$dt.jsonl
done
