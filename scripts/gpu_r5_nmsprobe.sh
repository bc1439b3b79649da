#!/bin/bash
# NMS reducer timeline probe (MXR_NMS_PROBE=1) at 16 and 8 blocks per workgroup, plus the sampler timing
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r5; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r5"
MXR_NMS_PROBE=1 timeout -k 10 120 python -u tools/microbench/proposal_chain.py > $OUT/nms_probe8.jsonl 2>&1 || { tail -20 $OUT/nms_probe8.jsonl; exit 1; }
MXR_NMS_PROBE=1 MXR_NMS_PER=16 timeout -k 10 120 python -u tools/microbench/proposal_chain.py > $OUT/nms_probe16.jsonl 2>&1 || { tail -20 $OUT/nms_probe8.jsonl; exit 1; }
grep -h '"probe"' $OUT/nms_probe16.jsonl $OUT/nms_probe8.jsonl | cut -c1-400
