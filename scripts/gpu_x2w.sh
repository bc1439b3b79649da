#!/bin/bash
# Wide-stage fp32-class conv (tile 26): x2 numerics tests, isolated timings vs tile 23, headline
# A/B (MXR_NO_X2W=1 keeps tile 26 out of the autotune), interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fp32x2.py > gpurun_out/t_x2w.log 2>&1 || { tail -30 gpurun_out/t_x2w.log; exit 1; }
tail -1 gpurun_out/t_x2w.log
timeout -k 10 300 python tools/microbench/conv_x2_tiles.py --shapes s3_1x1a,s3_3x3,s3_1x1b,s4_3x3,s4_1x1a,s4_1x1b,rpn_3x3 --tiles 23,26 --splits 1 > gpurun_out/x2w.jsonl 2>&1 || exit 1
grep -o '"shape": "[a-z0-9_]*", "tile": [0-9]*, "splits": 1, "us": [0-9.]*' gpurun_out/x2w.jsonl
for i in 1 2; do
  for e in MXR_NO_X2W=1 MXR_NONE=1; do
    timeout -k 10 300 env $e python bench.py --steps 30 --warmup 5 --no-bf16-extra > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "$e $i $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
  done
done
