#!/bin/bash
# fused fp32 (x3) kernels: numerics, parity, bench, and kernel traces of the fp32 and bf16x3 steps.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_fp32x2.py tests/test_conv_kg.py tests/test_parity.py tests/test_dgrad_bt.py \
  -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/x3f_tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/x3f_tests.log | head -30; tail -30 gpurun_out/x3f_tests.log; exit 1; }
grep -E "passed|failed|median cos" gpurun_out/x3f_tests.log | tail -8
timeout -k 10 400 python bench.py --steps 40 --warmup 5 > gpurun_out/x3f_bench.log 2>&1 || { tail -20 gpurun_out/x3f_bench.log; exit 1; }
grep '^{' gpurun_out/x3f_bench.log | cut -c1-200
grep '^{' gpurun_out/x3f_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bf16x3", d["config"]["bf16x3"]["value"], "bf16", d["config"]["bf16"]["value"])'
for d in fp32 bf16x3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$d -o run -- \
    python bench.py --steps 10 --warmup 3 --dtype $d --no-bf16-extra > gpurun_out/prof_$d.log 2>&1 || exit $?
  T=$(find gpurun_out/prof_$d -name '*kernel_trace.csv' | head -1)
  python tools/trace_groups.py "$T" --steps 10 --top 60 > gpurun_out/r4_${d}_groups.txt 2>&1
  python tools/stream_overlap.py "$T" --steps 5 > gpurun_out/r4_${d}_stream_overlap.txt 2>&1
  python tools/trace_shapes.py "$T" 10 nms_reduce > gpurun_out/r4_${d}_launch_shapes.txt 2>&1
  head -2 gpurun_out/r4_${d}_groups.txt
done
