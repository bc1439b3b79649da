#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_detection_ops.py tests/test_repeatability.py \
  -k "nms or proposal" -m gpu > gpurun_out/nms_tests.log 2>&1 || { tail -40 gpurun_out/nms_tests.log; exit 1; }
tail -1 gpurun_out/nms_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_nms -o run -- \
  python bench.py --steps 10 --warmup 3 --dtype bf16 > gpurun_out/prof_nms.log 2>&1 || exit $?
T=$(find gpurun_out/prof_nms -name '*kernel_trace.csv' | head -1)
python tools/trace_groups.py "$T" --steps 10 --top 12 | grep -E "nms|steps" | cut -c1-140
python tools/stream_overlap.py "$T" --steps 5 | head -4 | cut -c1-200
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 --dtype bf16 > gpurun_out/nms_bf16_$r.log 2>&1 || exit 1
  echo "bf16_$r $(grep '^{' gpurun_out/nms_bf16_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
