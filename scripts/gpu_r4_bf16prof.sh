#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bf16 -o run -- \
  python bench.py --steps 10 --warmup 3 --dtype bf16 > gpurun_out/prof_bf16.log 2>&1 || exit $?
T=$(find gpurun_out/prof_bf16 -name '*kernel_trace.csv' | head -1)
python tools/trace_groups.py "$T" --steps 10 --top 50 > gpurun_out/r4_final_bf16_groups.txt 2>&1
python tools/stream_overlap.py "$T" --steps 5 > gpurun_out/r4_final_bf16_stream_overlap.txt 2>&1
head -40 gpurun_out/r4_final_bf16_groups.txt | cut -c1-140
head -4 gpurun_out/r4_final_bf16_stream_overlap.txt | cut -c1-300
timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_repeatability.py tests/test_fp32x2.py -k "roi" -m gpu > gpurun_out/roi2.log 2>&1 || { tail -30 gpurun_out/roi2.log; exit 1; }
tail -1 gpurun_out/roi2.log
