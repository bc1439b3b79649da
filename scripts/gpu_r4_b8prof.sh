#!/bin/bash
# batch-8 inference (BASELINE config 5) kernel trace: where the 11.8 ms per batch goes
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b8 -o run -- \
  python bench_test.py --batch 8 --steps 10 --warmup 3 > gpurun_out/prof_b8.log 2>&1 || exit $?
T=$(find gpurun_out/prof_b8 -name '*kernel_trace.csv' | head -1)
python tools/trace_groups.py "$T" --steps 10 --top 45 > gpurun_out/r4_test_b8_groups.txt 2>&1
head -48 gpurun_out/r4_test_b8_groups.txt | cut -c1-150
