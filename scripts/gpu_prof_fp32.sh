#!/bin/bash
# rocprofv3 kernel traces of the fp32-class headline step and the batch-8 inference step.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fp32 -o run -- \
  python bench.py --steps 10 --warmup 3 --no-bf16-extra ${BENCH_ARGS} > gpurun_out/prof_fp32.log 2>&1 || exit $?
tail -1 gpurun_out/prof_fp32.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b8 -o run -- \
  python bench_test.py --steps 10 --warmup 3 --batch 8 > gpurun_out/prof_b8.log 2>&1 || exit $?
tail -1 gpurun_out/prof_b8.log | cut -c1-300
