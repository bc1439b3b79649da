#!/bin/bash
# rocprofv3 kernel-trace + stats of the graph-mode bench (the headline path).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=${OUT:-prof_graph}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$OUT -o run -- \
  python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/$OUT.log 2>&1
rc=$?; tail -2 gpurun_out/$OUT.log; exit $rc
