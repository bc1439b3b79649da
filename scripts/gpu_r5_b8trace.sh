#!/bin/bash
# batch-8 inference kernel trace (bench_test.py) -> gpurun_out/r5/b8_groups.txt
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r5; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/b8prof -o run -- \
  python bench_test.py --batch 8 --steps 10 --warmup 3 > $OUT/b8prof.log 2>&1 || { tail -20 $OUT/b8prof.log; exit 1; }
T=$(find $OUT/b8prof -name '*kernel_trace.csv' | head -1)
python tools/trace_groups.py "$T" --steps 10 --top 40 > $OUT/b8_groups.txt 2>&1
rm -rf $OUT/b8prof
head -30 $OUT/b8_groups.txt | cut -c1-150
