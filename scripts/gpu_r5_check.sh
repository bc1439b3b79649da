#!/bin/bash
# round-5 iteration check: touched GPU tests, then kernel traces of the fp32 / bf16 steps
# (groups, launch shapes, stream overlap) -> gpurun_out/r5/trace_*
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r5; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r5"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_detection_ops.py tests/test_repeatability.py tests/test_dist_gpu.py tests/test_image_prep.py tests/test_caches.py} \
  -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/check_tests.log 2>&1 || { tail -40 $OUT/check_tests.log; exit 1; }
tail -2 $OUT/check_tests.log
fi
for d in ${TRACE:-fp32 bf16}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$d -o run -- \
    python bench.py --steps 10 --warmup 3 --dtype $d --no-bf16-extra ${BENCH_ARGS:-} > $OUT/prof_$d.log 2>&1 || { tail -20 $OUT/prof_$d.log; exit 1; }
  T=$(find $OUT/prof_$d -name '*kernel_trace.csv' | head -1)
  python tools/trace_groups.py "$T" --steps 10 --top 200 > $OUT/trace_${d}_groups.txt 2>&1
  python tools/trace_shapes.py "$T" 10 nms_reduce > $OUT/trace_${d}_launch_shapes.txt 2>&1
  python tools/stream_overlap.py "$T" --steps 5 > $OUT/trace_${d}_stream_overlap.txt 2>&1
  head -3 $OUT/trace_${d}_stream_overlap.txt | cut -c1-200
  grep -c "at::native" $OUT/trace_${d}_launch_shapes.txt
  rm -rf $OUT/prof_$d
done
