#!/bin/bash
# round-6 measurements at HEAD: kernel traces of the fp32 / bf16 training steps (groups, launch
# shapes, stream overlap), test FPS at fp32 / bf16 (batch 1 and 8) with a kernel trace of each
# (vendor conv / GEMM kernels counted), -> gpurun_out/r6/
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r6; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r6"
for d in ${TRACE:-fp32 bf16}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$d -o run -- \
    python bench.py --steps 10 --warmup 3 --dtype $d --no-bf16-extra ${BENCH_ARGS:-} > $OUT/prof_$d.log 2>&1 || { tail -20 $OUT/prof_$d.log; exit 1; }
  T=$(find $OUT/prof_$d -name '*kernel_trace.csv' | head -1)
  python tools/trace_groups.py "$T" --steps 10 --top 200 > $OUT/trace_${d}_groups.txt 2>&1
  python tools/trace_shapes.py "$T" 10 nms_reduce_mc > $OUT/trace_${d}_launch_shapes.txt 2>&1
  python tools/stream_overlap.py "$T" --steps 5 > $OUT/trace_${d}_stream_overlap.txt 2>&1
  head -4 $OUT/trace_${d}_stream_overlap.txt | cut -c1-200
  grep '^{' $OUT/prof_$d.log | cut -c1-200
  rm -rf $OUT/prof_$d
done
for spec in ${TEST_FPS:-}; do  # e.g. "fp32:1 bf16:1 bf16:8 fp32:8"
  dt=${spec%%:*}; nb=${spec#*:}
  timeout -k 10 300 python bench_test.py --dtype $dt --batch $nb --steps 50 --warmup 5 > $OUT/test_${dt}_b$nb.log 2>&1 || { tail -20 $OUT/test_${dt}_b$nb.log; exit 1; }
  grep '^{' $OUT/test_${dt}_b$nb.log | cut -c1-260
  if [ "${TEST_TRACE:-0}" = 1 ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tprof -o run -- \
      python bench_test.py --dtype $dt --batch $nb --steps 10 --warmup 3 > $OUT/test_prof_${dt}_b$nb.log 2>&1 || { tail -20 $OUT/test_prof_${dt}_b$nb.log; exit 1; }
    T=$(find $OUT/tprof -name '*kernel_trace.csv' | head -1)
    python tools/trace_groups.py "$T" --marker nms_reduce_mc --steps 10 --top 80 > $OUT/test_trace_${dt}_b$nb.txt 2>&1
    echo "vendor conv/GEMM kernels in the $dt b$nb test trace: $(grep -ciE 'Cijk|miopen|igemm_fwd_gtc|naive_conv|rocblas|hipblas|at::native::.*(conv|gemm|addmm)' $OUT/test_trace_${dt}_b$nb.txt || true)"
    rm -rf $OUT/tprof
  fi
done
