#!/bin/bash
# multi-workgroup NMS reducer: NMS / proposal tests (new + existing oracles), isolated timing of
# both reducers and the proposal sampler, kernel-trace stats of the microbench -> gpurun_out/r5/nms_*
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r5; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r5"
timeout -k 10 600 python -u -m pytest tests/test_nms_multi.py tests/test_detection_ops.py tests/test_repeatability.py \
  -k "nms or proposal or multi" -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $OUT/nms_tests.log 2>&1 || { tail -40 $OUT/nms_tests.log; exit 1; }
tail -2 $OUT/nms_tests.log
timeout -k 10 120 python -u tools/microbench/proposal_chain.py > $OUT/nms_bench_mc.jsonl 2>&1 || { tail -20 $OUT/nms_bench_mc.jsonl; exit 1; }
MXR_NMS_PER=16 timeout -k 10 120 python -u tools/microbench/proposal_chain.py > $OUT/nms_bench_per16.jsonl 2>&1 || { tail -20 $OUT/nms_bench_per16.jsonl; exit 1; }
MXR_NMS_SERIAL=1 timeout -k 10 120 python -u tools/microbench/proposal_chain.py > $OUT/nms_bench_serial.jsonl 2>&1 || { tail -20 $OUT/nms_bench_serial.jsonl; exit 1; }
grep -h '^{' $OUT/nms_bench_mc.jsonl $OUT/nms_bench_per16.jsonl $OUT/nms_bench_serial.jsonl
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/nms_prof -o run -- \
  python -u tools/microbench/proposal_chain.py > $OUT/nms_prof.log 2>&1 || { tail -20 $OUT/nms_prof.log; exit 1; }
S=$(find $OUT/nms_prof -name '*kernel_stats.csv' | head -1)
grep -E "nms|proposal_sample" "$S" | cut -c1-220
