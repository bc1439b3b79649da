#!/bin/bash
# round-6 inference check: BN-fold tests, batch-8 tile sweep with the fold epilogue (bias + ReLU),
# then test FPS with kernel traces (scripts/gpu_r6_trace.sh TEST_FPS)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r6; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r6"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $OUT/infer_tests.log 2>&1 || { tail -60 $OUT/infer_tests.log; exit 1; }
  tail -3 $OUT/infer_tests.log
fi
timeout -k 10 300 python tools/microbench/conv_tiles.py --shapes ${SHAPES:-b8_s3_1x1a,b8_s3_3x3,s3_1x1a,s3_3x3} \
  --tiles ${TILES:-23,30,200,201,202,203,204} --splits 1 --bias-relu > $OUT/b8_tiles_fold.jsonl 2>&1 || { tail -20 $OUT/b8_tiles_fold.jsonl; exit 1; }
grep '^{' $OUT/b8_tiles_fold.jsonl | python -c "import sys, json; [print(json.loads(l)['name'], json.loads(l).get('best'), json.loads(l).get('hipblaslt_us'), json.loads(l).get('t204_s1')) for l in sys.stdin]"
TEST_FPS="${TEST_FPS:-bf16:8 bf16:1 fp32:1 fp32:8}" TRACE=" " TEST_TRACE=1 bash scripts/gpu_r6_trace.sh
