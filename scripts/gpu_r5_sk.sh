#!/bin/bash
# stream-K 64x64 conv (tile 40): numerics, isolated timing vs tiles 23 / 30, headline A/B with a
# fresh autotune (MXR_TUNE_PLAN=0) with / without the candidate
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r5; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r5"
timeout -k 10 300 python -u -m pytest tests/test_conv_sk.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $OUT/sk_tests.log 2>&1 || { tail -40 $OUT/sk_tests.log; exit 1; }
tail -1 $OUT/sk_tests.log
timeout -k 10 200 python tools/microbench/conv_x3_tiles.py --shapes s3_3x3,s3_1x1a,s3_1x1b --tiles 23,30,40 > $OUT/sk_x3.jsonl 2>&1 || { tail -5 $OUT/sk_x3.jsonl; exit 1; }
timeout -k 10 200 python tools/microbench/conv_tiles.py --shapes s3_3x3,s3_1x1a,s3_1x1b --tiles 23,30,40 --splits 1 > $OUT/sk_bf16.jsonl 2>&1 || { tail -5 $OUT/sk_bf16.jsonl; exit 1; }
grep -v Warn $OUT/sk_x3.jsonl $OUT/sk_bf16.jsonl | grep -v amdgpu.ids | cut -c1-170
ab() {  # name dtype env...
  local name=$1 d=$2; shift 2
  env "$@" MXR_TUNE_PLAN=0 timeout -k 10 200 python bench.py --steps 60 --warmup 5 --dtype $d --no-bf16-extra > $OUT/sk_ab_$name.log 2>&1 || { tail -5 $OUT/sk_ab_$name.log; return 1; }
  echo "$name $(grep '^{' $OUT/sk_ab_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for r in 1 2; do
  ab fp32_sk_$r fp32 X=1 || exit 1
  ab fp32_nosk_$r fp32 MXR_NO_SK=1 || exit 1
  ab bf16_sk_$r bf16 X=1 || exit 1
  ab bf16_nosk_$r bf16 MXR_NO_SK=1 || exit 1
done
