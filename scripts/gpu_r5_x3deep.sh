#!/bin/bash
# x3 (fp32) forward at ring depth 4 / 5 (tiles 33 / 34): isolated sweep + headline A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r5; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r5"
timeout -k 10 300 python tools/microbench/conv_x3_tiles.py > $OUT/x3deep_sweep.jsonl 2> $OUT/x3deep_sweep.err || { tail -20 $OUT/x3deep_sweep.err; exit 1; }
cat $OUT/x3deep_sweep.jsonl | cut -c1-160
ab() {  # name env...
  local name=$1; shift
  env "$@" MXR_TUNE_PLAN=0 timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-bf16-extra > $OUT/ab_$name.log 2>&1 || { tail -5 $OUT/ab_$name.log; return 1; }
  echo "$name $(grep '^{' $OUT/ab_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for r in 1 2; do
  ab deep_$r X=1 || exit 1
  ab nodeep_$r MXR_NO_X3DEEP=1 || exit 1
done
