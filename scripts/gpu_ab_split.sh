#!/bin/bash
# A/B: x2 split-K for the ~1-tile-per-CU convs (MXR_X2_SPLITK), fp32 headline step, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
MXR_BENCH_DUMP_TUNE=1 MXR_X2_SPLITK=2 timeout -k 10 300 python bench.py --steps 5 --warmup 3 --no-bf16-extra > "$OUT/ab_tune.log" 2>&1 || exit 1
for rep in 1 2; do
  for s in 1 2 3 4; do
    MXR_CONV_TUNE=0 MXR_X2_SPLITK=$s timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-bf16-extra > "$OUT/ab_split_${s}_$rep.log" 2>&1 || exit 1
    echo "split $s rep $rep: $(grep -o '"value": [0-9.]*' "$OUT/ab_split_${s}_$rep.log")"
  done
done
