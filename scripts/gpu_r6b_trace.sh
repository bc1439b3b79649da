#!/bin/bash
# kernel traces at HEAD of the fp32 training steps: ResNet-101 e2e (headline) and VGG16 e2e
# (BASELINE config 2), groups + stream overlap -> gpurun_out/r6b/
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r6b; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r6b"
run() {  # name, dtype, bench args...
  local n=$1 d=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$n -o run -- \
    python bench.py --steps 10 --warmup 3 --dtype $d --no-bf16-extra "$@" > $OUT/prof_$n.log 2>&1 || { tail -20 $OUT/prof_$n.log; return 1; }
  T=$(find $OUT/prof_$n -name '*kernel_trace.csv' | head -1)
  python tools/trace_groups.py "$T" --steps 10 --top 200 > $OUT/${n}_groups.txt 2>&1
  python tools/stream_overlap.py "$T" --steps 5 > $OUT/${n}_stream_overlap.txt 2>&1
  head -4 $OUT/${n}_stream_overlap.txt | cut -c1-200
  grep '^{' $OUT/prof_$n.log | cut -c1-200
  rm -rf $OUT/prof_$n
}
for spec in ${RUNS:-vgg16_fp32 r101_fp32}; do
  case $spec in
    vgg16_*) run $spec ${spec#vgg16_} --network vgg16 --image 600x1000 --num-classes 21 || exit 1 ;;
    r101_*) run $spec ${spec#r101_} || exit 1 ;;
  esac
done
