#!/bin/bash
# fp32 (x3) headline: kernel trace + summaries, and the K-group A/Bs (forward autotune candidates
# MXR_NO_KG=1, grouped backward MXR_GROUPED_KG=1|2|22) in both fp32 modes.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_kg.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/kg_tests.log 2>&1 || { tail -40 gpurun_out/kg_tests.log; exit 1; }
tail -1 gpurun_out/kg_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_x3 -o run -- \
  python bench.py --steps 10 --warmup 3 --no-bf16-extra > gpurun_out/prof_x3.log 2>&1 || exit $?
T=$(find gpurun_out/prof_x3 -name '*kernel_trace.csv' | head -1)
python tools/trace_shapes.py "$T" 10 nms_reduce > gpurun_out/r4_x3_launch_shapes.txt 2>&1
python tools/stream_overlap.py "$T" --steps 5 > gpurun_out/r4_x3_stream_overlap.txt 2>&1
python tools/trace_groups.py "$T" --steps 10 --top 50 > gpurun_out/r4_x3_groups.txt 2>&1
head -3 gpurun_out/r4_x3_launch_shapes.txt
ab() {  # name dtype env...
  local name=$1 d=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --steps 40 --warmup 5 --dtype $d > gpurun_out/ab_$name.log 2>&1 || { tail -5 gpurun_out/ab_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/ab_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for r in 1 2; do
  ab fp32_default_$r fp32 X=1 || exit 1
  ab fp32_gkg1_$r fp32 MXR_GROUPED_KG=1 || exit 1
  ab fp32_gkg22_$r fp32 MXR_GROUPED_KG=22 || exit 1
  ab fp32_nokg_$r fp32 MXR_NO_KG=1 MXR_GROUPED_KG=1 || exit 1
  ab bf16x3_default_$r bf16x3 X=1 || exit 1
  ab bf16x3_nokg_$r bf16x3 MXR_NO_KG=1 || exit 1
  ab bf16x3_gkg2_$r bf16x3 MXR_GROUPED_KG=2 || exit 1
  ab bf16_default_$r bf16 X=1 || exit 1
  ab bf16_nokg_$r bf16 MXR_NO_KG=1 || exit 1
done
