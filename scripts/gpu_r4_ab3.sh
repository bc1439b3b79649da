#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() {
  local name=$1 d=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --steps 40 --warmup 5 --dtype $d --no-bf16-extra > gpurun_out/ab3_$name.log 2>&1 || { tail -5 gpurun_out/ab3_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/ab3_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
ab fp32 fp32 X=1 && ab fp32_fwd2 fp32 MXR_X3_FWD_S=2 && ab fp32_b fp32 X=1 && ab fp32_fwd2_b fp32 MXR_X3_FWD_S=2 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fp32 -o run -- \
  python bench.py --steps 10 --warmup 3 --no-bf16-extra > gpurun_out/prof_fp32.log 2>&1 || exit $?
T=$(find gpurun_out/prof_fp32 -name '*kernel_trace.csv' | head -1)
python tools/trace_groups.py "$T" --steps 10 --top 50 > gpurun_out/r4_final_fp32_groups.txt 2>&1
python tools/trace_shapes.py "$T" 10 nms_reduce > gpurun_out/r4_final_fp32_launch_shapes.txt 2>&1
python tools/stream_overlap.py "$T" --steps 5 > gpurun_out/r4_final_fp32_stream_overlap.txt 2>&1
head -25 gpurun_out/r4_final_fp32_groups.txt | cut -c1-140
