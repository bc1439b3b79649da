#!/bin/bash
# VGG16 bf16 regression hunt: kernel trace + groups, A/B of the round-4 switches; top-k kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
V="--network vgg16 --image 600x1000 --num-classes 21"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_vgg -o run -- \
  python bench.py $V --steps 10 --warmup 3 --dtype bf16 --no-bf16-extra > gpurun_out/prof_vgg.log 2>&1 || exit $?
T=$(find gpurun_out/prof_vgg -name '*kernel_trace.csv' | head -1)
python tools/trace_groups.py "$T" --steps 10 --top 45 > gpurun_out/r4_vgg16_bf16_groups.txt 2>&1
head -48 gpurun_out/r4_vgg16_bf16_groups.txt | cut -c1-150
ab() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py $V --steps 40 --warmup 5 --dtype bf16 --no-bf16-extra > gpurun_out/vab_$name.log 2>&1 || { tail -5 gpurun_out/vab_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/vab_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
ab base X=1 && ab noclear MXR_FUSED_GRAD_CLEAR=0 && ab notopk MXR_TOPK=0 && ab nofused MXR_VGG_FUSED=0 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/topk_prof -o topk -- \
  python tools/microbench/topk_bench.py > gpurun_out/topk_prof.log 2>&1 || { tail -20 gpurun_out/topk_prof.log; exit 1; }
S=$(find gpurun_out/topk_prof -name '*kernel_stats.csv' | head -1)
cut -d, -f1-8 "$S" | head -20
