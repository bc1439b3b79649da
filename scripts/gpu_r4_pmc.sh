#!/bin/bash
# the wide-stage x2 kernel (tile 26, MXR_X2W=1) in the bf16x3 step vs isolated: L2 hit rate and wait
# fraction per dispatch against the default 64x64 buffer kernel (tile 23)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
C="SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES TCC_HIT_sum TCC_MISS_sum"
MXR_X2W=1 timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_step -o run -- \
  python bench.py --dtype bf16x3 --steps 3 --warmup 2 --no-bf16-extra > gpurun_out/pmc_step.log 2>&1 || { tail -20 gpurun_out/pmc_step.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_iso -o run -- \
  python tools/microbench/conv_x2_tiles.py --shapes s3_1x1a,s3_3x3,s3_1x1b --tiles 23,26 --splits 1 > gpurun_out/pmc_iso.log 2>&1 || { tail -20 gpurun_out/pmc_iso.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc_step --label in-step > gpurun_out/r4_x2w_pmc.jsonl
python tools/pmc_summary.py gpurun_out/pmc_iso --label isolated >> gpurun_out/r4_x2w_pmc.jsonl
cat gpurun_out/r4_x2w_pmc.jsonl | cut -c1-330
grep "us" gpurun_out/pmc_iso.log | head -8 | cut -c1-200
