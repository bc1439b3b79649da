#!/bin/bash
# PMC pass over the proposal-chain microbench: where the NMS mask / reduce and the sampler spend
# their cycles (VALU / LDS instruction counts, waits) -> gpurun_out/r5/nms_pmc.jsonl
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r5
OUT="$PWD/gpurun_out/r5"
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/nmspmc -o run -- \
  python tools/microbench/proposal_chain.py > $OUT/nmspmc.log 2>&1 || { tail -20 $OUT/nmspmc.log; exit 1; }
python tools/pmc_summary.py $OUT/nmspmc --match nms_mask_kernel,nms_reduce_mc_kernel,proposal_sample_kernel --label nms > $OUT/nms_pmc.jsonl
rm -rf $OUT/nmspmc
cat $OUT/nms_pmc.jsonl
