#!/bin/bash
# LDS-side PMC of the fp32 (x3) stage-3 forward conv in isolation: bank conflicts and LDS waits
# against busy cycles -> gpurun_out/r5/lds_pmc.jsonl
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r5
OUT="$PWD/gpurun_out/r5"
C="SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/ldspmc -o run -- \
  python tools/microbench/conv_x3_tiles.py --shapes s3_3x3,s3_1x1a --tiles 23 > $OUT/ldspmc.log 2>&1 || { tail -20 $OUT/ldspmc.log; exit 1; }
python tools/pmc_summary.py $OUT/ldspmc --match conv_igemm_buf_kernel --label x3_s3 > $OUT/lds_pmc.jsonl
rm -rf $OUT/ldspmc
cat $OUT/lds_pmc.jsonl
