#!/bin/bash
# PMC passes (one counter group per run, each under its own time limit) for one conv config.
# usage: SHAPE=s3_3x3 CONFIGS="3:0 16:0" bash scripts/gpu_pmc_conv.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum"
for cfg in $CONFIGS; do
  t=${cfg%%:*}; s=${cfg##*:}
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    d="$OUT/${SHAPE}_t${t}_s${s}_p$i"
    cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d "$d" -o run --output-format csv -- \
        python "$GRAFT_REPO_ROOT/tools/microbench/conv_one.py" "$SHAPE" "$t" "$s" 30 > "$d.log" 2>&1
    rc=$?; echo "$SHAPE t$t s$s pass$i rc=$rc"; [ $rc -ne 0 ] && tail -5 "$d.log" && exit $rc
  done
done
exit 0
