#!/bin/bash
# PMC passes over a few eager training steps of the headline config (one counter group per run,
# each under its own time limit): per-kernel counters for the step's HIP kernels.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc_step"
mkdir -p "$OUT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum"
P3="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  d="$OUT/p$i"
  cd /tmp && timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P -d "$d" -o run --output-format csv -- \
      python "$GRAFT_REPO_ROOT/bench.py" --mode eager --steps 2 --warmup 2 > "$d.log" 2>&1
  rc=$?; echo "pass$i rc=$rc"; [ $rc -ne 0 ] && tail -5 "$d.log" && exit $rc
done
exit 0
