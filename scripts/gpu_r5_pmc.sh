#!/bin/bash
# MFMA-pipe utilisation of the step's conv kernels (VERDICT r4 weak #1c): one PMC pass per
# precision (SQ_VALU_MFMA_BUSY_CYCLES against GRBM_GUI_ACTIVE, wait / issue fractions), per
# kernel and grid (tools/pmc_summary.py).
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r5
OUT="$PWD/gpurun_out/r5"
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
for d in ${PREC:-fp32 bf16}; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_$d -o run -- \
    python bench.py --dtype $d --steps 3 --warmup 2 --no-bf16-extra > $OUT/pmc_$d.log 2>&1 || { tail -20 $OUT/pmc_$d.log; exit 1; }
  python tools/pmc_summary.py $OUT/pmc_$d --label $d > $OUT/r5_pmc_mfma_$d.jsonl
  rm -rf $OUT/pmc_$d
  python -c "
import json,sys
rows=[json.loads(l) for l in open('$OUT/r5_pmc_mfma_$d.jsonl')]
rows.sort(key=lambda r: -r.get('GRBM_GUI_ACTIVE',0)*r['dispatches'])
for r in rows[:12]: print(r['label'], r['kernel'][:60], r['dispatches'], r.get('mfma_util'), r.get('wait_frac'))
"
done
