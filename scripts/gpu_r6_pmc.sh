#!/bin/bash
# round 6: one PMC pass over the fp32 (headline) step's conv kernels -- LDS pressure next to MFMA
# busy (SQ_LDS_IDX_ACTIVE / SQ_LDS_DATA_FIFO_FULL / SQ_WAIT_INST_LDS / SQ_LDS_BANK_CONFLICT,
# SQ_VALU_MFMA_BUSY_CYCLES, wait / wave cycles), per kernel and grid (tools/pmc_summary.py)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r6
OUT="$PWD/gpurun_out/r6"
C="${COUNTERS:-SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL GRBM_GUI_ACTIVE}"
for d in ${PREC:-fp32}; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_$d -o run -- \
    python bench.py --dtype $d --steps 3 --warmup 2 --no-bf16-extra > $OUT/pmc_$d.log 2>&1 || { tail -20 $OUT/pmc_$d.log; exit 1; }
  python tools/pmc_summary.py $OUT/pmc_$d --label $d > $OUT/r6_pmc_lds_$d.jsonl
  rm -rf $OUT/pmc_$d
  python - "$OUT/r6_pmc_lds_$d.jsonl" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
rows.sort(key=lambda r: -r.get('GRBM_GUI_ACTIVE', 0) * r['dispatches'])
for r in rows[:10]:
    busy = max(r.get('SQ_BUSY_CYCLES', 1), 1)
    wave = max(r.get('SQ_WAVE_CYCLES', 1), 1)
    print(r['label'], r['kernel'][:48], r['dispatches'], 'mfma_util %s' % r.get('mfma_util'), 'wait_frac %s' % r.get('wait_frac'),
          'lds_active %.3f' % (r.get('SQ_LDS_IDX_ACTIVE', 0) / busy), 'lds_fifo_full %.3f' % (r.get('SQ_LDS_DATA_FIFO_FULL', 0) / busy),
          'wait_inst_lds/wave %.3f' % (r.get('SQ_WAIT_INST_LDS', 0) / wave),
          'bank_conf %.3f' % (r.get('SQ_LDS_BANK_CONFLICT', 0) / busy))
PY
done
