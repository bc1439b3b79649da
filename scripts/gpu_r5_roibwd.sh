#!/bin/bash
# RoI-pool backward channels-per-workgroup A/B (MXR_ROI_BWD_CW=4 / 2 / 1) in the fp32 step trace
# (round 5: 122 / 220 / 221 us; the knob was removed afterwards, 4 channels stay)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r5; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r5"
timeout -k 10 300 python -u -m pytest tests/test_kernels.py -k "roi" -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/roibwd_tests.log 2>&1 || { tail -30 $OUT/roibwd_tests.log; exit 1; }
tail -1 $OUT/roibwd_tests.log
for cw in 4 2 1; do
  MXR_ROI_BWD_CW=$cw timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/roibwd_$cw -o run -- \
    python bench.py --steps 10 --warmup 3 --dtype fp32 --no-bf16-extra > $OUT/roibwd_$cw.log 2>&1 || { tail -20 $OUT/roibwd_$cw.log; exit 1; }
  S=$(find $OUT/roibwd_$cw -name '*kernel_stats.csv' | head -1)
  echo "cw=$cw $(python -c "import csv,sys; [print(r['Name'][:40], r['Calls'], r['AverageNs']) for r in csv.DictReader(open('$S')) if 'roi_pool_bwd' in r['Name']]")"
  rm -rf $OUT/roibwd_$cw
done
