#!/bin/bash
# fused FC weight update (VGG16 fc6 / fc7): tests, then VGG16 step A/B (MXR_FUSED_FC_SGD=1 vs 0) at
# the three precisions and a kernel trace of the fused bf16 step -> gpurun_out/r5/fcsgd_*
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r5; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r5"
timeout -k 10 600 python -u -m pytest tests/test_fused_fc_sgd.py tests/test_model.py tests/test_dgrad_bt.py -m gpu -x -v \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/fcsgd_tests.log 2>&1 || { tail -40 $OUT/fcsgd_tests.log; exit 1; }
tail -2 $OUT/fcsgd_tests.log
V="--network vgg16 --image 600x1000 --num-classes 21 --steps 60 --warmup 5"
for arm in 1 0 1 0; do
  MXR_FUSED_FC_SGD=$arm timeout -k 10 400 python bench.py $V > $OUT/fcsgd_ab_$arm.log 2>&1 || { tail -20 $OUT/fcsgd_ab_$arm.log; exit 1; }
  echo "fused=$arm $(grep '^{' $OUT/fcsgd_ab_$arm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c["bf16x3"]["value"], c["bf16"]["value"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fcsgd_prof -o run -- \
  python bench.py --network vgg16 --image 600x1000 --num-classes 21 --steps 10 --warmup 3 --dtype bf16 --no-bf16-extra \
  > $OUT/fcsgd_prof.log 2>&1 || { tail -20 $OUT/fcsgd_prof.log; exit 1; }
T=$(find $OUT/fcsgd_prof -name '*kernel_trace.csv' | head -1)
python tools/trace_groups.py "$T" --steps 10 --top 40 > $OUT/fcsgd_bf16_groups.txt 2>&1
head -14 $OUT/fcsgd_bf16_groups.txt | cut -c1-150
rm -rf $OUT/fcsgd_prof
