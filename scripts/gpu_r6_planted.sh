#!/bin/bash
# Round 6: planted-object detectors trained at fp32 (train_end2end.py, ResNet-101 / VGG16), each
# checkpoint then scored by test.py --has_rpn on held-out images (seed 1000) at --dtype fp32 (the
# reference's precision, three-plane operands on our kernels) and --dtype bf16.  NETS picks a subset.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r6; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r6"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
for net in ${NETS:-resnet101 vgg16}; do
  P=/tmp/pl_$net/e2e
  run planted_${net}_train 900 python train_end2end.py --synthetic ${PIMGS:-1024} --synthetic-kind planted \
      --synthetic-shape 600x1000 --network $net --num-classes 8 --max-steps ${PSTEPS:-16000} --frequent 500 \
      --pretrained none --lr 0.005 --factor-step ${FSTEP:-12000} --prefix $P --num_epoch 100
  E=$(ls $P-*.params | sed 's/.*-0*\([0-9]*\)\.params/\1/' | sort -n | tail -1)
  for dt in fp32 bf16; do
    run planted_${net}_test_$dt 600 python test.py --prefix $P --epoch $E --synthetic 100 --synthetic-kind planted \
        --synthetic-shape 600x1000 --seed 1000 --network $net --num-classes 8 --has_rpn --dtype $dt
  done
done
