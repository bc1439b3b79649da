#!/bin/bash
# Round 5: new GPU tests, CLI training throughput vs bench (raw uint8 images on/off), and the
# planted-object detector runs: train_end2end.py (ResNet-101 / VGG16, fp32) then test.py --has_rpn
# on held-out images (another seed).  STAGES picks a subset (default all).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r5; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r5"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
ST=${STAGES:-tests cli planted_r101 planted_vgg}
for s in $ST; do case $s in
tests)
  run newtests 400 python -u -m pytest tests/test_image_prep.py tests/test_kernels.py tests/test_model.py -m gpu -q \
      -p no:cacheprovider --timeout 200 --timeout-method thread -k "image_prep or nonfinite or overlapped" ;;
cli)
  run cli_e2e_raw 400 python train_end2end.py --synthetic 64 --synthetic-shape 800x1333 --network resnet101 \
      --num-classes 81 --max-steps 400 --frequent 50 --pretrained none --prefix /tmp/cli/e2e --num_epoch 10
  MXR_RAW_IMAGES=0 run cli_e2e_hostfloat 400 python train_end2end.py --synthetic 64 --synthetic-shape 800x1333 \
      --network resnet101 --num-classes 81 --max-steps 200 --frequent 50 --pretrained none --prefix /tmp/cli2/e2e --num_epoch 10 ;;
planted_r101)
  run planted_r101_train 900 python train_end2end.py --synthetic ${PIMGS:-256} --synthetic-kind planted --synthetic-shape 600x1000 \
      --network resnet101 --num-classes 8 --max-steps ${PSTEPS:-4000} --frequent 100 --pretrained none --lr 0.005 \
      --factor-step ${FSTEP:-3000} --prefix /tmp/pl_r101/e2e --num_epoch 100
  E=$(ls /tmp/pl_r101/e2e-*.params | sed 's/.*-0*\([0-9]*\)\.params/\1/' | sort -n | tail -1)
  run planted_r101_test 600 python test.py --prefix /tmp/pl_r101/e2e --epoch $E --synthetic 100 --synthetic-kind planted \
      --synthetic-shape 600x1000 --seed 1000 --network resnet101 --num-classes 8 --has_rpn ;;
planted_vgg)
  run planted_vgg_train 900 python train_end2end.py --synthetic ${PIMGS:-256} --synthetic-kind planted --synthetic-shape 600x1000 \
      --network vgg16 --num-classes 8 --max-steps ${PSTEPS:-4000} --frequent 100 --pretrained none --lr 0.005 \
      --factor-step ${FSTEP:-3000} --prefix /tmp/pl_vgg/e2e --num_epoch 100
  E=$(ls /tmp/pl_vgg/e2e-*.params | sed 's/.*-0*\([0-9]*\)\.params/\1/' | sort -n | tail -1)
  run planted_vgg_test 600 python test.py --prefix /tmp/pl_vgg/e2e --epoch $E --synthetic 100 --synthetic-kind planted \
      --synthetic-shape 600x1000 --seed 1000 --network vgg16 --num-classes 8 --has_rpn ;;
esac; done
