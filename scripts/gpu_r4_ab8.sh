#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
V="--network vgg16 --image 600x1000 --num-classes 21"
ab() {
  local name=$1; shift
  local args=$1; shift
  env "$@" timeout -k 10 200 python bench.py $args --steps 40 --warmup 5 --no-bf16-extra > gpurun_out/ab8_$name.log 2>&1 || { tail -8 gpurun_out/ab8_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/ab8_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
ab vgg32 "$V" X=1 && ab vgg32_b4k "$V" MXR_SGD_BLOCKS=4096 && ab vgg32_b16k "$V" MXR_SGD_BLOCKS=16384 && ab vgg32_b1k "$V" MXR_SGD_BLOCKS=1024 && \
ab r101 "" X=1 && ab r101_b16k "" MXR_SGD_BLOCKS=16384 || exit 1
