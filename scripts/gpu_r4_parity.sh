#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for m in rpn rcnn; do
  echo "== $m" >> gpurun_out/r4_parity_probe.txt
  timeout -k 10 500 python -u tools/parity_probe.py --mode $m >> gpurun_out/r4_parity_probe.txt 2>&1 || { tail -20 gpurun_out/r4_parity_probe.txt; exit 1; }
done
grep -E "==|median" gpurun_out/r4_parity_probe.txt | cut -c1-200
