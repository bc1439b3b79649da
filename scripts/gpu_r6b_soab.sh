#!/bin/bash
# same-box A/B of two builds of the extension: ab/_C_head.so (reference) vs the in-tree build
# ("new"); conv numerics tests on the new build first.  RUNS = bench arg sets separated by ';'.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/soab; export TMPDIR=/tmp
SO=mx_rcnn_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO ab/_C_new.so
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest ${TEST_FILES:-tests/test_kernels.py tests/test_fp32x2.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/soab/tests.log 2>&1 || { tail -30 gpurun_out/soab/tests.log; exit 1; }
  tail -1 gpurun_out/soab/tests.log
fi
IFS=';' read -ra SETS <<< "${RUNS:---steps 40 --warmup 5}"
for rep in 1 2; do
  for v in head new; do
    cp ab/_C_$v.so $SO
    for a in "${SETS[@]}"; do
      timeout -k 10 240 python bench.py $a > gpurun_out/soab/b.log 2>&1 || { tail -5 gpurun_out/soab/b.log; cp ab/_C_new.so $SO; exit 1; }
      echo "$v rep$rep [$a] $(grep '^{' gpurun_out/soab/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], (c.get("bf16x3") or {}).get("value"), (c.get("bf16") or {}).get("value"))')"
    done
  done
done
cp ab/_C_new.so $SO
