#!/bin/bash
# full GPU test suite + smoke + headline bench (+ extras) + bf16 determinism A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread \
  > gpurun_out/full_tests.log 2>&1 || { tail -60 gpurun_out/full_tests.log; exit 1; }
grep -E "FAILED|passed|failed" gpurun_out/full_tests.log | tail -12
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full_smoke.log 2>&1 || { tail -20 gpurun_out/full_smoke.log; exit 1; }
tail -1 gpurun_out/full_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/full_bench.log 2>&1 || { tail -20 gpurun_out/full_bench.log; exit 1; }
grep '^{' gpurun_out/full_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["dtype"], {k: c[k]["value"] for k in ("bf16x3","bf16") if k in c})'
for m in det nondet; do
  env $( [ $m = nondet ] && echo MXR_NONDETERMINISTIC=1 || echo X=1 ) timeout -k 10 200 python bench.py --dtype bf16 --steps 40 --warmup 5 > gpurun_out/full_bf16_$m.log 2>&1 || exit 1
  echo "bf16_$m $(grep '^{' gpurun_out/full_bf16_$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
