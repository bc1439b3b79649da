#!/bin/bash
# round-5 check: full GPU test tier (-x, as the driver runs it), smoke, headline bench
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/r5_full_tests.log 2>&1 || { tail -60 gpurun_out/r5_full_tests.log; exit 1; }
tail -3 gpurun_out/r5_full_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke.log 2>&1 || { tail -20 gpurun_out/r5_smoke.log; exit 1; }
tail -1 gpurun_out/r5_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r5_bench.log 2>&1 || { tail -20 gpurun_out/r5_bench.log; exit 1; }
grep '^{' gpurun_out/r5_bench.log
