#!/bin/bash
# round-6 check: full GPU test tier (without -x: every failure listed), smoke, headline bench
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r6; export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r6"
timeout -k 10 1000 python -u -m pytest tests -m gpu ${XFLAG:-} -q -p no:cacheprovider --timeout 150 --timeout-method thread \
  > $OUT/full_tests.log 2>&1
rc=$?
tail -8 $OUT/full_tests.log
grep -E "^FAILED|^ERROR" $OUT/full_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log
