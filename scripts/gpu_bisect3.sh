#!/bin/bash
# The graph test body outside pytest, then under pytest without the timeout plugin.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -3 "$OUT/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run t_direct 120 python -c "import sys, torch; sys.path.insert(0, '.'); from tests import test_model as t; t.test_e2e_step_gpu_graph(torch.device('cuda', 0)); print('direct OK')"
run t_pytest_plain 120 python -u -m pytest tests/test_model.py -m gpu -x -q -p no:cacheprovider -p no:timeout
