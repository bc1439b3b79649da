#!/bin/bash
# Replays the graph test's configuration knobs one at a time (stops at the first crash).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -3 "$OUT/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
MXR_BISECT_GTPAD=1 run b_gtpad 120 python tools/capture_bisect.py graphed
export MXR_BISECT_GTPAD=0
MXR_BISECT_POST=300 run b_post300 120 python tools/capture_bisect.py graphed
MXR_BISECT_PRE=800 MXR_BISECT_POST=300 run b_pre800 120 python tools/capture_bisect.py graphed
