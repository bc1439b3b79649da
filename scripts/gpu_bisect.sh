#!/bin/bash
# hipGraph capture bisect: one stage per process, stops at the first crash.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -3 "$OUT/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
for s in ${STAGES:-trunk_fwd trunk_fwdbwd rpn_fwdbwd e2e_fwd e2e_fwdbwd step}; do run bisect_$s 120 python tools/capture_bisect.py $s; done
