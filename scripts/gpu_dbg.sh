#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/debug_fused2.py > gpurun_out/debug_fused.log 2>&1; rc=$?; echo "rc=$rc"; cat gpurun_out/debug_fused.log | tail -40
