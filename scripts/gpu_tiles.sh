#!/bin/bash
# conv tile sweep (+ the conv numerics tests first, so a bad variant never gets timed)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "conv" > gpurun_out/tiles_tests.log 2>&1 || { tail -30 gpurun_out/tiles_tests.log; exit 1; }
tail -2 gpurun_out/tiles_tests.log
timeout -k 10 400 python tools/microbench/conv_tiles.py --shapes ${SHAPES:-s3_3x3,s3_1x1a,s3_1x1b,s2_3x3,s2_1x1a,s2_1x1b,rpn_3x3,s4_3x3,s4_1x1a,s4_1x1b} --tiles ${TILES:-0,23,24,25} --splits ${SPLITS:-0,1,2} > gpurun_out/tiles.log 2>&1
rc=$?; grep -v Warn gpurun_out/tiles.log; exit $rc
