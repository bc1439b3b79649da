#!/bin/bash
# fp32-class headline: a short bench (fp32 default + bf16 extra), then the whole GPU test tier.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT="$PWD/gpurun_out"
run() { local name=$1 t=$2; shift 2; echo "[r] $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "[r] $name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-1500; if [ $rc -ne 0 ]; then exit $rc; fi; }
run bench_fp32 400 python bench.py --steps 10 --warmup 3
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
