#!/bin/bash
# One GPU-box session: tests, bench, rocprof.  Each GPU step has its own time limit; a crash,
# abort, fault or timeout (rc not in {0,1}) ends the session immediately.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-all}
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[gpu_check] $name: $*" | tee -a gpurun_out/gpu_check.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[gpu_check] $name rc=$rc" | tee -a gpurun_out/gpu_check.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_check] stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
python -c "import torch; print(torch.cuda.get_device_name(0))" || exit 2
if [[ $STEPS == *tests* || $STEPS == all ]]; then
  run pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
fi
if [[ $STEPS == *bench* || $STEPS == all ]]; then
  run bench_graph 600 python bench.py --steps 20 --warmup 5
  run bench_eager 600 python bench.py --steps 10 --warmup 3 --mode eager
fi
if [[ $STEPS == *prof* || $STEPS == all ]]; then
  run rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
      python bench.py --steps 5 --warmup 2 --mode eager
fi
echo "[gpu_check] done"
