#!/bin/bash
# One GPU session: -m gpu tests, C2 bench (new and template LEAN scan), C3/C5 pattern grid modes.
# Every GPU step has its own time limit; the script stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --cpu-sample 0 > gpurun_out/bench_c2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2.log | cut -c1-900
KPE_OLD_LEAN=1 timeout -k 10 200 python bench.py --cpu-sample 0 > gpurun_out/bench_c2_old.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2_old.log | cut -c 560-900
[ -n "$SKIP_PAT" ] && exit 0
for c in c5 c3; do
  timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/bench_$c.log 2>&1 || exit $?
  echo "$c rows: $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/bench_$c.log | head -1)"
  KPE_PAT_CELLS=1 timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/bench_${c}_cells.log 2>&1 || exit $?
  echo "$c cells: $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/bench_${c}_cells.log | head -1)"
done
