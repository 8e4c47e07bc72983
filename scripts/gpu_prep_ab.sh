#!/bin/bash
# GPU tests, then the C2 bench with and without the per-evaluation prologue image.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n ${TAILN:-6} "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal exit class, stopping"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step bench_prep 300 python bench.py --steps 200 --warmup 20 --cpu-sample 0
KPE_NO_PREP=1 step bench_noprep 300 python bench.py --steps 200 --warmup 20 --cpu-sample 0
