#!/bin/bash
# GPU parity suite (one process, per-test timeout) + smoke. Stops at the first crash-class exit.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal exit class, stopping"; exit $rc; fi
  return 0
}
step pytest_gpu 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
