#!/bin/bash
# One gpurun call: build check, GPU parity tests, smoke, short bench.
# Stops at the first crash/timeout-class exit (124/134/137/139 or >128); a plain
# test failure (exit 1) still lets the bench run so we get numbers.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal exit class, stopping"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py ${BENCH_ARGS:---steps 100 --warmup 10}
