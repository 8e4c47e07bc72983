#!/bin/bash
# Round 4: memo-16 default: GPU pattern / parity tests, smoke, C5 / C3 benches.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r04_p
mkdir -p $O
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 1 "$O/$name.log" | cut -c1-200
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step c5 200 python bench.py --config c5 --steps 20 --warmup 3 --cpu-sample 0
step c3 200 python bench.py --config c3 --steps 20 --warmup 3 --cpu-sample 0
for f in $O/c*.log; do grep '^{' $f > ${f%.log}.json || true; done
exit 0
