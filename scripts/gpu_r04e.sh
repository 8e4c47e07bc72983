#!/bin/bash
# Round 4: LEAN5 scan records carry the pod's failing versioned checks (computed once by the
# summary pass). LEAN parity + digest tests, report-fixture messages, C2 benches, kernel trace.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r04_e}
O=gpurun_out/$TAG
mkdir -p $O
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-3} "$O/$name.log" | cut -c1-400
  [ $rc -ne 0 ] && exit $rc
  return 0
}
TAILN=6 step pytest_lean 600 python -u -m pytest tests/test_psum.py tests/test_gpu_lean.py tests/test_pattern_messages.py -m gpu -x -q --timeout 300 --timeout-method thread
step bench_c2_k20 300 python bench.py --steps 20 --warmup 5
step bench_c2_k200 300 python bench.py --steps 200 --warmup 20 --cpu-sample 0
step trace_c2 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-sample 0
for f in $O/bench_*.log; do grep '^{' $f > ${f%.log}.json || true; done
exit 0
