#!/bin/bash
# Round 4, first GPU pass: device PSA summary (digest + LEAN5 full matrices), the parity suite,
# the C2 bench with shards rotated past the Infinity Cache, and a rocprofv3 trace of it.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r04_a}
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
python3 -c "import bench, json; print(json.dumps(bench.cpu_budget()))" > $O/cpu_budget.json 2>&1
TAILN=12 step pytest_new 600 python -u -m pytest tests/test_psum.py tests/test_gpu_lean.py tests/test_exceptions.py tests/test_conditions_device.py tests/test_pattern_vars.py -m gpu -x -v --timeout 300 --timeout-method thread
step bench_c2 300 python bench.py --steps 200 --warmup 20
step bench_c2_k20 300 python bench.py --steps 20 --warmup 5 --cpu-sample 0
step trace_c2 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python3 bench.py --steps 200 --warmup 20 --cpu-sample 0
[ -n "$FULL" ] && TAILN=12 step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for f in $O/bench_*.log; do grep '^{' $f > ${f%.log}.json || true; done
exit 0
