#!/bin/bash
# Round 4 pattern-kernel pass: the pattern parity tests, C3 / C5 benches and rocprofv3 kernel
# traces of both.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r04_b}
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
TAILN=8 step pytest_pat 600 python -u -m pytest tests/test_gpu_pattern.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread
for c in c5 c3; do
  step bench_$c 400 python bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0
done
for c in c5 c3; do
  step trace_$c 300 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o $c --output-format csv -- python3 bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0
done
for f in $O/bench_*.log; do grep '^{' $f > ${f%.log}.json || true; done
exit 0
