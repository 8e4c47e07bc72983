#!/bin/bash
# Round 4 final pass on the final build: smoke, the whole -m gpu suite, every config's bench line
# (CPU baselines included) and rocprofv3 kernel traces of C2 and C5.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r04_final}
O=gpurun_out/$TAG
mkdir -p $O
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-1} "$O/$name.log" | cut -c1-200
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAILN=4 step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_c2 300 python bench.py
step bench_c2_k20 300 python bench.py --steps 20 --warmup 5 --cpu-sample 0
for c in c3 c4 c5; do
  step bench_$c 200 python bench.py --config $c --steps 20 --warmup 3
done
step trace_c2 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-sample 0
step trace_c5 200 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 --output-format csv -- python3 bench.py --config c5 --steps 10 --warmup 2 --cpu-sample 0
for f in $O/bench_*.log; do grep '^{' $f > ${f%.log}.json || true; done
exit 0
