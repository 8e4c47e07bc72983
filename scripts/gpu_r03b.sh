#!/bin/bash
# Pattern-kernel round: -m gpu suite, then C5 / C3 benches with the LDS-staged kernel and the
# lane-per-row kernel (KPE_PAT_LANE) for comparison.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-4} "gpurun_out/$name.log" | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  return 0
}
summ() { grep '^{' "gpurun_out/$1.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$1', 'step_ms %.4f' % d['ms_per_step'], r.get('kernel'), 'kernel_ms %.4f' % r['kernel_ms'], 'frac %.4f' % r['frac'])"; }
[ -n "$SKIP_TESTS" ] || TAILN=12 step pytest_gpu 800 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread ${PYTEST_ARGS:-}
for c in c5 c3; do
  step bench_$c 200 python bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0 && summ bench_$c
  KPE_PAT_LANE=1 step bench_${c}_lane 200 python bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0 && summ bench_${c}_lane
done
exit 0
