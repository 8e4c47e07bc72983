#!/bin/bash
# Pattern kernel with LDS frame stacks: parity tests, then C5 / C3 over build variants (KPE_LIB).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-2} "gpurun_out/$name.log" | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  return 0
}
summ() { grep '^{' "gpurun_out/$1.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$1', 'step_ms %.4f' % d['ms_per_step'], r.get('kernel'), 'kernel_ms %.4f' % r['kernel_ms'], 'frac %.4f' % r['frac'])"; }
[ -n "$SKIP_TESTS" ] || TAILN=25 step pat_tests 400 python -u -m pytest tests/test_gpu_pattern.py tests/test_pattern_messages.py tests/test_gpu_configs.py tests/test_pattern_vars.py -m gpu -q --timeout 200 --timeout-method thread
for v in ${VARIANTS:-base b128 s6 b128s6}; do
  for c in c5 c3; do
    KPE_LIB=$PWD/kyverno_amd/build/var/libkpe_$v.so step ${c}_$v 200 python bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0 && summ ${c}_$v
  done
done
exit 0
