#!/bin/bash
# Round 4: pattern kernel without the inline deep re-walk (KPE_DEEP_ cells go to
# kpe_pattern_deep_kernel, on a 14-frame LDS stack): pattern parity tests, C5 / C3 benches
# (LDS stack depth 6 default, 4 / 5 via KPE_LIB variant builds), traces and traffic passes.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r04_m}
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
TAILN=4 step pytest_pat 500 python -u -m pytest tests/test_gpu_pattern.py tests/test_gpu_configs.py tests/test_pattern_vars.py tests/test_pattern_messages.py tests/test_conditions_device.py -m gpu -x -q --timeout 300 --timeout-method thread
for c in c5 c3; do
  step bench_$c 200 python bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0
  for v in ; do
    step ${c}_$v 200 env KPE_LIB=kyverno_amd/build/diag/libkpe_$v.so python bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0
  done
  step trace_$c 200 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o $c --output-format csv -- python3 bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0
  for k in fetch write; do
    K=$(echo $k | tr a-z A-Z)_SIZE
    step ${c}pmc_$k 150 rocprofv3 --pmc $K -d $O/$c/prof_pmc_$k -o pmc_$k --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --cpu-sample 0
  done
done
for f in $O/bench_*.log $O/c*_d?.log; do grep '^{' $f > ${f%.log}.json || true; done
exit 0
