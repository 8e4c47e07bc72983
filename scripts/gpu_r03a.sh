#!/bin/bash
# Round-3 first evidence: -m gpu suite + smoke, then the default C2 bench.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step pytest_gpu 800 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 300 python bench.py
for v in base d512 d1024; do
  lib=kyverno_amd/libkpe.so; [ $v != base ] && lib=kyverno_amd/build/diag/libkpe_$v.so
  KPE_LIB=$PWD/$lib step pat_c5_$v 200 python bench.py --config c5 --steps 10 --warmup 2 --cpu-sample 0
done
exit 0
