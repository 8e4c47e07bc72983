#!/bin/bash
# Round 4: LDS frame-stack depth of the main pattern kernel (6 default / 5 / 4 via KPE_LIB variant
# builds) now that deep walks go to kpe_pattern_deep_kernel through doc_perm: C5 / C3 benches.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r04_n}
O=gpurun_out/$TAG
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
for c in c5 c3; do
  step ${c}_d6 200 python bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0
  for v in d5 d4; do
    step ${c}_$v 200 env KPE_LIB=kyverno_amd/build/diag/libkpe_$v.so python bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0
  done
done
for f in $O/c*_d?.log; do grep '^{' $f > ${f%.log}.json || true; done
exit 0
