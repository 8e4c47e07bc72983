#!/bin/bash
# Round 4: the pattern kernel's memo slots (32 default / 16 via a KPE_LIB variant build: 2 KiB less
# LDS per block, 8 resident blocks per CU instead of 7): C5 / C3 benches.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r04_o}
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
  step ${c}_base 200 python bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0
  for v in m16; do
    step ${c}_$v 200 env KPE_LIB=kyverno_amd/build/diag/libkpe_$v.so python bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0
  done
done
for f in $O/c*_*.log; do grep '^{' $f > ${f%.log}.json || true; done
exit 0
