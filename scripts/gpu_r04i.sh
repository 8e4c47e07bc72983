#!/bin/bash
# Round 4: every config's bench line on the current build, the pattern kernel's lanes-per-row
# A/B (KPE_PAT_SPLIT 1 / 2 / 4 via KPE_LIB variant builds), rocprofv3 kernel traces, and the
# FETCH_SIZE / WRITE_SIZE passes of C4's scan and C5 / C3's pattern kernel.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r04_i}
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
step bench_c2 300 python bench.py
for c in c3 c4 c5; do
  step bench_$c 200 python bench.py --config $c --steps 20 --warmup 3
done
for v in s2 s4; do
  for c in c5 c3; do
    step ${c}_$v 200 env KPE_LIB=kyverno_amd/build/diag/libkpe_$v.so python bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0
  done
done
for c in c3 c4 c5; do
  step trace_$c 200 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o $c --output-format csv -- python3 bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0
done
for c in c4 c5 c3; do
  for k in fetch write; do
    K=$(echo $k | tr a-z A-Z)_SIZE
    step ${c}pmc_$k 150 rocprofv3 --pmc $K -d $O/$c/prof_pmc_$k -o pmc_$k --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --cpu-sample 0
  done
done
for f in $O/bench_*.log $O/c*_s*.log; do grep '^{' $f > ${f%.log}.json || true; done
exit 0
