#!/bin/bash
# Round 4: C4 wide-scan occupancy A/B (KPE_SCAN_WAVES 7 default / 6 / 5 via KPE_LIB variant
# builds: spills vs residency), WRITE_SIZE of each, and the substituted pattern-message test.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r04_f}
O=gpurun_out/$TAG
mkdir -p $O
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-3} "$O/$name.log" | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  return 0
}
TAILN=4 step pytest_msg 300 python -u -m pytest tests/test_pattern_messages.py -m gpu -x -q --timeout 200 --timeout-method thread -k "substituted or report_fixture"
step c4_w7 200 python bench.py --config c4 --steps 20 --warmup 3 --cpu-sample 0
for w in w6 w5; do
  step c4_$w 200 env KPE_LIB=kyverno_amd/build/diag/libkpe_$w.so python bench.py --config c4 --steps 20 --warmup 3 --cpu-sample 0
done
step c4pmc_w7 120 rocprofv3 --pmc WRITE_SIZE -d $O/w7 -o w7 --output-format csv -- python3 bench.py --config c4 --steps 4 --warmup 1 --cpu-sample 0
for f in $O/c4_*.log; do grep '^{' $f > ${f%.log}.json || true; done
exit 0
