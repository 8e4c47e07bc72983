#!/bin/bash
# Round 4: rocprofv3 kernel traces of C5 and C3 with the 16-slot pattern memo.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r04_q
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
step trace_c5 200 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 --output-format csv -- python3 bench.py --config c5 --steps 10 --warmup 2 --cpu-sample 0
step trace_c3 200 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 --output-format csv -- python3 bench.py --config c3 --steps 10 --warmup 2 --cpu-sample 0
rm -f $O/prof_*/*_kernel_trace.csv
exit 0
