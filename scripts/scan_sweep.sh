#!/bin/bash
# Scan-kernel scaling experiment: kernel time (HIP events, single stream) vs rows per launch
# and vs scan blocks per CU (KPE_SCAN_BPC). Output: gpurun_out/sweep.log
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
out=gpurun_out/sweep.log
: > $out
one() {  # one <label> <env...> -- <bench args>
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 120 python3 bench.py --steps 60 --warmup 6 --cpu-sample 0 "$@" > gpurun_out/sweep_one.log 2>&1 || { echo "$label FAILED rc=$?" >> $out; tail -5 gpurun_out/sweep_one.log >> $out; return 1; }
  python3 - "$label" >> $out <<'PY'
import json, sys
l = [x for x in open("gpurun_out/sweep_one.log") if x.startswith("{")][-1]
d = json.loads(l); r = d["roofline"]
print(f'{sys.argv[1]:24s} rows={d["config"]["resources_per_gpu"]:>8} step_us={d["ms_per_step"]*1e3:7.2f} '
      f'kernel_us={r["kernel_ms"]*1e3:7.2f} alg_MB={r["alg_bytes_per_launch"]/1e6:6.1f} frac={r["frac"]:.3f}')
PY
}
for n in ${ROWS:-250000 500000 1000000 2000000 3000000}; do one "rows" KPE_X=1 -- --resources $n --replicas 2 || exit 1; done
for b in ${BPCS:-1 2 3 4 5 6}; do one "bpc=$b" KPE_SCAN_BPC=$b -- --replicas 2 || exit 1; done
cat $out
