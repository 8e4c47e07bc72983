#!/bin/bash
# Round 4: multi-shard LEAN5 with tiles per wave, selector requirement masks (C4), the pattern
# kernel's leaf table (C3 / C5). Parity tests, C2 / C4 / C5 / C3 benches, rocprofv3 traces, FETCH_SIZE / WRITE_SIZE passes of both dominant kernels.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r04_d}
O=gpurun_out/$TAG
mkdir -p $O
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-3} "$O/$name.log" | cut -c1-400
  [ $rc -ne 0 ] && exit $rc
  return 0
}
TAILN=6 step pytest_sel 600 python -u -m pytest tests/test_gpu_lean.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread
TAILN=6 step pytest_pat 400 python -u -m pytest tests/test_gpu_pattern.py tests/test_gpu_configs.py tests/test_pattern_vars.py -m gpu -x -q --timeout 300 --timeout-method thread
step bench_c5 200 python bench.py --config c5 --steps 20 --warmup 3 --cpu-sample 0
step bench_c3 200 python bench.py --config c3 --steps 20 --warmup 3 --cpu-sample 0
step bench_c2_k20 300 python bench.py --steps 20 --warmup 5
step bench_c2_k200 300 python bench.py --steps 200 --warmup 20 --cpu-sample 0
step bench_c4 300 python bench.py --config c4 --steps 20 --warmup 3 --cpu-sample 0
step trace_c2 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-sample 0
step trace_c4 300 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o c4 --output-format csv -- python3 bench.py --config c4 --steps 10 --warmup 2 --cpu-sample 0
for k in fetch write; do
  K=$(echo $k | tr a-z A-Z)_SIZE
  step pmc_$k 180 rocprofv3 --pmc $K -d $O/prof_pmc_$k -o pmc_$k --output-format csv -- python3 bench.py --steps 20 --replicas 20 --warmup 2 --cpu-sample 0
  step c4pmc_$k 180 rocprofv3 --pmc $K -d $O/c4/prof_pmc_$k -o pmc_$k --output-format csv -- python3 bench.py --config c4 --steps 4 --warmup 1 --cpu-sample 0
done
for f in $O/bench_*.log; do grep '^{' $f > ${f%.log}.json || true; done
exit 0
