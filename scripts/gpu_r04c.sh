#!/bin/bash
# Round 4, multi-shard LEAN5 pass: the LEAN5 parity tests (batch launches included), the C2
# bench at the driver's K=20 and at K=200, a rocprofv3 kernel trace, and the FETCH_SIZE /
# WRITE_SIZE passes of kpe_lean5_batch_kernel (every launch 20 shards: --replicas 20 --steps 20)
# (scripts/pmc_summary.py turns them into profiles/<tag> and perf/pmc_traffic_c2.json).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r04_c}
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
TAILN=12 step pytest_lean 600 python -u -m pytest tests/test_gpu_lean.py tests/test_psum.py -m gpu -x -v --timeout 300 --timeout-method thread
step bench_c2_k20 300 python bench.py --steps 20 --warmup 5
step bench_c2_k200 300 python bench.py --steps 200 --warmup 20 --cpu-sample 0
step trace_c2 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-sample 0
for k in fetch write; do
  K=$(echo $k | tr a-z A-Z)_SIZE
  step pmc_$k 180 rocprofv3 --pmc $K -d $O/prof_pmc_$k -o pmc_$k --output-format csv -- python3 bench.py --steps 20 --replicas 20 --warmup 2 --cpu-sample 0
done
# summarised here afterwards: CFG=c2 python3 scripts/pmc_summary.py gpurun_out/$TAG <profiles tag>
for f in $O/bench_*.log; do grep '^{' $f > ${f%.log}.json || true; done
exit 0
