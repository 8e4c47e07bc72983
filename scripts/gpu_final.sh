#!/bin/bash
# Round-end evidence on one MI355X: -m gpu suite + smoke, the default C2 bench (with the CPU
# baseline), rocprofv3 trace + PMC passes of C2 (profiles/<TAG>, pmc_traffic_c2.json), traces of
# C3 / C5, and a 2-rank functional run of the sharded path on the one device (gloo collectives).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r02_final}
set -o pipefail
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -ne 0 ] && exit $rc
  return 0
}
[ -n "$SKIP_TESTS" ] || step pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
[ -n "$SKIP_TESTS" ] || step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 300 python bench.py
step bench_ranks2 300 env KPE_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 --cpu-sample 0
for c in c3 c4 c5; do
  step bench_$c 300 python bench.py --config $c --steps 10 --warmup 2
done
BENCH_ARGS="--steps 100 --warmup 10 --cpu-sample 0" bash scripts/profile.sh || exit $?
for c in c3 c5; do
  step trace_$c 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace_$c -o $c --output-format csv -- python3 bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0
done
exit 0
