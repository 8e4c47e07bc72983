#!/bin/bash
# Round-3 evidence on one MI355X, everything under gpurun_out/$TAG: the -m gpu suite + smoke, the
# default C2 bench (CPU baseline included), C3 / C4 / C5 benches, a 2-rank functional run of the
# sharded path (gloo collectives, one device), and rocprofv3 kernel traces of C3 / C5.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r03_final}
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
[ -n "$SKIP_TESTS" ] || TAILN=12 step pytest_gpu 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
[ -n "$SKIP_TESTS" ] || step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 300 python bench.py
for c in c3 c4 c5; do step bench_$c 400 python bench.py --config $c --steps 20 --warmup 3; done
step bench_ranks2 300 env KPE_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 --cpu-sample 0
for c in c3 c5; do
  step trace_$c 240 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o $c --output-format csv -- python3 bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0
done
for f in $O/bench_*.log; do grep '^{' $f > ${f%.log}.json || true; done
exit 0
