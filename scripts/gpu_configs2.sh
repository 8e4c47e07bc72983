#!/bin/bash
# C3 / C4 / C5 bench lines (no CPU baseline), one process each.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${CFGS:-c3 c4 c5}; do
  timeout -k 10 400 python bench.py --config $c --steps 50 --warmup 5 --cpu-sample 0 > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "== $c rc=$rc"
  grep '^{' gpurun_out/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value %.3g step_ms %.3f scan_ms %.3f pat_ms %.3f frac %.3f' % (d['value'], d['ms_per_step'], r['kernel_ms'], r['pattern_kernel_ms'], r['frac']))"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_$c.log; exit $rc; }
done
exit 0
