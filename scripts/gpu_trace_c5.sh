#!/bin/bash
# Kernel trace of a short C5 (and C3) bench: per-kernel means (rocprofv3 --kernel-trace --stats).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${CFGS:-c5 c3}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$c -o $c --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/tr_$c.log 2>&1 || exit $?
  f=$(find gpurun_out/tr_$c -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -8
done
