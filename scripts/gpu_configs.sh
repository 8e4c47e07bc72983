#!/bin/bash
# Round 2: C3 / C5 parity on the GPU, bench lines for c2 / c3 / c5, rocprofv3 kernel traces of
# the c3 / c5 runs (scan + pattern kernels). Stops at the first crash-class exit.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal exit class, stopping"; exit $rc; fi
  return 0
}
step pytest_configs 900 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread
step bench_c2 300 python bench.py --steps 100 --warmup 10 --cpu-sample 0
step bench_c3 300 python bench.py --config c3 --steps 10 --warmup 2 --cpu-sample 0
step bench_c5 300 python bench.py --config c5 --steps 10 --warmup 2 --cpu-sample 0
step prof_c5 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 --output-format csv -- python3 bench.py --config c5 --steps 10 --warmup 2 --cpu-sample 0
step prof_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o c3 --output-format csv -- python3 bench.py --config c3 --steps 10 --warmup 2 --cpu-sample 0
