#!/bin/bash
# Pattern-kernel A/B on C5 and C3: the default build and the libraries in build/diag (KPE_LIB).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pattern.py tests/test_gpu_configs.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pat_tests.log 2>&1
rc=$?; tail -2 gpurun_out/pat_tests.log; [ $rc -ne 0 ] && exit $rc
for c in c5 c3; do
  for lib in kyverno_amd/libkpe.so kyverno_amd/build/diag/libkpe_*.so; do
    [ -e "$lib" ] || continue
    KPE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/pat_ab.log 2>&1 || { tail -3 gpurun_out/pat_ab.log; exit 1; }
    echo "$c $(basename $lib): $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/pat_ab.log | head -1)"
  done
done
