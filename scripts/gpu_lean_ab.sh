#!/bin/bash
# LEAN scan A/B: PSS parity tests with the default kernel, then scan-kernel time (events, C2 1M)
# for the default build, the persistent kernel (KPE_LEAN_PERSIST) and the KPE_LEAN_T variants.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
[ "$TESTS" = none ] || timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_configs.py} -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; [ "$TESTS" = none ] || { tail -3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc; }
: > gpurun_out/ab.jsonl
for i in 1 2; do
  timeout -k 10 120 python3 scripts/diag_time.py >> gpurun_out/ab.jsonl 2> gpurun_out/ab_err.log || exit $?
  KPE_LEAN_PERSIST=1 timeout -k 10 120 python3 scripts/diag_time.py | sed 's/"lib": "libkpe.so"/"lib": "persist"/' >> gpurun_out/ab.jsonl 2>> gpurun_out/ab_err.log || exit $?
  for lib in kyverno_amd/build/diag/libkpe_*.so; do [ -e "$lib" ] || continue
    KPE_LIB=$PWD/$lib timeout -k 10 120 python3 scripts/diag_time.py >> gpurun_out/ab.jsonl 2>> gpurun_out/ab_err.log || exit $?
  done
done
cat gpurun_out/ab.jsonl
[ -n "$PAT" ] || exit 0
for c in c5 c3; do
  timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/ab_$c.log 2>&1 || exit $?
  echo "$c perm: $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/ab_$c.log | head -1) step_ms $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$c.log)"
  KPE_NO_PERM=1 timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/ab_${c}_noperm.log 2>&1 || exit $?
  echo "$c noperm: $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/ab_${c}_noperm.log | head -1)"
done
