#!/bin/bash
# A build variant (kyverno_amd/build/var/libkpe_$V.so): pattern parity tests through it, then the
# C5 / C3 benches.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export KPE_LIB=$PWD/kyverno_amd/build/var/libkpe_${V:-single}.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_pattern.py tests/test_pattern_messages.py tests/test_gpu_configs.py tests/test_pattern_vars.py tests/test_conditions_device.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/var_tests.log 2>&1
rc=$?; tail -4 gpurun_out/var_tests.log; [ $rc -ne 0 ] && exit $rc
for c in c5 c3; do
  timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/var_$c.log 2>&1 || exit $?
  grep '^{' gpurun_out/var_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c', 'kernel_ms %.4f' % r['kernel_ms'])"
done
