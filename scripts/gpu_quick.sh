#!/bin/bash
# Quick GPU loop: PSS parity tests, then the C2 bench (no CPU baseline).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_pssx.py tests/test_gpu_configs.py} -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quick_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-sample 0 ${BENCH_ARGS:-} > gpurun_out/quick_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/quick_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value %.3g step_us %.2f scan_us %.2f frac %.3f dict_us %.2f single %.2f' % (d['value'], d['ms_per_step']*1e3, r['kernel_ms']*1e3, r['frac'], r['dict_kernel_ms']*1e3, r['single_stream_step_ms']*1e3))"
exit $rc
