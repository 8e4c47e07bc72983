#!/bin/bash
# Array sites (KPE_SITES=1): pattern parity tests, then C5 / C3 kernel traces per build variant.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pattern.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/sg_tests.log 2>&1
rc=$?; tail -4 gpurun_out/sg_tests.log; [ $rc -ne 0 ] && exit $rc
export KPE_SITES=1
VARIANTS="${VARIANTS:-sg4 sg3 sg2}" bash scripts/gpu_r03f.sh
