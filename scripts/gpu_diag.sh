#!/bin/bash
# One gpurun call: GPU parity tests, then the diagnostic variant timings.
# Stops at a crash/timeout-class exit (>= 124); a plain test failure still times.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q --timeout 300 > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest.log
[ $rc -ge 124 ] && exit $rc
bash scripts/diag_variants.sh
