#!/bin/bash
# Round 4 full GPU parity suite (every -m gpu test) and smoke().
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r04_h}
O=gpurun_out/$TAG
mkdir -p $O
echo "== smoke ($(date +%T))"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
echo "== pytest_gpu ($(date +%T))"
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "== pytest_gpu rc=$rc"; tail -15 $O/pytest_gpu.log
exit $rc
