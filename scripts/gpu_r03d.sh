#!/bin/bash
# C2 evidence: LEAN variant A/B (scripts/lean_ab.sh), then rocprofv3 kernel trace + PMC passes of
# the default C2 bench (scripts/profile.sh), summarised into profiles/$TAG.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03_c2}
[ -n "$SKIP_AB" ] || { timeout -k 10 900 bash scripts/lean_ab.sh || exit $?; }
BENCH_ARGS="--steps 100 --warmup 10 --cpu-sample 0" timeout -k 10 900 bash scripts/profile.sh || exit $?
python3 scripts/pmc_summary.py gpurun_out $TAG > gpurun_out/pmc_summary.log 2>&1; tail -30 gpurun_out/pmc_summary.log
mkdir -p gpurun_out/$TAG && cp -r profiles/$TAG/* gpurun_out/$TAG/ && cp perf/pmc_traffic_c2.json gpurun_out/$TAG/
exit 0
