#!/bin/bash
# PMC counters per program variant (scripts/exp_variants.py), one rocprofv3 pass per counter group.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d gpurun_out/pv_$name -o $name --output-format csv -- python3 scripts/exp_variants.py > gpurun_out/pv_$name.log 2>&1
  local rc=$?; echo "== $name rc=$rc"; [ $rc -ge 124 ] && exit $rc
  return 0
}
run trace --kernel-trace --stats
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_BRANCH
run sq2 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
