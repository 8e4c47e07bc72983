#!/bin/bash
# rocprofv3 passes over a short bench run (kernel trace + stats, then PMC passes
# in their own runs, as MI355X_MICROARCH.md prescribes). Output: gpurun_out/prof_*.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="${BENCH_ARGS:---steps 50 --warmup 5 --cpu-sample 0}"
run() {  # run <name> <timeout> <rocprof args...>
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" rocprofv3 "$@" -d gpurun_out/prof_$name -o $name --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 gpurun_out/prof_$name.log
  if [ $rc -ge 124 ]; then exit $rc; fi
}
run trace 300 --kernel-trace --stats
run pmc_sq 300 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY
[ -n "$QUICK" ] || run pmc_fetch 300 --pmc FETCH_SIZE
[ -n "$QUICK" ] || run pmc_write 300 --pmc WRITE_SIZE
run pmc_busy 300 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
run pmc_lds 300 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SMEM SQ_INST_CYCLES_SALU
