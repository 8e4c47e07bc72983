#!/bin/bash
# Round 4: pattern kernel after the leaf table. Occupancy A/B (KPE_PAT_MINW 3 default / 4 via a
# KPE_LIB variant build) on C5 / C3, then PMC passes on C5 (instruction mix, wait / busy
# cycles, L2 hits) in separate rocprofv3 runs.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r04_g}
O=gpurun_out/$TAG
mkdir -p $O
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-2} "$O/$name.log" | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for c in c5 c3; do
  step ${c}_w3 200 python bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0
  step ${c}_w4 200 env KPE_LIB=kyverno_amd/build/diag/libkpe_p4.so python bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0
done
B="--config c5 --steps 3 --warmup 1 --cpu-sample 0"
step pmc_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d $O/prof_pmc_sq -o pmc_sq --output-format csv -- python3 bench.py $B
step pmc_busy 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/prof_pmc_busy -o pmc_busy --output-format csv -- python3 bench.py $B
step pmc_tcc 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/prof_pmc_tcc -o pmc_tcc --output-format csv -- python3 bench.py $B
for f in $O/c*_w*.log; do grep '^{' $f > ${f%.log}.json || true; done
exit 0
