#!/bin/bash
# Round-3 profiles: C5 / C3 pattern kernel (kernel trace + PMC passes) and the C2 scan (LEAN A/B,
# kernel trace + PMC passes summarised into profiles/r03_c2 and perf/pmc_traffic_c2.json).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
prun() {  # prun <name> <config> <rocprof args...>
  local name=$1 cfg=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 240 rocprofv3 "$@" -d gpurun_out/prof_$name -o $name --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/prof_$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof_$name.log; exit $rc; fi
}
for c in c5 c3; do
  prun ${c}trace $c --kernel-trace --stats
  prun ${c}sq $c --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY
  prun ${c}busy $c --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
  prun ${c}tcc $c --pmc TCC_HIT_sum TCC_MISS_sum
  prun ${c}fetch $c --pmc FETCH_SIZE
done
mkdir -p gpurun_out/r03_pat
python3 scripts/pmc_summary.py gpurun_out r03_pat > gpurun_out/r03_pat/summary.log 2>&1
grep -E "kpe_pattern|kpe_scan" gpurun_out/r03_pat/summary.log | head -60
cp -r profiles/r03_pat/* gpurun_out/r03_pat/ 2>/dev/null
rm -rf gpurun_out/prof_c5* gpurun_out/prof_c3*
SKIP_AB= bash scripts/gpu_r03d.sh
