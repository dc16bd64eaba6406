#!/bin/bash
# PMC passes over the KMeans screen kernel (tt 1 / 2) and the split kernel; kernel trace only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
mkdir -p gpurun_out/pmc_km
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS"
run() {
  local name=$1 ctr=$2; shift 2
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$R/gpurun_out/pmc_km/$name" \
      -o run -- "$@") > "$R/gpurun_out/pmc_km/$name.log" 2>&1
}
A="$R/tools/prof_kmeans_assign.py --rows 20000000 --iters 2"
timeout -k 10 120 python3 $A --mode screen --tt 2 > gpurun_out/pmc_km/t_s2.txt \
&& timeout -k 10 120 python3 $A --mode screen --tt 1 > gpurun_out/pmc_km/t_s1.txt \
&& timeout -k 10 120 python3 $A --mode split > gpurun_out/pmc_km/t_sp.txt \
&& run s2_p1 "$P1" python3 $A --mode screen --tt 2 \
&& run s2_p2 "$P2" python3 $A --mode screen --tt 2 \
&& run s1_p1 "$P1" python3 $A --mode screen --tt 1 \
&& run s1_p2 "$P2" python3 $A --mode screen --tt 1
rc=$?
cat gpurun_out/pmc_km/t_*.txt
exit $rc
