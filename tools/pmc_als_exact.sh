#!/bin/bash
# Exact ALS kernels (rank 128, implicit): kernel-time stats, then PMC passes over the
# als_wood / als_dense kernels (kernel trace only, one counter group per run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
mkdir -p gpurun_out/pmc_als
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM"
P3="FETCH_SIZE"
P4="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
B="$R/tools/prof_als_exact.py --reps 1"
run() {
  local name=$1 ctr=$2
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$R/gpurun_out/pmc_als/$name" \
      -o run -- python3 $B) > "$R/gpurun_out/pmc_als/$name.log" 2>&1
}
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pmc_als/stats" \
    -o run -- python3 $B) > gpurun_out/pmc_als/stats.log 2>&1 \
&& run p1 "$P1" && run p2 "$P2" && run p3 "$P3" && run p4 "$P4"
rc=$?
python3 tools/pmc_summary.py gpurun_out/pmc_als als_wood > gpurun_out/pmc_als/summary_wood.txt
python3 tools/pmc_summary.py gpurun_out/pmc_als als_dense > gpurun_out/pmc_als/summary_dense.txt
exit $rc
