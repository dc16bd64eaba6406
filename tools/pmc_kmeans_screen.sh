#!/bin/bash
# Counter passes over the fp16 KMeans screen kernel alone (20M x 128, k=1024, blobs:
# no re-solve): MFMA busy vs SIMD cycles, VALU / LDS instruction counts, bank conflicts,
# wait vs active issue.  Each pass is its own short run within the per-block limits.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
O=gpurun_out/pmc_scr
mkdir -p $O
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS"
P3="SQ_WAIT_ANY SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE"
run() {   # name counters -- program args
  local name=$1 ctr=$2; shift 2
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$R/$O/$name" -o run -- "$@") \
    > "$R/$O/$name.log" 2>&1
}
A="$R/tools/prof_kmeans_assign.py --rows 20000000 --iters 2 --mode screen ${SCR_ARGS:-}"
run p1 "$P1" python3 $A && run p2 "$P2" python3 $A && run p3 "$P3" python3 $A
rc=$?
python3 tools/pmc_summary.py $O kmeans_screen > $O/summary.txt
exit $rc
