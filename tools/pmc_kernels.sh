#!/bin/bash
# Hardware-counter passes (rocprofv3 --pmc, kernel trace only) over the KMeans assign,
# GBT histogram / partition and ALS pass kernels.  Each pass is its own short run within
# the per-block counter limits (<= 8 SQ, <= 4 TCC, FETCH_SIZE = 3 TCC, <= 2 GRBM).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="FETCH_SIZE SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU"
run() {   # name pass-index counters -- program args
  local name=$1 idx=$2 ctr=$3; shift 3
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d "$R/gpurun_out/pmc/$name$idx" \
      -o run -- "$@") > "$R/gpurun_out/pmc/$name$idx.log" 2>&1
}
run kmeans 1 "$P1" python3 "$R/tools/prof_kmeans_assign.py" --rows 20000000 --iters 2 \
&& run kmeans 2 "$P2" python3 "$R/tools/prof_kmeans_assign.py" --rows 20000000 --iters 2 \
&& run gbt 1 "$P1" python3 "$R/tools/bench_gbt.py" --rows 8000000 --trees 1 \
&& run gbt 2 "$P2" python3 "$R/tools/bench_gbt.py" --rows 8000000 --trees 1 \
&& run als 1 "$P1" python3 "$R/tools/bench_als.py" --users 1000000 --items 100000 --ratings 20000000 --iters 1 \
&& run als 2 "$P2" python3 "$R/tools/bench_als.py" --users 1000000 --items 100000 --ratings 20000000 --iters 1
rc=$?
ls gpurun_out/pmc
exit $rc
