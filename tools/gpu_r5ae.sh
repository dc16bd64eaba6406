#!/bin/bash
# Round 5: PMC passes of the final exact ALS kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_als_exact.sh > gpurun_out/r5ae_pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/r5ae_pmc.log; exit 1; }
head -12 gpurun_out/pmc_als/summary_dense.txt
head -12 gpurun_out/pmc_als/summary_wood.txt
