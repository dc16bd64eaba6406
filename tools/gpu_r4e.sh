#!/bin/bash
# Round-4 GPU batch E: ALS dense-kernel locality probe (gather table 1M vs 50M rows) + PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for other in 1000000 8000000 50000000; do
  timeout -k 10 240 python -u tools/prof_als_exact.py --users 100000 --items 625000 --other 1000000 --other-item $other --reps 2 \
    > gpurun_out/r4e_als_other_$other.log 2>&1 || { echo "prof_als $other failed"; tail -20 gpurun_out/r4e_als_other_$other.log; exit 1; }
  echo "other=$other $(grep '^item' gpurun_out/r4e_als_other_$other.log)"
done
timeout -k 10 600 bash tools/pmc_als_exact.sh || { echo "pmc als failed"; exit 1; }
cat gpurun_out/pmc_als/summary_dense.txt
