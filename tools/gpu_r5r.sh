#!/bin/bash
# Round 5: dense exact-ALS kernel phase clocks (item-side rows, rank 128 implicit).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for other in ${OTHERS:-5000000}; do
timeout -k 10 300 python -u tools/als_dense_phases.py --other $other > gpurun_out/r5r_phases_$other.json 2> gpurun_out/r5r_phases.err \
  || { echo "phases failed"; tail -20 gpurun_out/r5r_phases.err; exit 1; }
cat gpurun_out/r5r_phases_$other.json
done
