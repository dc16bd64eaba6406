#!/bin/bash
# Round 5: tree histogram kernel micro-benchmark (A/B of scheduling fences).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_hist.py > gpurun_out/r5ac_hist_${1:-x}.json 2> gpurun_out/r5ac_hist.err \
  || { echo "hist failed"; tail -20 gpurun_out/r5ac_hist.err; exit 1; }
cat gpurun_out/r5ac_hist_${1:-x}.json
