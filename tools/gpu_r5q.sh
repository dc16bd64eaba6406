#!/bin/bash
# Round 5: random-row gather rate (the floor of an exact ALS iteration).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_gather.py > gpurun_out/r5q_gather.json 2> gpurun_out/r5q_gather.err \
  || { echo "gather failed"; tail -20 gpurun_out/r5q_gather.err; exit 1; }
cat gpurun_out/r5q_gather.json
